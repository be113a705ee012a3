"""Host-side weight layouts of the fp32-parity DenseNet kernels (CPU)."""
import torch

from triton_client_amd.ops import hip


def test_x3_w3_fragments_matches_kernel_indexing():
    """x3_conv3x3_v2_kernel loads wave (kq) lane (h, col) tap t half kc from
    offset (((t*4 + kq)*2 + kc)*64 + h*32 + col)*8: that must be
    w[col][t*128 + 32kq + 16kc + 8h .. +8] of the plain [32][9*128] layout."""
    w = torch.arange(32 * 9 * 128, dtype=torch.int64).reshape(32, 9 * 128)
    f = hip.x3_w3_fragments(w).reshape(-1)
    t, kq, kc, h, col, e = torch.meshgrid(*(torch.arange(n) for n in (9, 4, 2, 2, 32, 8)), indexing="ij")
    off = ((((t * 4 + kq) * 2 + kc) * 64 + h * 32 + col) * 8 + e).reshape(-1)
    src = w[col.reshape(-1), (t * 128 + 32 * kq + 16 * kc + 8 * h + e).reshape(-1)]
    assert torch.equal(f[off], src)
    assert sorted(f.tolist()) == list(range(w.numel()))  # a permutation


def test_x3_stem_fragments_matches_kernel_indexing():
    """x3_stem_weights loads half nh, k-step s, lane (hh, jj) from offset
    ((nh*14 + s)*64 + hh*32 + jj)*8: w[nh*32 + jj][16s + 8hh .. +8]."""
    w = torch.arange(64 * 224, dtype=torch.int64).reshape(64, 224)
    f = hip.x3_stem_fragments(w).reshape(-1)
    nh, s, hh, jj, e = torch.meshgrid(*(torch.arange(n) for n in (2, 14, 2, 32, 8)), indexing="ij")
    off = ((((nh * 14 + s) * 64) + hh * 32 + jj) * 8 + e).reshape(-1)
    assert torch.equal(f[off], w[(nh * 32 + jj).reshape(-1), (16 * s + 8 * hh + e).reshape(-1)])


def test_x3_w1_fragments_matches_kernel_indexing():
    """x3_dense_fused_kernel's 1x1 phase loads k16 step ks, wave quarter q1,
    lane (h, col) from offset ((ks*4 + q1)*64 + h*32 + col)*8: that must be
    w[32q1 + col][16ks + 8h .. +8] of the plain [128][K] layout."""
    K = 96
    w = torch.arange(128 * K, dtype=torch.int64).reshape(128, K)
    f = hip.x3_w1_fragments(w).reshape(-1)
    ks, q, h, col, e = torch.meshgrid(*(torch.arange(n) for n in (K // 16, 4, 2, 32, 8)), indexing="ij")
    off = ((((ks * 4 + q) * 64) + h * 32 + col) * 8 + e).reshape(-1)
    assert torch.equal(f[off], w[(32 * q + col).reshape(-1), (16 * ks + 8 * h + e).reshape(-1)])
    assert sorted(f.tolist()) == list(range(w.numel()))


def test_x3_w3f_fragments_matches_kernel_indexing():
    """The fused kernel's 3x3 phase (16x16x32 MFMA, wave = (kq, oh)) loads tap
    t, lane (h, col) from offset (((t*4 + kq)*2 + oh)*64 + h*16 + col)*8:
    w[16oh + col][t*128 + 32kq + 8h .. +8]."""
    w = torch.arange(32 * 9 * 128, dtype=torch.int64).reshape(32, 9 * 128)
    f = hip.x3_w3f_fragments(w).reshape(-1)
    t, kq, oh, h, col, e = torch.meshgrid(*(torch.arange(n) for n in (9, 4, 2, 4, 16, 8)), indexing="ij")
    off = ((((t * 4 + kq) * 2 + oh) * 64 + h * 16 + col) * 8 + e).reshape(-1)
    src = w[(16 * oh + col).reshape(-1), (t * 128 + 32 * kq + 8 * h + e).reshape(-1)]
    assert torch.equal(f[off], src)
    assert sorted(f.tolist()) == list(range(w.numel()))


def test_k14x_seven_tile_split_fits_the_stream_share():
    """DensenetFP32's K14x tiling rule (CPU, pure): the native choice's 7-tile
    split of small 14x14 batches stays only while its grid (images padded to
    8) fits one round of this stream's share of the CUs; other choices pass
    through."""
    from triton_client_amd.models.densenet_fp32 import stream_share_tiles

    assert stream_share_tiles(7, 32, 256, 1) == 7   # 224 workgroups <= 256
    assert stream_share_tiles(7, 33, 256, 1) == 4   # 280 > 256
    assert stream_share_tiles(7, 16, 256, 2) == 7   # 112 <= 128
    assert stream_share_tiles(7, 17, 256, 2) == 4   # 168 > 128
    assert stream_share_tiles(7, 1, 256, 3) == 7    # 56 <= 85
    assert stream_share_tiles(7, 16, 256, 3) == 4   # 112 > 85
    for t in (1, 2, 4):
        assert stream_share_tiles(t, 24, 256, 2) == t
