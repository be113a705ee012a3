"""Numerics of the fp32-parity DenseNet kernels (K8x/K9x/K10x, bf16x3 split
precision) against plain PyTorch fp32 / fp64 references of the same op.

The split-precision product is accurate to ~2^-16 relative per term, so the
tolerances here are fp32-class (1e-5 .. 1e-4), three orders of magnitude
tighter than the bf16 engine's tests (tests/test_densenet_kernels_gpu.py).
"""

import pytest

torch = pytest.importorskip("torch")
F = torch.nn.functional

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _hip():
    from triton_client_amd.ops import hip

    hip.lib()
    return hip


def _rel(got, ref):
    got, ref = got.double(), ref.double()
    assert torch.isfinite(got).all()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _split(t):
    hi = t.to(torch.bfloat16)
    lo = (t - hi.float()).to(torch.bfloat16)
    return hi.contiguous(), lo.contiguous()


def _st():
    return torch.cuda.current_stream().cuda_stream


def test_split_is_exact_to_2e17():
    _need_gpu()
    hip = _hip()
    w = torch.randn(100003, device=DEV) * 3
    hi = torch.empty(w.numel(), device=DEV, dtype=torch.bfloat16)
    lo = torch.empty_like(hi)
    hip.x3_split(w.data_ptr(), hi.data_ptr(), lo.data_ptr(), w.numel(), stream=_st())
    torch.cuda.synchronize()
    rh, rl = _split(w)
    assert torch.equal(hi, rh) and torch.equal(lo, rl)
    err = ((hi.double() + lo.double()) - w.double()).abs() / w.double().abs().clamp_min(1e-30)
    assert err.max().item() <= 2.0 ** -17


@pytest.mark.parametrize("M,K,ldx", [(100, 64, 96), (37, 992, 1024), (6272, 512, 1024), (50000, 224, 256),
                                     (401408, 96, 256), (25088, 640, 1024), (1568, 768, 1024), (392, 992, 1024),
                                     (65555, 32, 32), (100352, 480, 512), (70001, 1024, 1024)])
def test_x3_conv1x1_split_out(M, K, ldx):
    """Dense-layer 1x1: z = relu(relu(x*s+t) @ W^T + b) as hi/lo planes
    (M >= 16384: the warp-specialised persistent kernel, incl. ragged block
    ranges and a single K step; mid M: whole-K tiles; small M: split-K
    workspace + reduce)."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(M + K)
    x = torch.randn(M, ldx, device=DEV, generator=g)
    s = torch.rand(K, device=DEV, generator=g) + 0.5
    t = torch.randn(K, device=DEV, generator=g) * 0.2
    w = torch.randn(128, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(128, device=DEV, generator=g) * 0.1
    wh, wl = _split(w)
    zh = torch.empty(M, 128, device=DEV, dtype=torch.bfloat16)
    zl = torch.empty_like(zh)
    wsb = hip.x3_conv1x1_ws_bytes(M, K)
    ws = torch.empty(max(wsb, 16), device=DEV, dtype=torch.uint8)
    hip.x3_conv1x1(x.data_ptr(), ldx, M, K, s.data_ptr(), t.data_ptr(), wh.data_ptr(), wl.data_ptr(),
                   out_bias=b.data_ptr(), z_hi=zh.data_ptr(), z_lo=zl.data_ptr(), ws=ws.data_ptr(), ws_bytes=wsb,
                   stream=_st())
    torch.cuda.synchronize()
    a = torch.relu(x[:, :K].double() * s.double() + t.double())
    ref = torch.relu(a @ w.double().t() + b.double())
    got = zh.double() + zl.double()
    assert _rel(got, ref) < 3e-5


@pytest.mark.parametrize("imgs,H,C,ldy", [(2, 56, 256, 128), (1, 14, 1024, 640), (16, 28, 512, 384),
                                          (128, 8, 1024, 1024), (64, 56, 256, 160)])
def test_x3_conv1x1_transition_pool(imgs, H, C, ldy):
    """Transition: y = avgpool2x2(relu(x*s+t)) @ W^T, fp32 into the next block buffer."""
    _need_gpu()
    if H % 2:
        H += 1
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * H + C)
    x = torch.randn(imgs * H * H, C, device=DEV, generator=g)
    s = torch.rand(C, device=DEV, generator=g) + 0.5
    t = torch.randn(C, device=DEV, generator=g) * 0.2
    N = C // 2
    w = torch.randn(N, C, device=DEV, generator=g) / C ** 0.5
    wh, wl = _split(w)
    Mo = imgs * (H // 2) * (H // 2)
    y = torch.full((Mo, ldy), 7.0, device=DEV)
    wsb = hip.x3_conv1x1_ws_bytes(Mo, C, N)
    ws = torch.empty(max(wsb, 16), device=DEV, dtype=torch.uint8)
    hip.x3_conv1x1(x.data_ptr(), C, Mo, C, s.data_ptr(), t.data_ptr(), wh.data_ptr(), wl.data_ptr(),
                   y=y.data_ptr(), ldy=ldy, pool=1, H=H, W=H, ws=ws.data_ptr(), ws_bytes=wsb, stream=_st(), N=N)
    torch.cuda.synchronize()
    a = torch.relu(x.double() * s.double() + t.double()).reshape(imgs, H, H, C).permute(0, 3, 1, 2)
    a = F.avg_pool2d(a, 2).permute(0, 2, 3, 1).reshape(Mo, C)
    ref = a @ w.double().t()
    assert _rel(y[:, :N], ref) < 3e-5
    assert (y[:, N:] == 7.0).all(), "wrote outside the N-channel slice"


@pytest.mark.parametrize("imgs,H", [(1, 7), (3, 14), (2, 56), (48, 28), (24, 56), (1, 28)])
def test_x3_conv3x3(imgs, H):
    """3x3 128->32 pad 1 on split planes into an fp32 channel slice (the
    multi-tile cases exercise the sliding LDS ring across tile runs)."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * 100 + H)
    M = imgs * H * H
    z = torch.relu(torch.randn(M, 128, device=DEV, generator=g))
    w = torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5
    zh, zl = _split(z)
    wh, wl = (hip.x3_w3_fragments(t) for t in _split(w.permute(0, 2, 3, 1).reshape(32, -1)))
    ldy, off = 96, 32
    y = torch.full((M, ldy), 7.0, device=DEV)
    hip.x3_conv3x3(zh.data_ptr(), zl.data_ptr(), imgs, H, H, wh.data_ptr(), wl.data_ptr(), y.data_ptr() + 4 * off,
                   ldy, stream=_st())
    torch.cuda.synchronize()
    zin = (zh.double() + zl.double()).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
    ref = F.conv2d(zin, w.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 32)
    assert _rel(y[:, off:off + 32], ref) < 2e-5
    assert (y[:, :off] == 7.0).all() and (y[:, off + 32:] == 7.0).all()


@pytest.mark.parametrize("imgs,H,K", [(1, 56, 224), (1, 28, 480), (8, 14, 992), (1, 7, 992), (8, 7, 512),
                                      (2, 56, 64), (128, 14, 256), (20, 28, 128)])
def test_x3_dense_layer(imgs, H, K):
    """1x1 -> 3x3 dense layer through one entry point: small M plans split-K and
    the 3x3 sums the partials (+bias, ReLU, split) while staging its band (no
    reduce launch); big M runs the plain z round trip.  Against fp64 torch."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * 1000 + H + K)
    M, ldx = imgs * H * H, K + 64
    x = torch.randn(M, ldx, device=DEV, generator=g)
    s = torch.rand(K, device=DEV, generator=g) + 0.5
    t = torch.randn(K, device=DEV, generator=g) * 0.2
    w1 = torch.randn(128, K, device=DEV, generator=g) / K ** 0.5
    b1 = torch.randn(128, device=DEV, generator=g) * 0.1
    w2 = torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5
    w1h, w1l = _split(w1)
    w2h, w2l = (hip.x3_w3_fragments(u) for u in _split(w2.permute(0, 2, 3, 1).reshape(32, -1)))
    zh = torch.empty(M, 128, device=DEV, dtype=torch.bfloat16)
    zl = torch.empty_like(zh)
    wsb = hip.x3_conv1x1_ws_bytes(M, K)
    ws = torch.empty(max(wsb, 16), device=DEV, dtype=torch.uint8)
    xc = x.clone()
    hip.x3_dense_layer(x.data_ptr(), ldx, imgs, H, H, K, s.data_ptr(), t.data_ptr(), w1h.data_ptr(), w1l.data_ptr(),
                       b1.data_ptr(), zh.data_ptr(), zl.data_ptr(), w2h.data_ptr(), w2l.data_ptr(),
                       x.data_ptr() + 4 * K, ldx, ws=ws.data_ptr(), ws_bytes=wsb, stream=_st())
    torch.cuda.synchronize()
    a = torch.relu(xc[:, :K].double() * s.double() + t.double())
    z = torch.relu(a @ w1.double().t() + b1.double()).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
    ref = F.conv2d(z, w2.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 32)
    assert _rel(x[:, K:K + 32], ref) < 3e-5
    assert torch.equal(x[:, :K], xc[:, :K]) and torch.equal(x[:, K + 32:], xc[:, K + 32:])


@pytest.mark.parametrize("imgs,H,K", [(1, 14, 992), (1, 7, 992), (8, 14, 512), (8, 7, 1024), (1, 28, 480),
                                      (2, 14, 256), (3, 9, 48), (1, 1, 128), (7, 5, 640)])
def test_x3s_dense_layer(imgs, H, K):
    """K13x small-M dense layer: the 1x1 adds into a zeroed fp32 accumulator
    with float atomics over many workgroups, the 3x3 reads it (bias + ReLU +
    split in registers) and zeroes the next layer's accumulator.  Against fp64
    torch; run to run within float-atomic ordering noise (the 3x3 quarters add into y)."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * 31 + H * 7 + K)
    M, ldx = imgs * H * H, K + 64
    x = torch.randn(M, ldx, device=DEV, generator=g)
    s = torch.rand(K, device=DEV, generator=g) + 0.5
    t = torch.randn(K, device=DEV, generator=g) * 0.2
    w1 = torch.randn(128, K, device=DEV, generator=g) / K ** 0.5
    b1 = torch.randn(128, device=DEV, generator=g) * 0.1
    w2 = torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5
    f1h, f1l = (hip.x3_w1_fragments(u) for u in _split(w1))
    f2h, f2l = (hip.x3_w3_fragments(u) for u in _split(w2.permute(0, 2, 3, 1).reshape(32, -1)))
    xc = x.clone()
    outs = []
    for _ in range(2):
        x.copy_(xc)
        zacc = torch.zeros(M + 5, 128, device=DEV)
        znext = torch.full((M + 5, 128), 3.0, device=DEV)
        hip.x3s_dense_layer(x.data_ptr(), ldx, imgs, H, H, K, s.data_ptr(), t.data_ptr(), f1h.data_ptr(),
                            f1l.data_ptr(), b1.data_ptr(), zacc.data_ptr(), znext.data_ptr(), f2h.data_ptr(),
                            f2l.data_ptr(), x.data_ptr() + 4 * K, ldx, stream=_st())
        torch.cuda.synchronize()
        assert (znext[:M] == 0).all() and (znext[M:] == 3.0).all()
        outs.append(x[:, K:K + 32].clone())
    a = torch.relu(xc[:, :K].double() * s.double() + t.double())
    zraw = a @ w1.double().t()
    assert _rel(zacc[:M], zraw) < 3e-5 and (zacc[M:] == 0).all()
    z = torch.relu(zraw + b1.double()).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
    ref = F.conv2d(z, w2.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 32)
    assert _rel(x[:, K:K + 32], ref) < 3e-5
    assert _rel(outs[0], outs[1]) < 2e-6
    assert torch.equal(x[:, :K], xc[:, :K]) and torch.equal(x[:, K + 32:], xc[:, K + 32:])


@pytest.mark.parametrize("imgs,H,C0,n", [(1, 14, 256, 6), (8, 14, 256, 3), (1, 7, 512, 5), (32, 7, 512, 2),
                                         (1, 28, 256, 4), (2, 28, 256, 1), (3, 9, 64, 4), (1, 31, 96, 3),
                                         (1, 56, 64, 6), (1, 63, 64, 2), (2, 40, 128, 3)])
def test_x3c_chain(imgs, H, C0, n):
    """K13x chain: a run of n dense layers as one base launch (every layer's
    1x1 over the first C0 channels) plus one launch per layer (its 3x3, the
    previous layer's 1x1 chunk for the tile + halo, and that chunk fanned out
    to every later layer).  The whole block buffer against fp64 torch layer
    by layer."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * 131 + H * 17 + C0 + n)
    M, ctot = imgs * H * H, C0 + 32 * n + 32  # 32 spare channels past the run
    x = torch.randn(M, ctot, device=DEV, generator=g)
    x[:, C0:] = 5.0  # the y slices must be zeroed by the base launch
    x[:, C0 + 32 * n:] = 7.0
    xc = x.clone()
    zc = torch.full((n, M + 3, 128), 9.0, device=DEV)
    keep, ent = [], []
    for j in range(n):
        K = C0 + 32 * j
        s = torch.rand(K, device=DEV, generator=g) + 0.5
        t = torch.randn(K, device=DEV, generator=g) * 0.2
        w1 = torch.randn(128, K, device=DEV, generator=g) / K ** 0.5
        b1 = torch.randn(128, device=DEV, generator=g) * 0.1
        w2 = torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5
        f1h, f1l = (hip.x3_w1_fragments(u) for u in _split(w1))
        f2h, f2l = (hip.x3_w3_fragments(u) for u in _split(w2.permute(0, 2, 3, 1).reshape(32, -1)))
        keep.append((s, t, w1, b1, w2, f1h, f1l, f2h, f2l))
        ent.append(hip.x3c_layer_entry(f1h.data_ptr(), f1l.data_ptr(), s.data_ptr(), t.data_ptr(), b1.data_ptr(),
                                       f2h.data_ptr(), f2l.data_ptr(), zc[j].data_ptr(), K))
    table = torch.tensor(ent, dtype=torch.int64, device=DEV)
    hip.x3c_base(table.data_ptr(), n, x.data_ptr(), ctot, imgs, H, H, stream=_st())
    for j in range(n):
        hip.x3c_layer(table.data_ptr(), j, n, x.data_ptr(), ctot, imgs, H, H, stream=_st())
    torch.cuda.synchronize()
    ref = xc.double()
    for j, (s, t, w1, b1, w2, *_) in enumerate(keep):
        K = C0 + 32 * j
        a = torch.relu(ref[:, :K] * s.double() + t.double())
        z = torch.relu(a @ w1.double().t() + b1.double()).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
        ref[:, K:K + 32] = F.conv2d(z, w2.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 32)
    for j in range(n):
        K = C0 + 32 * j
        assert _rel(x[:, K:K + 32], ref[:, K:K + 32]) < 5e-5, "layer %d" % j
    assert torch.equal(x[:, :C0], xc[:, :C0]) and (x[:, C0 + 32 * n:] == 7.0).all()


@pytest.mark.parametrize("imgs,H,K", [(1, 56, 64), (8, 56, 224), (32, 56, 128), (64, 28, 224), (5, 28, 96),
                                      (3, 28, 192), (2, 16, 160), (128, 28, 128), (40, 56, 192), (16, 28, 480),
                                      (3, 28, 320), (24, 28, 256), (2, 20, 416)])
@pytest.mark.parametrize("version", [1, 3, 5])
def test_x3_dense_fused(imgs, H, K, version):
    """K11x (v1; v3: v1 with the next chunk's 1x1 interleaved into the 3x3;
    5 = K11w, v1 on producer / consumer waves, bitwise v1's output): the whole dense layer in one kernel (z produced into the 3x3's LDS
    ring, never written to HBM): one block's band prologue only, several tiles
    per block, ragged tails, every block width, and every K-step instantiation
    (K = 64..480, 2..15 steps).  Against fp64
    torch, and against the two-kernel path (same split products)."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * 7919 + H + K)
    M, ldx = imgs * H * H, K + 64
    x = torch.randn(M, ldx, device=DEV, generator=g)
    s = torch.rand(K, device=DEV, generator=g) + 0.5
    t = torch.randn(K, device=DEV, generator=g) * 0.2
    w1 = torch.randn(128, K, device=DEV, generator=g) / K ** 0.5
    b1 = torch.randn(128, device=DEV, generator=g) * 0.1
    w2 = torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5
    w1h, w1l = _split(w1)
    w2p = _split(w2.permute(0, 2, 3, 1).reshape(32, -1))
    f1h, f1l = (hip.x3_w1_fragments(u) for u in (w1h, w1l))
    frag = hip.x3_w3f_fragments
    fused = {1: hip.x3_dense_fused, 3: hip.x3_dense_fused3, 5: hip.x3_dense_fused_ws}[version]
    f2h, f2l = (frag(u) for u in w2p)
    xc = x.clone()
    fused(x.data_ptr(), ldx, imgs, H, H, K, s.data_ptr(), t.data_ptr(), f1h.data_ptr(), f1l.data_ptr(),
          b1.data_ptr(), f2h.data_ptr(), f2l.data_ptr(), x.data_ptr() + 4 * K, ldx, stream=_st())
    torch.cuda.synchronize()
    a = torch.relu(xc[:, :K].double() * s.double() + t.double())
    z = torch.relu(a @ w1.double().t() + b1.double()).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
    ref = F.conv2d(z, w2.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 32)
    assert _rel(x[:, K:K + 32], ref) < 3e-5
    assert torch.equal(x[:, :K], xc[:, :K]) and torch.equal(x[:, K + 32:], xc[:, K + 32:])
    # the two-kernel path on the same inputs
    y2 = xc.clone()
    w2h, w2l = (hip.x3_w3_fragments(u) for u in w2p)
    zh = torch.empty(M, 128, device=DEV, dtype=torch.bfloat16)
    zl = torch.empty_like(zh)
    hip.x3_dense_layer(y2.data_ptr(), ldx, imgs, H, H, K, s.data_ptr(), t.data_ptr(), w1h.data_ptr(),
                       w1l.data_ptr(), b1.data_ptr(), zh.data_ptr(), zl.data_ptr(), w2h.data_ptr(), w2l.data_ptr(),
                       y2.data_ptr() + 4 * K, ldx, stream=_st())
    torch.cuda.synchronize()
    assert _rel(x[:, K:K + 32], y2[:, K:K + 32]) < 2e-5
    if version == 5:  # same products in the same order as v1
        y1 = xc.clone()
        hip.x3_dense_fused(y1.data_ptr(), ldx, imgs, H, H, K, s.data_ptr(), t.data_ptr(), f1h.data_ptr(),
                           f1l.data_ptr(), b1.data_ptr(), f2h.data_ptr(), f2l.data_ptr(), y1.data_ptr() + 4 * K, ldx,
                           stream=_st())
        torch.cuda.synchronize()
        assert torch.equal(x, y1)


@pytest.mark.parametrize("imgs,H,K", [(1, 14, 64), (3, 14, 256), (8, 14, 288), (9, 14, 992), (17, 14, 640),
                                      (128, 14, 512), (16, 14, 96), (1, 7, 512), (5, 7, 992), (64, 7, 768),
                                      (130, 7, 544), (2, 7, 64), (40, 14, 416), (37, 14, 736), (64, 14, 1024),
                                      (37, 7, 320), (8, 7, 1024)])
@pytest.mark.parametrize("tiles", [1, 2, 4, 7])
def test_x3_dense_small(imgs, H, K, tiles):
    """K14x: the whole dense layer of a 14x14 or 7x7 block in one kernel over
    row tiles of the images (tiles per image: 14x14 2, 4 or 7, 7x7 1, 2, 4 or 7;
    every tile recomputes the 1x1 of its halo rows), z in a zero-padded LDS
    image of the tile.  Ragged image counts (not multiples of 8: the grid
    groups the tiles of images 8g+j), uneven tiles (14 rows in 4 tiles, 7 in 2
    or 4), K from 64 to 992 (2..31 K steps) and a layer slice in the middle of
    a wider block buffer.  Against fp64 torch (< 3e-5, and per image), and
    against the two-kernel path on the same split products."""
    _need_gpu()
    if H == 14 and tiles == 1:
        pytest.skip("14x14 takes 2 or 4 tiles per image")
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * 131 + H * 7 + K)
    M, ldx = imgs * H * H, K + 96
    x = torch.randn(M, ldx, device=DEV, generator=g)
    s = torch.rand(K, device=DEV, generator=g) + 0.5
    t = torch.randn(K, device=DEV, generator=g) * 0.2
    w1 = torch.randn(128, K, device=DEV, generator=g) / K ** 0.5
    b1 = torch.randn(128, device=DEV, generator=g) * 0.1
    w2 = torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5
    w1h, w1l = _split(w1)
    w2p = _split(w2.permute(0, 2, 3, 1).reshape(32, -1))
    f2h, f2l = (hip.x3_w3f_fragments(u) for u in w2p)
    f1h, f1l = (hip.x3_w1_fragments(u) for u in (w1h, w1l))
    xc = x.clone()
    hip.x3_dense_small(x.data_ptr(), ldx, imgs, H, H, K, s.data_ptr(), t.data_ptr(), f1h.data_ptr(), f1l.data_ptr(),
                       b1.data_ptr(), f2h.data_ptr(), f2l.data_ptr(), x.data_ptr() + 4 * K, ldx, stream=_st(),
                       tiles=tiles)
    torch.cuda.synchronize()
    a = torch.relu(xc[:, :K].double() * s.double() + t.double())
    z = torch.relu(a @ w1.double().t() + b1.double()).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
    ref = F.conv2d(z, w2.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 32)
    err = _rel(x[:, K:K + 32], ref)
    # per image too: a tile written to the wrong image / rows shows even when the total is close
    per_img = ((x[:, K:K + 32].double() - ref).reshape(imgs, -1).norm(dim=1) / ref.reshape(imgs, -1).norm(dim=1))
    print("K14x imgs %d H %d K %d tiles %d: rel %.3g, worst image %.3g" % (imgs, H, K, tiles, err,
                                                                         per_img.max().item()))
    assert err < 3e-5 and per_img.max().item() < 1e-4
    assert torch.equal(x[:, :K], xc[:, :K]) and torch.equal(x[:, K + 32:], xc[:, K + 32:])
    y2 = xc.clone()
    w2h, w2l = (hip.x3_w3_fragments(u) for u in w2p)
    zh = torch.empty(M, 128, device=DEV, dtype=torch.bfloat16)
    zl = torch.empty_like(zh)
    hip.x3_dense_layer(y2.data_ptr(), ldx, imgs, H, H, K, s.data_ptr(), t.data_ptr(), w1h.data_ptr(),
                       w1l.data_ptr(), b1.data_ptr(), zh.data_ptr(), zl.data_ptr(), w2h.data_ptr(), w2l.data_ptr(),
                       y2.data_ptr() + 4 * K, ldx, stream=_st())
    torch.cuda.synchronize()
    assert _rel(x[:, K:K + 32], y2[:, K:K + 32]) < 2e-5


def test_x3_small_tiles_fill_the_chip():
    """The default tiling: the fewest tiles per image that give every CU a
    workgroup; 14x14 images too few for that with quarters take 7 two-row
    tiles while those still fit one round of the CUs."""
    _need_gpu()
    hip = _hip()
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    for imgs in (1, 8, 24, 32, 40, 64, 128, 256):
        for W, opts in ((14, (2, 4)), (7, (1, 2, 4))):
            t = hip.x3_small_tiles(imgs, W)
            padded = (imgs + 7) // 8 * 8
            fill = [o for o in opts if padded * o >= ncu]
            if fill:
                want = fill[0]
            elif W == 14 and padded * 7 <= ncu:
                want = 7
            else:
                want = opts[-1]
            assert t == want, (imgs, W, t)


def test_x3_dense_small_rejects_bad_shapes():
    _need_gpu()
    hip = _hip()
    x = torch.zeros(2 * 196, 320, device=DEV)
    w = torch.zeros(128 * 256, device=DEV)
    for H, W, K, tiles in [(28, 28, 256, 0), (14, 7, 256, 0), (14, 14, 250, 0), (14, 14, 32, 0), (14, 14, 256, 1),
                           (7, 7, 256, 3), (14, 14, 256, 8), (7, 7, 2080, 0)]:
        with pytest.raises(Exception):
            hip.x3_dense_small(x.data_ptr(), 320, 2, H, W, K, w.data_ptr(), w.data_ptr(), w.data_ptr(), w.data_ptr(),
                               w.data_ptr(), w.data_ptr(), w.data_ptr(), x.data_ptr() + 4 * K, 320, stream=_st(),
                               tiles=tiles)


@pytest.mark.parametrize("imgs", [3, 20])  # 20: more tiles than the persistent grid (several per block)
def test_x3_stem(imgs):
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(imgs, 3, 224, 224, device=DEV, generator=g)
    w = torch.randn(64, 3, 7, 7, device=DEV, generator=g) / 12
    bias = torch.randn(64, device=DEV, generator=g) * 0.1
    wp = torch.zeros(64, 7, 8, 4, device=DEV)
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    wh, wl = (hip.x3_stem_fragments(t) for t in _split(wp.reshape(64, -1)))
    ptrs = torch.tensor([x[i].data_ptr() for i in range(imgs)], device=DEV, dtype=torch.int64)
    ldy = 96
    y = torch.full((imgs * 56 * 56, ldy), 7.0, device=DEV)
    hip.x3_stem(ptrs.data_ptr(), wh.data_ptr(), wl.data_ptr(), bias.data_ptr(), y.data_ptr(), imgs, ldy, stream=_st())
    torch.cuda.synchronize()
    c = F.conv2d(x.double(), w.double(), stride=2, padding=3)
    ref = torch.relu(F.max_pool2d(c, 3, 2, 1) + bias.double().view(1, -1, 1, 1))
    ref = ref.permute(0, 2, 3, 1).reshape(-1, 64)
    assert _rel(y[:, :64], ref) < 2e-5
    assert (y[:, 64:] == 7.0).all()


@pytest.mark.parametrize("imgs,HW,C", [(5, 49, 1024), (1, 49, 1024), (3, 7, 1000), (2, 1, 64), (4, 50, 512)])
def test_x3_head_pool(imgs, HW, C):
    _need_gpu()
    hip = _hip()
    x = torch.randn(imgs * HW, C, device=DEV)
    s = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV)
    out = torch.full((imgs + 1, C), 7.0, device=DEV)
    hip.x3_head_pool(x.data_ptr(), s.data_ptr(), b.data_ptr(), out.data_ptr(), imgs, HW, C, stream=_st())
    torch.cuda.synchronize()
    ref = torch.relu(x.double() * s.double() + b.double()).reshape(imgs, HW, C).mean(1)
    assert _rel(out[:imgs], ref) < 1e-6
    assert (out[imgs:] == 7.0).all()


@pytest.fixture(scope="module")
def fp32_engine():
    _need_gpu()
    from triton_client_amd.models import densenet_fp32

    eng, model = densenet_fp32.build(max_batch=32, device=DEV)
    return eng, model


@pytest.mark.parametrize("b", [1, 8, 19])
def test_fp32_engine_matches_fp32_module(fp32_engine, b):
    """The headline engine: rel-L2 of the logits vs the fp32 torch module
    (same folded weights) must be fp32-class, < 1e-3 (measured ~1e-5)."""
    eng, model = fp32_engine
    g = torch.Generator(device=DEV).manual_seed(100 + b)
    x = torch.randn(b, 3, 224, 224, device=DEV, generator=g)
    with torch.no_grad():
        got = eng(x)
        ref = model.to(DEV).float()(x)
    torch.cuda.synchronize()
    err = _rel(got, ref)
    print("fp32 engine b=%d rel-L2 vs fp32 module: %.3g" % (b, err))
    assert err < 1e-3


@pytest.mark.parametrize("b", [1, 3, 8, 9, 24, 32])  # (37 / 64 images: test_x3_dense_small, per layer)
def test_fp32_engine_k14x_blocks_match_fp32_module(fp32_engine, b):
    """The engine with K14x forced on for the 14x14 and 7x7 blocks at every
    batch (ragged image counts: the grid groups the tiles of images 8g+j; up
    to 32 images the 14x14 layers take 7 tiles per image, then 4), against
    the fp32 module, and against the same engine with K14x off."""
    eng, model = fp32_engine
    g = torch.Generator(device=DEV).manual_seed(300 + b)
    x = torch.randn(b, 3, 224, 224, device=DEV, generator=g)
    keep = eng.smallf_min_blocks
    try:
        eng.smallf_min_blocks = 1
        with torch.no_grad():
            got = eng(x).clone()
        eng.smallf_min_blocks = 0
        with torch.no_grad():
            base = eng(x).clone()
            ref = model.to(DEV).float()(x)
    finally:
        eng.smallf_min_blocks = keep
    torch.cuda.synchronize()
    e_ref, e_base = _rel(got, ref), _rel(got, base)
    print("K14x engine b=%d: rel vs fp32 module %.3g, vs the pair path %.3g" % (b, e_ref, e_base))
    assert e_ref < 1e-3 and e_base < 1e-4


def test_k14x_routing_follows_stream_concurrency(fp32_engine):
    """TCAMD_X3_SMALLF_MIN_BLOCKS unset: K14x takes the 14x14 / 7x7 blocks from
    48 workgroups (images x row tiles, counted at up to 4 tiles per image)
    when the engine is one of several concurrent streams, from 64 on one
    stream (profiles/r5_engine_ab.md, r5_k14x_tiles.md)."""
    eng, _ = fp32_engine
    keep = eng.smallf_min_blocks, eng.concurrent_streams
    try:
        eng.smallf_min_blocks = None
        eng.concurrent_streams = 1
        assert [b for b in range(1, 33) if eng._small_fused(b, 14)] == list(range(16, 33))
        eng.concurrent_streams = 2
        assert [b for b in range(1, 33) if eng._small_fused(b, 14)] == list(range(12, 33))
        assert [b for b in range(1, 33) if eng._small_fused(b, 7)] == list(range(12, 33))
        assert not eng._small_fused(64, 28)
    finally:
        eng.smallf_min_blocks, eng.concurrent_streams = keep


def test_k14x_seven_tiles_fit_the_stream_share(fp32_engine):
    """Small 14x14 batches take 7 two-row tiles per image when those fit one
    round of the engine's share of the CUs (all of them on one stream, half
    on two), else quarters; 7x7 never takes 7; TCAMD_X3_SMALLF_TILES wins."""
    eng, _ = fp32_engine
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    keep = eng.smallf_tiles, eng.concurrent_streams
    try:
        eng.smallf_tiles = 0
        for streams in (1, 2):
            eng.concurrent_streams = streams
            for b in (8, 16, 24, 32, 40):
                padded = (b + 7) // 8 * 8
                want = 7 if padded * 4 < ncu and padded * 7 <= ncu // streams else \
                    (2 if padded * 2 >= ncu else 4)
                assert eng._small_tiles(b, 14) == want, (streams, b)
                assert eng._small_tiles(b, 7) != 7
        eng.smallf_tiles = 2
        assert eng._small_tiles(16, 14) == 2
    finally:
        eng.smallf_tiles, eng.concurrent_streams = keep


_ROUTES = [{"fuse_min_tiles": 0}, {"fuse_big_k_min_tiles": 4}, {"fuse_v3": 0}, {"fuse_v3": 16},
           {"small_m": 0}, {"use_chain": False}, {"chain_m": 0}, {"small_m": 0, "chain_m": 0},
           {"smallf_min_blocks": 1, "smallf_tiles": 2}, {"smallf_min_blocks": 1, "smallf_tiles": 4}]


@pytest.mark.parametrize("b", [2, 24])
def test_fp32_engine_routing_knobs(fp32_engine, b):
    """Every engine routing knob (the TCAMD_X3_* engine attributes: K11x on /
    off, its big-K floor, v3 placement, K13x two-launch and chain, chain size,
    K14x tiling) gives the default route's logits to fp32 parity, and the
    fp32 module's within the engine bound."""
    eng, model = fp32_engine
    g = torch.Generator(device=DEV).manual_seed(500 + b)
    x = torch.randn(b, 3, 224, 224, device=DEV, generator=g)
    with torch.no_grad():
        base = eng(x).clone()
        ref = model.to(DEV).float()(x)
    for route in _ROUTES:
        keep = {k: getattr(eng, k) for k in route}
        try:
            for k, v in route.items():
                setattr(eng, k, v)
            with torch.no_grad():
                got = eng(x).clone()
        finally:
            for k, v in keep.items():
                setattr(eng, k, v)
        torch.cuda.synchronize()
        e_base, e_ref = _rel(got, base), _rel(got, ref)
        print("engine b=%d %s: rel vs default route %.3g, vs fp32 module %.3g" % (b, route, e_base, e_ref))
        assert e_base < 1e-4 and e_ref < 1e-3, route


def test_fp32_engine_vs_fp64_and_graph_capture(fp32_engine):
    """Against an fp64 CPU reference the engine must stay fp32-class (rel-L2
    < 1e-4; measured 4.5e-5, torch's own fp32 forward 2.2e-6 on MI355X, the
    bf16 engine 3e-2); and a captured HIP graph replays the same logits (to
    float-atomic ordering noise: the small-M layers sum with atomics)."""
    eng, model = fp32_engine
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(2, 3, 224, 224, device=DEV, generator=g)
    with torch.no_grad():
        got = eng(x).clone()
        ref32 = model.to(DEV).float()(x)
        ref64 = model.to("cpu").double()(x.cpu().double())
        model.float()
    e_eng, e_torch = _rel(got.cpu(), ref64), _rel(ref32.cpu(), ref64)
    print("vs fp64: engine %.3g, torch fp32 %.3g" % (e_eng, e_torch))
    assert e_eng < 1e-4
    s = torch.cuda.Stream()
    out = torch.zeros(32, 1000, device=DEV)
    eng.ptrs[:2] = eng._img_off[:2] + x.data_ptr()
    with torch.cuda.stream(s), torch.no_grad():
        eng.forward_ptrs(2, out=out)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            eng.forward_ptrs(2, out=out)
        out.zero_()
        gr.replay()
    s.synchronize()
    assert _rel(out[:2], got) < 2e-5  # measured run to run: 6e-6 (tools/engine_repeat.py)


def test_fp32_engine_workspace_covers_every_batch(fp32_engine):
    """The split-K workspace is sized for every batch up to the capacity: a
    serving engine (capacity 32 here, 256 in the server) must still split
    (and reduce inside the 3x3) at bs1, where the partials are largest."""
    from triton_client_amd.ops import hip

    eng, _ = fp32_engine
    for bi, layers in enumerate(eng.blocks):
        hw = eng.block_dims[bi][0]
        for L in layers:
            for b in (1, 2, 8, eng.max_batch):
                assert eng.ws.numel() >= hip.x3_conv1x1_ws_bytes(b * hw * hw, L["cin"])
