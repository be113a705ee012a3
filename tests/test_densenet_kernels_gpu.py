"""Numerics of the fused DenseNet kernels (K8-K10) against plain PyTorch fp32.

Each HIP kernel is compared with an fp32 reference of the same op; the
reference rounds exactly where the kernel rounds (bf16 activations between
the prologue and the MFMA), so tolerances only cover accumulation order.
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


def _close(got, ref, tol=2e-2):
    got = got.float()
    ref = ref.float()
    err = (got - ref).norm() / ref.norm().clamp_min(1e-6)
    assert err.item() < tol, "rel-L2 %.4g" % err.item()
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("M,K,ldx,N,off", [(100, 64, 96, 128, 32), (40000, 224, 256, 128, 0),
                                           (70000, 96, 128, 128, 0), (3000, 512, 512, 256, 0)])
@pytest.mark.parametrize("variant", [0, 11, 21, 41, 211, 212, 221, 222])
def test_conv1x1_prologue_epilogue(M, K, ldx, N, off, variant):
    _need_gpu()
    if variant == 300 and K > 256:
        pytest.skip("K8w covers K <= 256")
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(M + K)
    x = torch.randn(M, ldx, device=DEV, generator=g).bfloat16()
    s = torch.rand(K, device=DEV, generator=g) + 0.5
    b = torch.randn(K, device=DEV, generator=g) * 0.2
    w = (torch.randn(N, K, device=DEV, generator=g) / K ** 0.5).bfloat16()
    ob = torch.randn(N, device=DEV, generator=g) * 0.1
    ldy = N + off + 32
    y = torch.full((M, ldy), 7.0, device=DEV).bfloat16()
    hip.dn_conv1x1(x.data_ptr(), ldx, M, K, s.data_ptr(), b.data_ptr(), w.data_ptr(), N, ob.data_ptr(), 1,
                   y.data_ptr() + 2 * off, ldy, stream=torch.cuda.current_stream().cuda_stream, variant=variant)
    torch.cuda.synchronize()
    a = torch.relu(x[:, :K].float() * s + b).bfloat16().float()
    ref = torch.relu(a @ w.float().t() + ob)
    _close(y[:, off:off + N], ref)
    # columns outside the output slice are untouched
    assert (y[:, :off] == 7.0).all() and (y[:, off + N:] == 7.0).all()


@pytest.mark.parametrize("M,K,N,pool,splits", [(49, 992, 128, 0, 0), (196, 640, 128, 0, 4), (49, 1024, 512, 1, 0),
                                               (300, 96, 128, 0, 3), (1000, 512, 256, 0, 16)])
@pytest.mark.parametrize("variant", [0, 11, 12, 21, 42])
def test_conv1x1_split_k(M, K, N, pool, splits, variant):
    """Split-K partials + reduce must equal the single-pass kernel's math."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(K + N)
    H = 14 if pool else 0
    rows = M * 4 if pool else M
    if pool:
        M = 49
        rows = 196
    x = torch.randn(rows, K, device=DEV, generator=g).bfloat16()
    s = torch.rand(K, device=DEV, generator=g) + 0.5
    b = torch.randn(K, device=DEV, generator=g) * 0.2
    w = (torch.randn(N, K, device=DEV, generator=g) / K ** 0.5).bfloat16()
    ob = None if pool else torch.randn(N, device=DEV, generator=g)
    ws = torch.empty(16 * M * N * 4, device=DEV, dtype=torch.uint8)
    y = torch.zeros(M, N, device=DEV).bfloat16()
    hip.dn_conv1x1(x.data_ptr(), K, M, K, s.data_ptr(), b.data_ptr(), w.data_ptr(), N,
                   ob.data_ptr() if ob is not None else None, 0 if pool else 1, y.data_ptr(), N, pool=pool, H=H, W=H,
                   variant=variant, splits=splits, ws=ws.data_ptr(), ws_bytes=ws.numel())
    torch.cuda.synchronize()
    a = torch.relu(x.float() * s + b)
    if pool:
        a = F.avg_pool2d(a.view(1, 14, 14, K).permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1).reshape(M, K)
    a = a.bfloat16().float()
    ref = a @ w.float().t()
    if ob is not None:
        ref = torch.relu(ref + ob)
    _close(y, ref)


def test_conv1x1_plain_gemm():
    _need_gpu()
    hip = _hip()
    M, K, N = 777, 128, 128
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    y = torch.empty(M, N, device=DEV).bfloat16()
    hip.dn_conv1x1(x.data_ptr(), K, M, K, None, None, w.data_ptr(), N, None, 0, y.data_ptr(), N)
    torch.cuda.synchronize()
    _close(y, x.float() @ w.float().t())


@pytest.mark.parametrize("imgs,H,C,N", [(2, 14, 256, 128), (3, 28, 512, 256), (64, 14, 1024, 512)])
def test_conv1x1_transition_pool(imgs, H, C, N):
    _need_gpu()
    hip = _hip()
    x = torch.randn(imgs, H, H, C, device=DEV).bfloat16()
    s = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV) * 0.2
    w = (torch.randn(N, C, device=DEV) / C ** 0.5).bfloat16()
    Ho = H // 2
    M = imgs * Ho * Ho
    ldy = N + 64
    y = torch.zeros(M, ldy, device=DEV).bfloat16()
    hip.dn_conv1x1(x.data_ptr(), C, M, C, s.data_ptr(), b.data_ptr(), w.data_ptr(), N, None, 0, y.data_ptr(), ldy,
                   pool=1, H=H, W=H)
    torch.cuda.synchronize()
    a = torch.relu(x.float() * s + b).permute(0, 3, 1, 2)
    a = F.avg_pool2d(a, 2, 2).permute(0, 2, 3, 1).reshape(M, C).bfloat16().float()
    _close(y[:, :N], a @ w.float().t())
    assert (y[:, N:] == 0).all()


@pytest.mark.parametrize("variant", [0, 11, 70, 92])
@pytest.mark.parametrize("imgs,H", [(1, 7), (3, 14), (8, 56), (48, 56), (5, 28)])
def test_conv3x3(imgs, H, variant):
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(imgs * 100 + H)
    z = torch.randn(imgs, H, H, 128, device=DEV, generator=g).bfloat16()
    w = (torch.randn(32, 128, 3, 3, device=DEV, generator=g) / 34.0).bfloat16()
    wt = w.permute(0, 2, 3, 1).contiguous()
    ldy = 96
    y = torch.full((imgs * H * H, ldy), -3.0, device=DEV).bfloat16()
    hip.dn_conv3x3(z.data_ptr(), imgs, H, H, wt.data_ptr(), y.data_ptr() + 2 * 32, ldy, variant=variant)
    torch.cuda.synchronize()
    ref = F.conv2d(z.float().permute(0, 3, 1, 2), w.float(), padding=1).permute(0, 2, 3, 1).reshape(-1, 32)
    _close(y[:, 32:64], ref)
    assert (y[:, :32] == -3.0).all() and (y[:, 64:] == -3.0).all()


def test_stem_pool():
    _need_gpu()
    hip = _hip()
    x = torch.randn(3, 112, 112, 64, device=DEV).bfloat16()
    b = torch.randn(64, device=DEV)
    ldy = 256
    y = torch.zeros(3 * 56 * 56, ldy, device=DEV).bfloat16()
    hip.dn_stem_pool(x.data_ptr(), b.data_ptr(), y.data_ptr(), 3, 112, 112, 64, ldy)
    torch.cuda.synchronize()
    ref = torch.relu(F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1) + b.view(1, -1, 1, 1))
    ref = ref.permute(0, 2, 3, 1).reshape(-1, 64)
    _close(y[:, :64], ref, tol=1e-2)
    assert (y[:, 64:] == 0).all()


def _stem_ref(img_bf16_nchw, w, b):
    """fp32 conv7x7/2 on bf16-rounded operands, conv output rounded to bf16
    (the kernel keeps its conv tile in LDS as bf16), then max-pool + bias + ReLU."""
    c = F.conv2d(img_bf16_nchw.float(), w.bfloat16().float(), stride=2, padding=3).bfloat16().float()
    return torch.relu(F.max_pool2d(c, 3, 2, 1) + b.view(1, -1, 1, 1)).permute(0, 2, 3, 1).reshape(-1, 64)


def _pack_stem_w(w):
    wp = torch.zeros(64, 7, 8, 4, device=w.device)
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    return wp.reshape(64, -1).bfloat16().contiguous()


@pytest.mark.parametrize("imgs", [1, 3])
@pytest.mark.parametrize("mode", ["ptrs_fp32_nchw", "bf16_nhwc"])
def test_stem_fused(imgs, mode):
    """K10s (conv 7x7/2 + bias + ReLU + max-pool 3x3/2 in one kernel) vs torch fp32."""
    _need_gpu()
    hip = _hip()
    g = torch.Generator(device=DEV).manual_seed(11 + imgs)
    w = torch.randn(64, 3, 7, 7, device=DEV, generator=g) * 0.1
    b = torch.randn(64, device=DEV, generator=g) * 0.2
    x = torch.randn(imgs, 3, 224, 224, device=DEV, generator=g)
    ldy = 256
    y = torch.full((imgs * 56 * 56, ldy), 5.0, device=DEV).bfloat16()
    wp = _pack_stem_w(w)
    if mode == "ptrs_fp32_nchw":
        # separate allocations, as with one shm region per request
        imgs_t = [x[i].clone() for i in range(imgs)]
        tbl = torch.tensor([t.data_ptr() for t in imgs_t], device=DEV, dtype=torch.int64)
        hip.dn_stem_fused(tbl.data_ptr(), None, wp.data_ptr(), b.data_ptr(), y.data_ptr(), imgs, ldy)
    else:
        xn = x.bfloat16().permute(0, 2, 3, 1).contiguous()
        hip.dn_stem_fused(None, xn.data_ptr(), wp.data_ptr(), b.data_ptr(), y.data_ptr(), imgs, ldy)
    torch.cuda.synchronize()
    ref = _stem_ref(x.bfloat16(), w, b)
    _close(y[:, :64], ref, tol=1e-2)
    assert (y[:, 64:] == 5.0).all()


def test_head_pool():
    _need_gpu()
    hip = _hip()
    x = torch.randn(5, 49, 1024, device=DEV).bfloat16()
    s = torch.rand(1024, device=DEV) + 0.5
    b = torch.randn(1024, device=DEV) * 0.1
    out = torch.empty(5, 1024, device=DEV).bfloat16()
    hip.dn_head_pool(x.data_ptr(), s.data_ptr(), b.data_ptr(), out.data_ptr(), 5, 49, 1024)
    torch.cuda.synchronize()
    ref = torch.relu(x.float() * s + b).mean(1)
    _close(out, ref, tol=1e-2)


def test_rejects_bad_shapes():
    _need_gpu()
    hip = _hip()
    x = torch.zeros(64, 64, device=DEV).bfloat16()
    with pytest.raises(Exception):  # N not a multiple of 128
        hip.dn_conv1x1(x.data_ptr(), 64, 64, 64, None, None, x.data_ptr(), 64, None, 0, x.data_ptr(), 64)
    with pytest.raises(Exception):  # K not a multiple of 32
        hip.dn_conv1x1(x.data_ptr(), 64, 64, 48, None, None, x.data_ptr(), 128, None, 0, x.data_ptr(), 128)


@pytest.mark.parametrize("batch", [1, 5, 32])
def test_fused_densenet_matches_fp32_module(batch):
    """End to end vs the fp32 module; the yardstick is the plain bf16 torch
    module's own error (bf16 storage through 121 layers), not a fixed bound."""
    _need_gpu()
    import copy

    from triton_client_amd.models import densenet_fused

    eng, model = densenet_fused.build(max_batch=32, device=DEV)
    m32 = copy.deepcopy(model).to(DEV).float()
    m16 = copy.deepcopy(model).to(DEV, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(batch, 3, 224, 224, device=DEV)
    with torch.no_grad():
        ref = m32(x)
        xb = x.bfloat16().contiguous(memory_format=torch.channels_last)
        got = eng(xb)
        base = m16(xb).float()
    torch.cuda.synchronize()
    assert got.shape == (batch, 1000) and got.dtype == torch.float32
    rel = lambda a: ((a - ref).norm() / ref.norm()).item()  # noqa: E731
    e_fused, e_torch = rel(got), rel(base)
    print("rel-L2 vs fp32: fused %.4f  torch-bf16 %.4f" % (e_fused, e_torch))
    assert e_fused < max(0.03, 1.5 * e_torch)
    assert torch.isfinite(got).all()
    cos = F.cosine_similarity(got, ref, dim=1)
    assert cos.min().item() > 0.99


def test_fused_densenet_graph_replay():
    _need_gpu()
    from triton_client_amd.models import densenet_fused

    eng, _ = densenet_fused.build(max_batch=8, device=DEV)
    x = torch.randn(8, 3, 224, 224, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    out = torch.zeros(8, 1000, device=DEV)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s), torch.no_grad():
        eng(x, out)
        eager = out.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            eng(x, out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
