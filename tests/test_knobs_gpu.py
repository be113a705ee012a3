"""The native knobs (csrc/runtime/knobs.hip), switched in-process, against the
same fp64 references as the default paths: every plan variant a knob selects
must give the default path's numbers, the diagnostic ablations must run and
leave the next default launch correct, and the stamp / timeline builds must
record and still compute.  Knob table: triton_client_amd/utils/knobs.py."""

import numpy as np
import pytest

torch = pytest.importorskip("torch")
F = torch.nn.functional

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture
def hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from triton_client_amd.ops import hip as h

    h.lib()
    before = {k: v["value"] for k, v in h.knobs().items()}
    yield h
    assert {k: v["value"] for k, v in h.knobs().items()} == before, "a knob was left changed"


def _rel(got, ref):
    got, ref = got.double(), ref.double()
    assert torch.isfinite(got).all()
    return ((got - ref).norm() / ref.norm().clamp_min(1e-30)).item()


def _split(t):
    hi = t.to(torch.bfloat16)
    return hi.contiguous(), (t - hi.float()).to(torch.bfloat16).contiguous()


def _st():
    return torch.cuda.current_stream().cuda_stream


def _layer(M, K, seed, ldx=None):
    g = torch.Generator(device=DEV).manual_seed(seed)
    ldx = ldx or K + 64
    d = {"x": torch.randn(M, ldx, device=DEV, generator=g), "ldx": ldx, "K": K, "M": M,
         "s": torch.rand(K, device=DEV, generator=g) + 0.5, "t": torch.randn(K, device=DEV, generator=g) * 0.2,
         "w1": torch.randn(128, K, device=DEV, generator=g) / K ** 0.5,
         "b1": torch.randn(128, device=DEV, generator=g) * 0.1,
         "w2": torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5}
    return d


def _z_ref(d):
    a = torch.relu(d["x"][:, :d["K"]].double() * d["s"].double() + d["t"].double())
    return torch.relu(a @ d["w1"].double().t() + d["b1"].double())


def _layer_ref(d, imgs, H):
    z = _z_ref(d).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
    return F.conv2d(z, d["w2"].double(), padding=1).permute(0, 2, 3, 1).reshape(-1, 32)


def _conv1x1(hip, d):
    M, K = d["M"], d["K"]
    wh, wl = _split(d["w1"])
    zh = torch.empty(M, 128, device=DEV, dtype=torch.bfloat16)
    zl = torch.empty_like(zh)
    wsb = hip.x3_conv1x1_ws_bytes(M, K)
    ws = torch.empty(max(wsb, 16), device=DEV, dtype=torch.uint8)
    hip.x3_conv1x1(d["x"].data_ptr(), d["ldx"], M, K, d["s"].data_ptr(), d["t"].data_ptr(), wh.data_ptr(),
                   wl.data_ptr(), out_bias=d["b1"].data_ptr(), z_hi=zh.data_ptr(), z_lo=zl.data_ptr(),
                   ws=ws.data_ptr(), ws_bytes=wsb, stream=_st())
    torch.cuda.synchronize()
    return zh.double() + zl.double(), wsb


def _fused(hip, d, imgs, H, version=1):
    K, ldx = d["K"], d["ldx"]
    f1h, f1l = (hip.x3_w1_fragments(u) for u in _split(d["w1"]))
    f2h, f2l = (hip.x3_w3f_fragments(u) for u in _split(d["w2"].permute(0, 2, 3, 1).reshape(32, -1)))
    y = d["x"].clone()
    fn = hip.x3_dense_fused3 if version == 3 else hip.x3_dense_fused
    fn(y.data_ptr(), ldx, imgs, H, H, K, d["s"].data_ptr(), d["t"].data_ptr(), f1h.data_ptr(), f1l.data_ptr(),
       d["b1"].data_ptr(), f2h.data_ptr(), f2l.data_ptr(), y.data_ptr() + 4 * K, ldx, stream=_st())
    torch.cuda.synchronize()
    return y[:, K:K + 32]


def _small(hip, d, imgs, H, tiles=0):
    K, ldx = d["K"], d["ldx"]
    f1h, f1l = (hip.x3_w1_fragments(u) for u in _split(d["w1"]))
    f2h, f2l = (hip.x3_w3f_fragments(u) for u in _split(d["w2"].permute(0, 2, 3, 1).reshape(32, -1)))
    y = d["x"].clone()
    hip.x3_dense_small(y.data_ptr(), ldx, imgs, H, H, K, d["s"].data_ptr(), d["t"].data_ptr(), f1h.data_ptr(),
                       f1l.data_ptr(), d["b1"].data_ptr(), f2h.data_ptr(), f2l.data_ptr(), y.data_ptr() + 4 * K, ldx,
                       stream=_st(), tiles=tiles)
    torch.cuda.synchronize()
    return y[:, K:K + 32]


def _conv3x3(hip, imgs, H, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    M = imgs * H * H
    z = torch.relu(torch.randn(M, 128, device=DEV, generator=g))
    w = torch.randn(32, 128, 3, 3, device=DEV, generator=g) / (9 * 128) ** 0.5
    zh, zl = _split(z)
    wh, wl = (hip.x3_w3_fragments(t) for t in _split(w.permute(0, 2, 3, 1).reshape(32, -1)))
    y = torch.zeros(M, 32, device=DEV)
    hip.x3_conv3x3(zh.data_ptr(), zl.data_ptr(), imgs, H, H, wh.data_ptr(), wl.data_ptr(), y.data_ptr(), 32,
                   stream=_st())
    torch.cuda.synchronize()
    zin = (zh.double() + zl.double()).reshape(imgs, H, H, 128).permute(0, 3, 1, 2)
    return y, F.conv2d(zin, w.double(), padding=1).permute(0, 2, 3, 1).reshape(M, 32)


_PLANS = [{}, {"TCAMD_X3_BM": 32}, {"TCAMD_X3_BM": 64}, {"TCAMD_X3_BM": 128}, {"TCAMD_X3_SPLITK_BELOW": 0},
          {"TCAMD_X3_SPLITK_BELOW": 100000}, {"TCAMD_X3_MAX_SPLITS": 1}, {"TCAMD_X3_MAX_SPLITS": 8},
          {"TCAMD_X3_WS": 0}, {"TCAMD_X3_WS_MIN": 60000}]


@pytest.mark.parametrize("M,K", [(392, 992), (6272, 512), (50000, 224), (65555, 64)])
def test_k8x_plan_knobs(hip, M, K):
    """K8x 1x1 under every plan knob (tile rows, split-K threshold and cap,
    warp-specialised kernel off / floor moved) against fp64; the split-K
    workspace size follows the plan."""
    d = _layer(M, K, seed=M + K)
    ref = _z_ref(d)
    sizes = {}
    for kn in _PLANS:
        with hip.knob(**kn):
            got, wsb = _conv1x1(hip, d)
        sizes[tuple(kn.items())] = wsb
        err = _rel(got, ref)
        print("K8x M %d K %d %s: rel %.3g, split-K ws %d B" % (M, K, kn or "default", err, wsb))
        assert err < 3e-5, kn
    if M == 392:  # 4 tiles of 128 rows: split-K by default, none when the threshold is 0
        assert sizes[()] > 0 and sizes[(("TCAMD_X3_SPLITK_BELOW", 0),)] == 0
        assert sizes[(("TCAMD_X3_MAX_SPLITS", 1),)] == 0


@pytest.mark.parametrize("bpc", [1, 2, 4, 8])
def test_stem_blocks_per_cu(hip, bpc):
    """K10x stem with TCAMD_X3_STEM_BPC persistent workgroups per CU (fewer:
    more tiles per workgroup) against fp64."""
    imgs = 24
    g = torch.Generator(device=DEV).manual_seed(bpc)
    x = torch.randn(imgs, 3, 224, 224, device=DEV, generator=g)
    w = torch.randn(64, 3, 7, 7, device=DEV, generator=g) / 12
    bias = torch.randn(64, device=DEV, generator=g) * 0.1
    wp = torch.zeros(64, 7, 8, 4, device=DEV)
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    wh, wl = (hip.x3_stem_fragments(t) for t in _split(wp.reshape(64, -1)))
    ptrs = torch.tensor([x[i].data_ptr() for i in range(imgs)], device=DEV, dtype=torch.int64)
    y = torch.full((imgs * 56 * 56, 64), 7.0, device=DEV)
    with hip.knob(TCAMD_X3_STEM_BPC=bpc):
        hip.x3_stem(ptrs.data_ptr(), wh.data_ptr(), wl.data_ptr(), bias.data_ptr(), y.data_ptr(), imgs, 64,
                    stream=_st())
    torch.cuda.synchronize()
    c = F.conv2d(x.double(), w.double(), stride=2, padding=3)
    ref = torch.relu(F.max_pool2d(c, 3, 2, 1) + bias.double().view(1, -1, 1, 1)).permute(0, 2, 3, 1).reshape(-1, 64)
    assert _rel(y, ref) < 2e-5


def _x3s(hip, d, imgs, H):
    K, ldx, M = d["K"], d["ldx"], d["M"]
    f1h, f1l = (hip.x3_w1_fragments(u) for u in _split(d["w1"]))
    f2h, f2l = (hip.x3_w3_fragments(u) for u in _split(d["w2"].permute(0, 2, 3, 1).reshape(32, -1)))
    y = d["x"].clone()
    zacc = torch.zeros(M, 128, device=DEV)
    hip.x3s_dense_layer(y.data_ptr(), ldx, imgs, H, H, K, d["s"].data_ptr(), d["t"].data_ptr(), f1h.data_ptr(),
                        f1l.data_ptr(), d["b1"].data_ptr(), zacc.data_ptr(), None, f2h.data_ptr(), f2l.data_ptr(),
                        y.data_ptr() + 4 * K, ldx, stream=_st())
    torch.cuda.synchronize()
    return y[:, K:K + 32].clone()


def test_k13x_chunking_and_split3(hip):
    """K13x small-M layer under its knobs: K chunking (target workgroups, chunk
    cap) and the 3x3 split over input quarters; with <= 2 chunks and the split
    off the layer is bitwise reproducible (no float-atomic ordering left)."""
    imgs, H, K = 2, 14, 512
    d = _layer(imgs * H * H, K, seed=7)
    ref = _layer_ref(d, imgs, H)
    for kn in ({}, {"TCAMD_X3S_BLOCKS": 64}, {"TCAMD_X3S_BLOCKS": 2048}, {"TCAMD_X3S_MAX_CHUNKS": 1},
               {"TCAMD_X3S_MAX_CHUNKS": 16}, {"TCAMD_X3S_SPLIT3": 0}):
        with hip.knob(**kn):
            assert _rel(_x3s(hip, d, imgs, H), ref) < 3e-5, kn
    with hip.knob(TCAMD_X3S_MAX_CHUNKS=2, TCAMD_X3S_SPLIT3=0):
        runs = [_x3s(hip, d, imgs, H) for _ in range(3)]
    assert all(torch.equal(runs[0], r) for r in runs[1:])


def test_k3_general_walk_mode(hip):
    """TCAMD_K3_MODE=1 sends every index through the general pointer-doubling
    walk (path 2) with the same offsets / lengths as the windowed v3 walk."""
    rng = np.random.default_rng(0)
    n = 3000
    lens = rng.integers(0, 41, n).astype(np.uint32)
    buf, offs = bytearray(), np.empty(n, np.uint64)
    for i, L in enumerate(lens):
        buf += int(L).to_bytes(4, "little")
        offs[i] = len(buf)
        buf += bytes(rng.integers(97, 123, int(L), dtype=np.uint8))
    data = torch.frombuffer(bytearray(bytes(buf) + b"\0" * 64), dtype=torch.uint8).cuda()
    o = torch.empty(n, dtype=torch.int64, device=DEV)
    ln = torch.empty(n, dtype=torch.int32, device=DEV)
    st = torch.empty(4, dtype=torch.int32, device=DEV)
    s = torch.cuda.current_stream().cuda_stream
    for mode, path in ((1, 2), (0, 1)):
        o.zero_()
        with hip.knob(TCAMD_K3_MODE=mode):
            hip.index_bytes(data.data_ptr(), len(buf), n, o.data_ptr(), ln.data_ptr(), st.data_ptr(), s)
            assert hip.index_bytes_last_path()[0] == path
        torch.cuda.synchronize()
        assert int(st[0]) == 0
        np.testing.assert_array_equal(o.cpu().numpy().astype(np.uint64), offs)
        np.testing.assert_array_equal(ln.cpu().numpy().astype(np.uint32), lens)


def test_bert_tuned_gemm_table(monkeypatch):
    """TC_BERT_TUNED_GEMMS=1: the committed TunableOp table loads in this image
    (its validators match) and a bf16 forward through it agrees with the
    library-default solutions to bf16 rounding.  TunableOp is process-wide:
    switched off again at the end."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.cuda.tunable as tun

    from triton_client_amd.models import bert

    m = bert.build(device="cuda", dtype=torch.bfloat16, layers=2)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(1000, 30000, (8, 384), generator=g).cuda()
    mask = torch.ones(8, 384, dtype=torch.int32, device="cuda")
    tt = torch.zeros(8, 384, dtype=torch.long, device="cuda")
    with torch.no_grad():
        base = [t.float() for t in m(ids, mask, tt)]
    monkeypatch.setenv("TC_BERT_TUNED_GEMMS", "0")
    assert not bert.use_tuned_gemms()
    monkeypatch.setenv("TC_BERT_TUNED_GEMMS", "1")
    try:
        on = bert.use_tuned_gemms()
        assert on, "the gfx950 TunableOp table did not load (validators differ from this image?)"
        with torch.no_grad():
            got = [t.float() for t in m(ids, mask, tt)]
    finally:
        tun.enable(False)
    for a, b in zip(got, base):
        assert _rel(a, b) < 2e-2
