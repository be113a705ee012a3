"""Numerics of the CDNA4 kernels (csrc/kernels/*.hip) against numpy / fp32
torch references of the same op.  All tests run through libtcamd_hip.so."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from tests.philox_ref import raw_u32, uniform_f32  # noqa: E402


@pytest.fixture(scope="module")
def env():
    import torch

    from triton_client_amd.ops import hip

    torch.cuda.set_device(0)
    return torch, hip


def _stream(torch):
    return torch.cuda.current_stream().cuda_stream


def test_native_library_is_loaded(env):
    torch, hip = env
    import os

    assert os.path.exists(hip.loaded_path())
    assert hip.device_count() >= 1
    assert hip.device_arch(0).startswith("gfx950")


@pytest.mark.parametrize("n", [1, 15, 4096, 1000003])
def test_synth_uniform_fp32_matches_philox_reference(env, n):
    torch, hip = env
    t = torch.empty(n + 16, device="cuda", dtype=torch.float32)
    hip.synth_fill(t.data_ptr(), n, "FP32", hip.SYNTH_UNIFORM, -2.0, 3.0, seed=99, stream_id=5,
                   stream=_stream(torch))
    got = t[:n].cpu().numpy()
    ref = uniform_f32(n, -2.0, 3.0, seed=99, stream_id=5)
    np.testing.assert_array_equal(got, ref)


def test_synth_int32_range_and_determinism(env):
    torch, hip = env
    n = 100000
    a = torch.empty(n, device="cuda", dtype=torch.int32)
    b = torch.empty(n, device="cuda", dtype=torch.int32)
    for t in (a, b):
        hip.synth_fill(t.data_ptr(), n, "INT32", hip.SYNTH_UNIFORM, 0, 30521, seed=3, stream=_stream(torch))
    assert torch.equal(a, b)
    x = a.cpu().numpy()
    assert x.min() >= 0 and x.max() <= 30521
    ref = (raw_u32(n, 4, seed=3).astype(np.int64) % 30522).astype(np.int32)
    np.testing.assert_array_equal(x, ref)


@pytest.mark.parametrize("dt,tdt", [("BF16", "bfloat16"), ("FP16", "float16"), ("INT8", "int8"),
                                    ("UINT8", "uint8"), ("INT64", "int64"), ("BOOL", "bool")])
def test_synth_other_dtypes(env, dt, tdt):
    torch, hip = env
    n = 4099
    t = torch.zeros(n + 64, device="cuda", dtype=getattr(torch, tdt))
    lo, hi = (0, 1) if dt == "BOOL" else (-5, 5) if dt in ("INT8", "INT64") else (0, 200) if dt == "UINT8" else (-1.0, 1.0)
    hip.synth_fill(t.data_ptr(), n, dt, hip.SYNTH_UNIFORM, lo, hi, seed=11, stream=_stream(torch))
    x = t[:n].float().cpu().numpy()
    assert x.min() >= lo and x.max() <= hi
    assert np.unique(x).size > 1
    assert (t[n:].float() == 0).all()  # no overrun past n elements


def test_synth_zero_const_normal(env):
    torch, hip = env
    n = 1 << 20
    t = torch.ones(n, device="cuda")
    hip.synth_fill(t.data_ptr(), n, "FP32", hip.SYNTH_ZERO, stream=_stream(torch))
    assert float(t.abs().sum()) == 0.0
    hip.synth_fill(t.data_ptr(), n, "FP32", hip.SYNTH_CONST, 2.5, stream=_stream(torch))
    assert bool((t == 2.5).all())
    hip.synth_fill(t.data_ptr(), n, "FP32", hip.SYNTH_NORMAL, 1.0, 2.0, seed=4, stream=_stream(torch))
    assert abs(float(t.mean()) - 1.0) < 0.02 and abs(float(t.std()) - 2.0) < 0.02


@pytest.mark.parametrize("n", [7, 8, 1023, 262147])
def test_convert_bf16_trunc_is_wire_compatible(env, n):
    torch, hip = env
    from tritonclient.utils import serialize_bf16_tensor

    x = torch.randn(n, device="cuda") * 100
    y = torch.empty(n, device="cuda", dtype=torch.int16)
    hip.convert(x.data_ptr(), "FP32", y.data_ptr(), "BF16", n, "trunc", _stream(torch))
    got = y.cpu().numpy().tobytes()
    assert got == serialize_bf16_tensor(x.cpu().numpy()).item()


def test_convert_bf16_rne_matches_torch(env):
    torch, hip = env
    n = 100003
    x = torch.randn(n, device="cuda") * 10
    y = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    hip.convert(x.data_ptr(), "FP32", y.data_ptr(), "BF16", n, "rne", _stream(torch))
    assert torch.equal(y, x.to(torch.bfloat16))
    back = torch.empty(n, device="cuda")
    hip.convert(y.data_ptr(), "BF16", back.data_ptr(), "FP32", n, stream=_stream(torch))
    assert torch.equal(back, y.float())


def test_convert_fp16_roundtrip(env):
    torch, hip = env
    n = 65541
    x = torch.randn(n, device="cuda") * 50
    y = torch.empty(n, device="cuda", dtype=torch.float16)
    hip.convert(x.data_ptr(), "FP32", y.data_ptr(), "FP16", n, stream=_stream(torch))
    assert torch.equal(y, x.half())
    z = torch.empty(n, device="cuda")
    hip.convert(y.data_ptr(), "FP16", z.data_ptr(), "FP32", n, stream=_stream(torch))
    assert torch.equal(z, y.float())


@pytest.mark.parametrize("fmt,tfmt", [("FP8_E4M3", "float8_e4m3fn"), ("FP8_E5M2", "float8_e5m2")])
def test_convert_fp8_matches_reference(env, fmt, tfmt):
    torch, hip = env
    from tritonclient.utils import deserialize_fp8_tensor, serialize_fp8_tensor

    n = 40961
    x = torch.randn(n, device="cuda") * (100 if fmt == "FP8_E4M3" else 10000)
    y = torch.empty(n, device="cuda", dtype=torch.uint8)
    hip.convert(x.data_ptr(), "FP32", y.data_ptr(), fmt, n, stream=_stream(torch))
    got = y.cpu().numpy()
    ref = np.frombuffer(serialize_fp8_tensor(x.cpu().numpy(), fmt).item(), dtype=np.uint8)
    np.testing.assert_array_equal(got, ref)
    # in-range values also match torch's (non-saturating) float8 cast
    maxv = 448.0 if fmt == "FP8_E4M3" else 57344.0
    inr = x.abs() < maxv
    tref = x.to(getattr(torch, tfmt)).view(torch.uint8)
    assert torch.equal(y[inr], tref[inr])
    z = torch.empty(n, device="cuda")
    hip.convert(y.data_ptr(), fmt, z.data_ptr(), "FP32", n, stream=_stream(torch))
    np.testing.assert_array_equal(z.cpu().numpy(), deserialize_fp8_tensor(got.tobytes(), fmt))


def test_layout_pack_nchw_to_nhwc_bf16_gather(env):
    torch, hip = env
    imgs = [torch.randn(3, 224, 224, device="cuda") for _ in range(5)]
    out = torch.empty(5, 224, 224, 3, device="cuda", dtype=torch.bfloat16)
    hip.layout_pack([t.data_ptr() for t in imgs], "FP32", "NCHW", out.data_ptr(), "BF16", "NHWC", 3, 224, 224,
                    stream=_stream(torch))
    ref = torch.stack(imgs).permute(0, 2, 3, 1).to(torch.bfloat16)
    assert torch.equal(out, ref)


def test_layout_pack_affine_u8_nhwc_to_nchw(env):
    torch, hip = env
    img = torch.randint(0, 256, (2, 64, 48, 3), device="cuda", dtype=torch.uint8)
    out = torch.empty(2, 3, 64, 48, device="cuda")
    scale = [1 / 127.5] * 3
    bias = [-1.0] * 3
    hip.layout_pack([img[0].data_ptr(), img[1].data_ptr()], "UINT8", "NHWC", out.data_ptr(), "FP32", "NCHW",
                    3, 64, 48, scale=scale, bias=bias, stream=_stream(torch))
    ref = img.permute(0, 3, 1, 2).float() * (1 / 127.5) - 1.0
    assert torch.allclose(out, ref, atol=1e-6)


@pytest.mark.parametrize("C,H,W", [(37, 9, 13), (64, 14, 14), (5, 7, 7)])
def test_layout_pack_general_c_tiled_path(env, C, H, W):
    torch, hip = env
    x = torch.randn(3, C, H, W, device="cuda")
    out = torch.empty(3, H, W, C, device="cuda", dtype=torch.float16)
    hip.layout_pack([x[i].data_ptr() for i in range(3)], "FP32", "NCHW", out.data_ptr(), "FP16", "NHWC",
                    C, H, W, stream=_stream(torch))
    assert torch.equal(out, x.permute(0, 2, 3, 1).half())
    back = torch.empty(3, C, H, W, device="cuda")
    hip.layout_pack([out[i].data_ptr() for i in range(3)], "FP16", "NHWC", back.data_ptr(), "FP32", "NCHW",
                    C, H, W, stream=_stream(torch))
    assert torch.equal(back, x.half().float())


def test_batched_copy_mixed_alignment(env):
    torch, hip = env
    src = torch.randint(0, 255, (1 << 20,), device="cuda", dtype=torch.uint8)
    dst = torch.zeros_like(src)
    rng = np.random.default_rng(0)
    srcs, dsts, sizes = [], [], []
    off = 0
    for i in range(40):
        n = int(rng.integers(1, 20000))
        so = int(rng.integers(0, 4)) if i % 3 == 0 else 0
        srcs.append(src.data_ptr() + off + so)
        dsts.append(dst.data_ptr() + off)
        sizes.append(n)
        off += ((n + so + 15) // 16) * 16 + 16
    hip.batched_copy(srcs, dsts, sizes, _stream(torch))
    torch.cuda.synchronize()
    s = src.cpu().numpy()
    d = dst.cpu().numpy()
    for sp, dp, n in zip(srcs, dsts, sizes):
        a = sp - src.data_ptr()
        b = dp - dst.data_ptr()
        assert (s[a : a + n] == d[b : b + n]).all()


def test_pack_and_index_bytes_match_wire_format(env):
    torch, hip = env
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(1)
    elems = [bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8)) for _ in range(5000)]
    lens = np.array([len(e) for e in elems], dtype=np.uint32)
    payload = np.frombuffer(b"".join(elems), dtype=np.uint8)
    d_payload = torch.from_numpy(payload.copy()).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32).copy()).cuda()
    total = int(lens.sum()) + 4 * len(elems)
    out = torch.zeros(total, device="cuda", dtype=torch.uint8)
    ws = torch.empty(hip.pack_bytes_workspace(len(elems)), device="cuda", dtype=torch.uint8)
    hip.pack_bytes(d_payload.data_ptr(), d_lens.data_ptr(), len(elems), out.data_ptr(), ws.data_ptr(),
                   _stream(torch))
    ref = serialize_byte_tensor(np.array(elems, dtype=np.object_)).item()
    assert out.cpu().numpy().tobytes() == ref
    offs = torch.empty(len(elems), device="cuda", dtype=torch.int64)
    lns = torch.empty(len(elems), device="cuda", dtype=torch.int32)
    status = torch.zeros(4, device="cuda", dtype=torch.int32)
    hip.index_bytes(out.data_ptr(), total, len(elems), offs.data_ptr(), lns.data_ptr(), status.data_ptr(),
                    _stream(torch))
    st = status.cpu().numpy()
    assert st[0] == 0
    np.testing.assert_array_equal(lns.cpu().numpy().view(np.uint32), lens)
    exp_offs = np.cumsum(np.concatenate([[0], lens[:-1].astype(np.int64) + 4])) + 4
    np.testing.assert_array_equal(offs.cpu().numpy(), exp_offs)


@pytest.mark.parametrize("n,maxlen,seed", [(300000, 24, 5), (4000, 6000, 6), (70000, 1, 7)])
def test_pack_and_index_bytes_large(env, n, maxlen, seed):
    """K2 output-centric emit and the K3 parallel block walk on large inputs:
    many short strings, few very long ones (each spans many 16-B chunks and
    several 8 KiB index blocks), and all-but-empty elements."""
    torch, hip = env
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen + 1, n).astype(np.uint32)
    payload = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    d_payload = torch.from_numpy(payload).cuda() if payload.size else torch.zeros(16, device="cuda", dtype=torch.uint8)
    d_lens = torch.from_numpy(lens.view(np.int32).copy()).cuda()
    total = int(lens.sum()) + 4 * n
    out = torch.zeros(total + 64, device="cuda", dtype=torch.uint8)
    ws = torch.empty(hip.pack_bytes_workspace(n), device="cuda", dtype=torch.uint8)
    hip.pack_bytes(d_payload.data_ptr(), d_lens.data_ptr(), n, out.data_ptr(), ws.data_ptr(), _stream(torch))
    starts = np.concatenate([[0], np.cumsum(lens.astype(np.int64))])
    elems = [payload[starts[i]:starts[i + 1]].tobytes() for i in range(n)]
    ref = serialize_byte_tensor(np.array(elems, dtype=np.object_)).item()
    got = out.cpu().numpy()
    assert got[:total].tobytes() == ref and not got[total:].any()
    offs = torch.empty(n, device="cuda", dtype=torch.int64)
    lns = torch.empty(n, device="cuda", dtype=torch.int32)
    status = torch.zeros(4, device="cuda", dtype=torch.int32)
    # index over the whole (zero-padded) buffer: trailing zeros are not asked for
    hip.index_bytes(out.data_ptr(), total + 64, n, offs.data_ptr(), lns.data_ptr(), status.data_ptr(), _stream(torch))
    st = status.cpu().numpy()
    assert st[0] == 0 and int(st[2:4].view(np.uint64)[0]) == n
    np.testing.assert_array_equal(lns.cpu().numpy().view(np.uint32), lens)
    exp_offs = starts[:-1] + 4 * np.arange(1, n + 1)
    np.testing.assert_array_equal(offs.cpu().numpy(), exp_offs)
    # truncate the buffer inside element n//2: malformed (the element is requested)
    e = n // 2
    cut = int(exp_offs[e]) + int(lens[e]) - 1 if lens[e] > 0 else int(exp_offs[e]) - 2
    status.zero_()
    hip.index_bytes(out.data_ptr(), cut, n, offs.data_ptr(), lns.data_ptr(), status.data_ptr(), _stream(torch))
    assert int(status[0].item()) == -1
    # fewer elements asked than present: status ok, only those indexed
    status.zero_()
    hip.index_bytes(out.data_ptr(), total, n // 3, offs.data_ptr(), lns.data_ptr(), status.data_ptr(), _stream(torch))
    assert int(status[0].item()) == 0
    np.testing.assert_array_equal(offs.cpu().numpy()[: n // 3], exp_offs[: n // 3])


def _index(torch, hip, buf, nbytes, n):
    offs = torch.empty(max(n, 1), device="cuda", dtype=torch.int64)
    lns = torch.empty(max(n, 1), device="cuda", dtype=torch.int32)
    status = torch.zeros(4, device="cuda", dtype=torch.int32)
    hip.index_bytes(buf.data_ptr(), nbytes, n, offs.data_ptr(), lns.data_ptr(), status.data_ptr(), _stream(torch))
    st = status.cpu().numpy()
    return int(st[0]), int(st[2:4].view(np.uint64)[0]), offs.cpu().numpy()[:n], lns.cpu().numpy().view(np.uint32)[:n]


def _wire(elems):
    from tritonclient.utils import serialize_byte_tensor

    return np.frombuffer(serialize_byte_tensor(np.array(elems, dtype=np.object_)).item(), dtype=np.uint8)


def _expect(elems):
    lens = np.array([len(e) for e in elems], dtype=np.int64)
    return np.cumsum(np.concatenate([[0], lens[:-1] + 4])) + 4, lens.astype(np.uint32)


@pytest.mark.parametrize("kind", ["ascii", "zeros", "binary", "empty"])
def test_index_bytes_v3_speculative_walk(env, kind):
    """K3 v3: candidate walks + resolve + emit on ~1.5 MB of BYTES with a
    tail of unrelated region bytes; must match the host walk and take the
    v3 path with the 64-B candidate window (elements shorter than 60 B)."""
    torch, hip = env
    rng = np.random.default_rng({"ascii": 1, "zeros": 2, "binary": 3, "empty": 4}[kind])
    n = 60000
    if kind == "empty":
        elems = [b""] * n
    else:
        ln = rng.integers(0, 40, n)
        if kind == "zeros":
            elems = [bytes(int(k)) for k in ln]
        elif kind == "binary":
            elems = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in ln]
        else:
            elems = [bytes(rng.integers(32, 127, int(k), dtype=np.uint8)) for k in ln]
    wire = _wire(elems)
    region = np.concatenate([wire, rng.integers(0, 256, 5000, dtype=np.uint8)])
    buf = torch.from_numpy(region).cuda()
    st, found, offs, lens = _index(torch, hip, buf, region.size, n)
    path, window = hip.index_bytes_last_path()
    assert st == 0 and found == n
    eo, el = _expect(elems)
    np.testing.assert_array_equal(offs, eo)
    np.testing.assert_array_equal(lens, el)
    assert path == 1, "expected the v3 speculative walk, got path %d" % path


def test_index_bytes_small_tensor_in_large_region_scans_a_window(env):
    """a small BYTES tensor (>= 2048 elements) at the start of a
    256 MB region must not walk (or allocate scratch for) the whole region."""
    torch, hip = env
    rng = np.random.default_rng(9)
    elems = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(0, 30, 3000)]
    wire = _wire(elems)
    buf = torch.zeros(256 << 20, device="cuda", dtype=torch.uint8)
    buf[: wire.size] = torch.from_numpy(wire).cuda()
    st, found, offs, lens = _index(torch, hip, buf, buf.numel(), len(elems))
    path, window = hip.index_bytes_last_path()
    assert st == 0 and found == len(elems)
    eo, el = _expect(elems)
    np.testing.assert_array_equal(offs, eo)
    np.testing.assert_array_equal(lens, el)
    assert path == 1 and window <= (1 << 20), (path, window)


def test_index_bytes_window_grows_and_long_elements_fall_back(env):
    torch, hip = env
    rng = np.random.default_rng(10)
    # 4000 elements of ~700 B: 64 * n = 256 KB is too small a first window (retry x8),
    # and elements longer than 252 B send the chain to the general walk
    elems = [bytes(rng.integers(0, 256, int(k), dtype=np.uint8)) for k in rng.integers(500, 900, 4000)]
    wire = _wire(elems)
    buf = torch.from_numpy(np.concatenate([wire, np.zeros(1 << 22, np.uint8)])).cuda()
    st, found, offs, lens = _index(torch, hip, buf, buf.numel(), len(elems))
    path, _ = hip.index_bytes_last_path()
    assert st == 0 and found == len(elems) and path == 2
    eo, el = _expect(elems)
    np.testing.assert_array_equal(offs, eo)
    np.testing.assert_array_equal(lens, el)
    # elements of 150-250 B and a first window that is too small: v3 retries
    # with 8x windows, and with the 256-B candidate window (longer than 60 B)
    elems = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(150, 250, 12000)]
    wire = _wire(elems)
    buf = torch.from_numpy(np.concatenate([wire, np.zeros(1 << 22, np.uint8)])).cuda()
    st, found, offs, lens = _index(torch, hip, buf, buf.numel(), len(elems))
    path, window = hip.index_bytes_last_path()
    assert st == 0 and found == len(elems) and path == 3 and window > (1 << 20)
    eo, el = _expect(elems)
    np.testing.assert_array_equal(offs, eo)


def test_index_bytes_v3_short_and_malformed(env):
    torch, hip = env
    elems = [b"abcdefghij"] * 20000
    wire = _wire(elems)
    buf = torch.from_numpy(wire.copy()).cuda()
    st, found, _, _ = _index(torch, hip, buf, wire.size, 20001)
    assert st == 1 and found == 20000
    bad = wire.copy()
    bad[14 * 10000: 14 * 10000 + 4] = np.frombuffer((1 << 30).to_bytes(4, "little"), np.uint8)
    buf = torch.from_numpy(bad).cuda()
    st, _, _, _ = _index(torch, hip, buf, bad.size, 20000)
    assert st == -1


@pytest.mark.parametrize("n,width", [(5000, 24), (70000, 7), (3, 40000)])
def test_pack_bytes_strided_fixed_width(env, n, width):
    """K2 over a numpy 'S' array's buffer (no host join): lengths are the
    element lengths with trailing NULs stripped (numpy / serialize_byte_tensor)."""
    torch, hip = env
    rng = np.random.default_rng(n)
    raw = rng.integers(97, 123, (n, width), dtype=np.uint8)
    cut = rng.integers(0, width + 1, n)
    raw[np.arange(width)[None, :] >= cut[:, None]] = 0
    arr = raw.view("S%d" % width).reshape(n)
    lens = np.char.str_len(arr).astype(np.uint32)
    d_data = torch.from_numpy(raw.reshape(-1).copy()).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32).copy()).cuda()
    total = int(lens.sum()) + 4 * n
    out = torch.zeros(total + 32, device="cuda", dtype=torch.uint8)
    ws = torch.empty(hip.pack_bytes_workspace(n), device="cuda", dtype=torch.uint8)
    hip.pack_bytes_strided(d_data.data_ptr(), width, d_lens.data_ptr(), n, out.data_ptr() + 3, ws.data_ptr(),
                           _stream(torch))
    from tritonclient.utils import serialize_byte_tensor

    ref = serialize_byte_tensor(arr).item()
    got = out.cpu().numpy()
    assert got[3:3 + total].tobytes() == ref and not got[:3].any() and not got[3 + total:].any()


def test_index_bytes_detects_malformed(env):
    torch, hip = env
    buf = torch.tensor([5, 0, 0, 0, 1, 2], device="cuda", dtype=torch.uint8)
    offs = torch.empty(4, device="cuda", dtype=torch.int64)
    lns = torch.empty(4, device="cuda", dtype=torch.int32)
    status = torch.zeros(4, device="cuda", dtype=torch.int32)
    hip.index_bytes(buf.data_ptr(), 6, 1, offs.data_ptr(), lns.data_ptr(), status.data_ptr(), _stream(torch))
    assert int(status[0]) == -1


@pytest.mark.parametrize("scaling", ["NONE", "INCEPTION", "VGG"])
@pytest.mark.parametrize("fmt", ["NCHW", "NHWC"])
@pytest.mark.parametrize("dtype", ["FP32", "FP16"])
def test_image_preprocess_on_device_matches_host(env, scaling, fmt, dtype):
    """K6 as image_client's device preprocessing vs the numpy path it replaces."""
    from triton_client_amd.utils.image import preprocess, preprocess_batch_device, resize_bilinear

    rng = np.random.default_rng(3)
    raw = [rng.integers(0, 256, size=(37 + 5 * i, 41, 3), dtype=np.uint8) for i in range(3)]
    npdt = np.float32 if dtype == "FP32" else np.float16
    want = np.stack([preprocess(r, 3, 32, 48, scaling, fmt, npdt) for r in raw])
    got = preprocess_batch_device([resize_bilinear(r, 32, 48) for r in raw], scaling, fmt, dtype)
    assert got.shape == want.shape and got.dtype == want.dtype
    tol = 1e-5 if dtype == "FP32" else 2e-3
    np.testing.assert_allclose(got.astype(np.float32), want.astype(np.float32), rtol=tol, atol=tol * 128)


def _pack_ref(payload, lens):
    """Wire-format reference built with numpy (u32 LE length || bytes)."""
    n = lens.size
    out = np.empty(int(lens.sum()) + 4 * n, dtype=np.uint8)
    o_starts = np.concatenate([[0], np.cumsum(lens.astype(np.int64) + 4)[:-1]])
    pre = lens.astype("<u4").view(np.uint8).reshape(n, 4)
    for k in range(4):
        out[o_starts + k] = pre[:, k]
    # payload bytes: output index = payload index + 4 * (element index + 1)
    elem = np.repeat(np.arange(n), lens.astype(np.int64))
    out[np.arange(payload.size) + 4 * (elem + 1)] = payload
    return out


@pytest.mark.parametrize("doff,ooff", [(0, 0), (5, 3), (1, 14)])
def test_pack_bytes_dword_assembly_misaligned(env, doff, ooff):
    """K2 dword-assembled emit (pk_emit_packed): empty, short, tile-spanning
    and block-spanning elements, with data / output pointers off 16-B."""
    torch, hip = env
    rng = np.random.default_rng(doff * 7 + ooff)
    n = 60000
    lens = rng.integers(0, 40, n).astype(np.uint32)
    lens[rng.integers(0, n, 40)] = 0
    lens[rng.integers(0, n, 12)] = rng.integers(8000, 70000, 12).astype(np.uint32)  # > one tile / part
    lens[1024:2048] = 0  # a whole block of prefixes only
    payload = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
    d_payload = torch.zeros(payload.size + 32, device="cuda", dtype=torch.uint8)
    d_payload[doff:doff + payload.size] = torch.from_numpy(payload).cuda()
    d_lens = torch.from_numpy(lens.view(np.int32).copy()).cuda()
    total = int(lens.sum()) + 4 * n
    out = torch.zeros(total + 64, device="cuda", dtype=torch.uint8)
    ws = torch.empty(hip.pack_bytes_workspace(n), device="cuda", dtype=torch.uint8)
    hip.pack_bytes(d_payload.data_ptr() + doff, d_lens.data_ptr(), n, out.data_ptr() + ooff, ws.data_ptr(),
                   _stream(torch))
    got = out.cpu().numpy()
    ref = _pack_ref(payload, lens)
    assert np.array_equal(got[ooff:ooff + total], ref)
    assert not got[:ooff].any() and not got[ooff + total:].any()


_BIG_PATH_SCRIPT = r"""
import numpy as np, torch, sys
sys.path.insert(0, %r)
from triton_client_amd.ops import hip
from tests.test_kernels_gpu import _pack_ref
rng = np.random.default_rng(3)
n = 5000
lens = rng.integers(0, 60, n).astype(np.uint32)
lens[7] = 100000
payload = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
total = int(lens.sum()) + 4 * n
out = torch.zeros(total + 16, device="cuda", dtype=torch.uint8)
ws = torch.empty(hip.pack_bytes_workspace(n), device="cuda", dtype=torch.uint8)
d_p = torch.from_numpy(payload).cuda()
d_l = torch.from_numpy(lens.view(np.int32).copy()).cuda()
hip.pack_bytes(d_p.data_ptr(), d_l.data_ptr(), n, out.data_ptr() + 1, ws.data_ptr(),
               torch.cuda.current_stream().cuda_stream)
got = out.cpu().numpy()
assert np.array_equal(got[1:1 + total], _pack_ref(payload, lens)), "mismatch"
assert got[0] == 0 and not got[1 + total:].any()
print("BIG_OK")
"""


@pytest.mark.timeout(300)
def test_pack_bytes_big_block_path():
    """Blocks whose output passes the 32-bit local-offset limit take a 64-bit
    byte path; TCAMD_PK_BIG_LIM=0 forces every block onto it (own process,
    the limit is read once)."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, TCAMD_PK_BIG_LIM="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _BIG_PATH_SCRIPT % repo], capture_output=True, text=True,
                       timeout=280, env=env, cwd=repo)
    assert r.returncode == 0 and "BIG_OK" in r.stdout, r.stderr[-3000:]
