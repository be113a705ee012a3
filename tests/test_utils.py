"""tritonclient.utils codecs (reference tritonclient/utils/__init__.py:36-348)."""

import struct

import numpy as np
import pytest

from tritonclient import utils


def _ref_serialize_bytes(arr):
    # the reference's element loop, written independently
    out = b""
    for x in arr.reshape(-1, order="C"):
        s = x if isinstance(x, bytes) else str(x).encode("utf-8")
        out += struct.pack("<I", len(s)) + s
    return out


def test_dtype_maps_roundtrip():
    for dt in ["BOOL", "INT8", "INT16", "INT32", "INT64", "UINT8", "UINT16", "UINT32", "UINT64",
               "FP16", "FP32", "FP64", "BYTES"]:
        assert utils.np_to_triton_dtype(utils.triton_to_np_dtype(dt)) == dt
    assert utils.triton_to_np_dtype("BF16") == np.float32
    assert utils.np_to_triton_dtype(np.dtype("S5")) == "BYTES"
    assert utils.np_to_triton_dtype(np.complex64) is None
    assert utils.triton_to_np_dtype("NOPE") is None


@pytest.mark.parametrize("arr", [
    np.array([[b"a", "bc"], [b"", "é"]], dtype=np.object_),
    np.array([1, 2.5, "x"], dtype=np.object_),
    np.array([b"abc", b"de"], dtype=np.bytes_),
])
def test_serialize_byte_tensor_matches_reference_layout(arr):
    s = utils.serialize_byte_tensor(arr)
    assert s.dtype == np.object_ and s.ndim == 0
    assert s.item() == _ref_serialize_bytes(arr)
    back = utils.deserialize_bytes_tensor(s.item())
    assert back.dtype == np.object_
    assert [bytes(x) for x in back] == [x if isinstance(x, bytes) else str(x).encode() for x in arr.reshape(-1)]


def test_serialize_empty_and_invalid():
    assert utils.serialize_byte_tensor(np.array([], dtype=np.object_)).size == 0
    with pytest.raises(utils.InferenceServerException):
        utils.serialize_byte_tensor(np.array([1, 2], dtype=np.int32))
    with pytest.raises(utils.InferenceServerException):
        utils.deserialize_bytes_tensor(b"\x05\x00\x00\x00ab")


def test_large_bytes_native_path():
    arr = np.array([("x" * (i % 17)).encode() for i in range(20000)], dtype=np.object_)
    s = utils.serialize_byte_tensor(arr).item()
    assert s == _ref_serialize_bytes(arr)
    back = utils.deserialize_bytes_tensor(s)
    assert list(back) == list(arr)


def test_bf16_truncation_wire_compat():
    x = np.array([1.0, -2.5, 3.14159265, 1e-40, np.inf, -0.0], dtype=np.float32)
    s = utils.serialize_bf16_tensor(x).item()
    assert s == b"".join(struct.pack("<f", v)[2:4] for v in x)
    back = utils.deserialize_bf16_tensor(s)
    assert back.dtype == np.float32
    np.testing.assert_array_equal(back.view(np.uint32), x.view(np.uint32) & 0xFFFF0000)
    with pytest.raises(utils.InferenceServerException):
        utils.serialize_bf16_tensor(x.astype(np.float64))


def test_serialized_byte_size():
    assert utils.serialized_byte_size(np.array([b"ab", b"cde"], dtype=np.object_)) == 5
    with pytest.raises(utils.InferenceServerException):
        utils.serialized_byte_size(np.array([1]))


@pytest.mark.parametrize("fmt", ["FP8_E4M3", "FP8_E5M2"])
def test_fp8_codec_matches_torch_in_range(fmt):
    import torch

    rng = np.random.default_rng(0)
    scale = 100.0 if fmt == "FP8_E4M3" else 5000.0
    x = (rng.standard_normal(10000) * scale).astype(np.float32)
    maxv = 448.0 if fmt == "FP8_E4M3" else 57344.0
    x = x[np.abs(x) < maxv]
    codes = np.frombuffer(utils.serialize_fp8_tensor(x, fmt).item(), dtype=np.uint8)
    tdt = torch.float8_e4m3fn if fmt == "FP8_E4M3" else torch.float8_e5m2
    ref = torch.from_numpy(x).to(tdt).view(torch.uint8).numpy()
    np.testing.assert_array_equal(codes, ref)
    dec = utils.deserialize_fp8_tensor(codes.tobytes(), fmt)
    np.testing.assert_array_equal(dec, torch.from_numpy(ref).view(tdt).float().numpy())


def test_fp8_saturates():
    x = np.array([1e6, -1e6, np.nan], dtype=np.float32)
    dec = utils.deserialize_fp8_tensor(utils.serialize_fp8_tensor(x).item())
    assert dec[0] == 448.0 and dec[1] == -448.0 and np.isnan(dec[2])


def test_exception_str_and_accessors():
    e = utils.InferenceServerException("boom", status="400", debug_details="dbg")
    assert str(e) == "[400] boom"
    assert e.message() == "boom" and e.status() == "400" and e.debug_details() == "dbg"
    with pytest.raises(utils.InferenceServerException):
        utils.raise_error("x")


def test_dlpack_host_view_zero_copy():
    import torch

    from tritonclient.utils import SharedMemoryTensor, _dlpack

    a = np.arange(24, dtype=np.float32)
    t = torch.from_dlpack(SharedMemoryTensor("FP32", [2, 3, 4], a.ctypes.data, 0, a.nbytes, -1))
    assert t.shape == (2, 3, 4)
    a[5] = -1
    assert float(t.reshape(-1)[5]) == -1.0
    c = _dlpack.consume(torch.ones(3, 5, dtype=torch.int64))
    assert c.shape == [3, 5] and c.datatype == "INT64" and c.byte_size() == 120 and not c.is_device()
    c.release()
    nc = _dlpack.consume(torch.ones(4, 4).t())
    assert not nc.is_contiguous()
    nc.release()


@pytest.mark.parametrize("lens", [[0] * 50, [3, 0, 70000, 5], [20] * 5000, [40000, 40000, 1], [1] * 3])
def test_hip_shm_host_bytes_walk_grows_its_prefix(lens):
    """The HIP-shm BYTES host path (small tensors) walks the length-prefixed
    chain over a prefix copied D2H in growing chunks; on CPU the 'device' is a
    numpy buffer (a fake memcpy_d2h), so every growth case runs here: empty
    elements, an element longer than the first chunk, exactly n elements."""
    from tritonclient.utils import hip_shared_memory as hipshm
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(len(lens))
    data = np.array([bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in lens], dtype=np.object_)
    ser = np.frombuffer(serialize_byte_tensor(data).item(), dtype=np.uint8)
    dev = np.zeros(ser.size + 300, dtype=np.uint8)  # a region larger than the stream (zeros = empty elements)
    dev[:ser.size] = ser
    copies = []

    class FakeHip:
        @staticmethod
        def memcpy_d2h(dst, src, nbytes, d):
            copies.append(nbytes)
            dst[:nbytes] = dev[src:src + nbytes]

    host, offs, lens_out = hipshm._index_bytes_host(FakeHip, 0, dev.size, len(lens), 0)
    got = [bytes(host[o:o + n]) for o, n in zip(offs.tolist(), lens_out.tolist())]
    assert got == list(data)
    assert sum(copies) <= dev.size  # each byte copied at most once
    # more elements than the stream holds: the zero tail parses as empty
    # elements up to the region end, then it is an error
    with pytest.raises(hipshm.CudaSharedMemoryException):
        hipshm._index_bytes_host(FakeHip, 0, dev.size, len(lens) + 76, 0)
    # an element that runs past the region end
    bad = dev[:ser.size].copy()
    bad[:4] = np.frombuffer(np.uint32(10 ** 6).tobytes(), np.uint8)

    class BadHip:
        @staticmethod
        def memcpy_d2h(dst, src, nbytes, d):
            dst[:nbytes] = bad[src:src + nbytes]

    with pytest.raises(hipshm.CudaSharedMemoryException, match="past the end"):
        hipshm._index_bytes_host(BadHip, 0, bad.size, len(lens), 0)
