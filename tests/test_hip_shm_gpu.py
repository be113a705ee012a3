"""HIP shared memory (the cuda_shared_memory replacement) and the zero-copy
inference path through the GPU bench server.  Mirrors reference
src/python/library/tests/test_cuda_shared_memory.py:37-168 plus the
simple_*_cudashm_client examples."""

import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hipshm():
    import torch

    torch.cuda.set_device(0)
    from tritonclient.utils import hip_shared_memory

    return hip_shared_memory


def test_create_set_get_destroy(hipshm):
    h = hipshm.create_shared_memory_region("r0", 256, 0)
    assert "r0" in hipshm.allocated_shared_memory_regions()
    a = np.arange(16, dtype=np.int32)
    b = np.arange(16, 32, dtype=np.int32)
    hipshm.set_shared_memory_region(h, [a, b])
    np.testing.assert_array_equal(hipshm.get_contents_as_numpy(h, np.int32, [16]), a)
    np.testing.assert_array_equal(hipshm.get_contents_as_numpy(h, np.int32, [16], offset=64), b)
    raw = hipshm.get_raw_handle(h)
    import base64

    assert len(base64.b64decode(raw)) == 64
    hipshm.destroy_shared_memory_region(h)
    assert "r0" not in hipshm.allocated_shared_memory_regions()


def test_bytes_roundtrip(hipshm):
    from tritonclient.utils import serialize_byte_tensor

    data = np.array([b"hello", b"", b"mi355x" * 10], dtype=np.object_)
    ser = serialize_byte_tensor(data)
    h = hipshm.create_shared_memory_region("rb", len(ser.item()), 0)
    hipshm.set_shared_memory_region(h, [ser])
    out = hipshm.get_contents_as_numpy(h, np.object_, [3])
    assert list(out) == list(data)
    hipshm.destroy_shared_memory_region(h)


def test_unserialized_bytes_packed_by_k2_and_indexed_by_k3(hipshm):
    """set_shared_memory_region with a raw BYTES tensor serialises it on the
    device (K2) into the region; get_contents_as_numpy indexes it on the device
    (K3, parallel block walk at this size).  Bytes must equal the host codec's."""
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(3)
    data = np.array([bytes(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8)) for _ in range(20000)],
                    dtype=np.object_).reshape(100, 200)
    ser = serialize_byte_tensor(data).item()
    head = np.arange(8, dtype=np.int32)
    h = hipshm.create_shared_memory_region("rk2", 32 + len(ser) + 256, 0)
    hipshm.set_shared_memory_region(h, [head, data], serialize_bytes=True)  # int32 head, then K2 at offset 32
    raw = hipshm.get_contents_as_numpy(h, np.uint8, [32 + len(ser)])
    assert raw[32:].tobytes() == ser
    for path in ("device", "auto"):  # K3 / the host walk ("auto" always walks on the host)
        out = hipshm.get_contents_as_numpy(h, np.object_, [100, 200], offset=32, bytes_path=path)
        assert out.shape == (100, 200) and list(out.ravel()) == list(data.ravel())
    # asking for more elements than the region holds is an error, not garbage
    small = hipshm.create_shared_memory_region("rk3", len(serialize_byte_tensor(data[:1]).item()), 0)
    hipshm.set_shared_memory_region(small, [data[:1]], serialize_bytes=True)
    for path in ("device", "auto"):
        with pytest.raises(hipshm.CudaSharedMemoryException):
            hipshm.get_contents_as_numpy(small, np.object_, [400], bytes_path=path)
    hipshm.destroy_shared_memory_region(small)
    hipshm.destroy_shared_memory_region(h)


def test_bytes_set_semantics_match_reference_and_system_shm(hipshm):
    """without serialize_bytes an object array is the output of
    serialize_byte_tensor (copied as-is, whatever its size) and an np.bytes_
    array is copied raw (size * itemsize), exactly like the system-shm module
    and the reference; serialize_bytes=True serialises both on the device
    (fixed-width np.bytes_ straight from its buffer, no host join)."""
    from tritonclient.utils import serialize_byte_tensor
    from tritonclient.utils import shared_memory as sysshm

    one = np.array([b"abc"], dtype=np.object_)  # a 1-element UNserialised tensor
    fixed = np.array([b"ab", b"xyz\x00", b""], dtype="S5")
    h = hipshm.create_shared_memory_region("sem", 64, 0)
    key = "/sem_%d" % os.getpid()
    sh = sysshm.create_shared_memory_region("sem_sys", key, 64)
    try:
        for mod, handle in ((hipshm, h), (sysshm, sh)):
            mod.set_shared_memory_region(handle, [one, fixed])
            raw = mod.get_contents_as_numpy(handle, np.uint8, [3 + 15])
            assert raw.tobytes() == b"abc" + fixed.tobytes()
            mod.set_shared_memory_region(handle, [one, fixed], serialize_bytes=True)
            want = serialize_byte_tensor(one).item() + serialize_byte_tensor(fixed).item()
            raw = mod.get_contents_as_numpy(handle, np.uint8, [len(want)])
            assert raw.tobytes() == want
    finally:
        hipshm.destroy_shared_memory_region(h)
        sysshm.destroy_shared_memory_region(sh)
    # a large fixed-width array through the strided K2
    rng = np.random.default_rng(5)
    big = np.array([bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(0, 17, 30000)],
                   dtype="S16")
    want = serialize_byte_tensor(big).item()
    h = hipshm.create_shared_memory_region("sem_big", len(want), 0)
    hipshm.set_shared_memory_region(h, [big], serialize_bytes=True)
    assert hipshm.get_contents_as_numpy(h, np.uint8, [len(want)]).tobytes() == want
    back = hipshm.get_contents_as_numpy(h, np.object_, [30000])
    assert list(back) == list(big)
    hipshm.destroy_shared_memory_region(h)


@pytest.mark.parametrize("dt", ["BF16", "FP16", "FP8_E4M3", "FP8_E5M2"])
def test_device_dtype_conversion_on_set_and_get(hipshm, dt):
    """K4/K5 on the HIP-shm set/get paths: float32 in -> narrow region bytes
    wire-exact with the host codecs (BF16 = serialize_bf16_tensor truncation),
    and narrow region -> float32 out widened on the device."""
    from tritonclient.utils import deserialize_bf16_tensor, serialize_bf16_tensor
    from tritonclient import utils as tu

    rng = np.random.default_rng(11)
    x = (rng.standard_normal(100003) * 50).astype(np.float32)
    size = {"BF16": 2, "FP16": 2}.get(dt, 1)
    h = hipshm.create_shared_memory_region("cvt_" + dt, 16 + x.size * size + 16, 0)
    try:
        for off in (0, 16, 3):  # aligned and unaligned region offsets
            hipshm.set_shared_memory_region(h, [x], offset=off, datatype=dt)
            raw = hipshm.get_contents_as_numpy(h, np.uint8, [x.size * size], offset=off)
            if dt == "BF16":
                want = np.frombuffer(serialize_bf16_tensor(x).item(), np.uint8)
                back_ref = deserialize_bf16_tensor(want.tobytes())
            elif dt == "FP16":
                want = x.astype(np.float16).view(np.uint8)
                back_ref = x.astype(np.float16).astype(np.float32)
            else:  # saturating RNE, the host reference of v_cvt_pk_fp8_f32
                want = np.frombuffer(tu.serialize_fp8_tensor(x, dt).item(), np.uint8)
                back_ref = tu.deserialize_fp8_tensor(want.tobytes(), dt)
            np.testing.assert_array_equal(raw, np.asarray(want, np.uint8))
            back = hipshm.get_contents_as_numpy(h, np.float32, [x.size], offset=off, region_datatype=dt)
            np.testing.assert_array_equal(back, back_ref)
    finally:
        hipshm.destroy_shared_memory_region(h)


def test_dlpack_roundtrip_torch(hipshm):
    import torch

    h = hipshm.create_shared_memory_region("rd", 4 * 64, 0)
    src = torch.arange(32, dtype=torch.float32, device="cuda")
    host = torch.arange(32, 64, dtype=torch.float32)
    hipshm.set_shared_memory_region_from_dlpack(h, [src, host])
    view = torch.from_dlpack(hipshm.as_shared_memory_tensor(h, "FP32", [64]))
    assert view.device.type == "cuda"
    assert torch.equal(view.cpu(), torch.arange(64, dtype=torch.float32))
    view[0] = 42.0  # zero-copy: writes land in the region
    torch.cuda.synchronize()
    assert hipshm.get_contents_as_numpy(h, np.float32, [1])[0] == 42.0
    del view
    hipshm.destroy_shared_memory_region(h)


def test_device_side_synthetic_and_bf16(hipshm):
    h = hipshm.create_shared_memory_region("rs", 4096, 0)
    hipshm.fill_synthetic_data(h, "FP32", 1024, "constant", 1.5)
    assert (hipshm.get_contents_as_numpy(h, np.float32, [1024]) == 1.5).all()
    x = np.linspace(-3, 3, 512).astype(np.float32)
    hipshm.set_shared_memory_region_from_fp32(h, x, "BF16")
    from tritonclient.utils import deserialize_bf16_tensor, serialize_bf16_tensor

    raw = hipshm.get_contents_as_numpy(h, np.uint8, [1024])
    assert raw.tobytes() == serialize_bf16_tensor(x).item()
    np.testing.assert_array_equal(deserialize_bf16_tensor(raw.tobytes()), deserialize_bf16_tensor(serialize_bf16_tensor(x).item()))
    hipshm.destroy_shared_memory_region(h)




def test_simple_cudashm_grpc(gpu_server, hipshm):
    """Port of simple_grpc_cudashm_client.py: INT32 add/sub via device shm."""
    import tritonclient.grpc as grpcclient

    c = grpcclient.InferenceServerClient(gpu_server.grpc_url)
    c.unregister_cuda_shared_memory()
    a = np.arange(16, dtype=np.int32).reshape(1, 16)
    b = np.ones((1, 16), dtype=np.int32)
    hin = hipshm.create_shared_memory_region("in_data", 128, 0)
    hout = hipshm.create_shared_memory_region("out_data", 128, 0)
    hipshm.set_shared_memory_region(hin, [a, b])
    c.register_cuda_shared_memory("in_data", hipshm.get_raw_handle(hin), 0, 128)
    c.register_cuda_shared_memory("out_data", hipshm.get_raw_handle(hout), 0, 128)
    st = c.get_cuda_shared_memory_status(as_json=True)
    assert set(st["regions"]) == {"in_data", "out_data"}
    ins = [grpcclient.InferInput("INPUT0", [1, 16], "INT32"), grpcclient.InferInput("INPUT1", [1, 16], "INT32")]
    ins[0].set_shared_memory("in_data", 64)
    ins[1].set_shared_memory("in_data", 64, offset=64)
    outs = [grpcclient.InferRequestedOutput("OUTPUT0"), grpcclient.InferRequestedOutput("OUTPUT1")]
    outs[0].set_shared_memory("out_data", 64)
    outs[1].set_shared_memory("out_data", 64, offset=64)
    c.infer("simple", ins, outputs=outs)
    np.testing.assert_array_equal(hipshm.get_contents_as_numpy(hout, np.int32, [1, 16]), a + b)
    np.testing.assert_array_equal(hipshm.get_contents_as_numpy(hout, np.int32, [1, 16], offset=64), a - b)
    c.unregister_cuda_shared_memory()
    hipshm.destroy_shared_memory_region(hin)
    hipshm.destroy_shared_memory_region(hout)
    c.close()


def _reference_logits(x, dtype_name="float32"):
    import torch

    from triton_client_amd.models import densenet

    dtype = getattr(torch, dtype_name)
    m = densenet.build(device="cuda", dtype=dtype)
    xt = torch.from_numpy(x).cuda().to(dtype).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        return m(xt).float().cpu().numpy()




def test_densenet_zero_copy_matches_fp32_reference(gpu_server, hipshm):
    """densenet_onnx bs=2 through HIP shm (K6 gather in, K7 scatter out)
    against an fp32 torch reference of the same random-init weights."""
    import tritonclient.grpc as grpcclient
    import tritonclient.http as httpclient

    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 3, 224, 224)).astype(np.float32)
    ref = _reference_logits(x)
    hin = hipshm.create_shared_memory_region("d_in", x.nbytes, 0)
    hout = hipshm.create_shared_memory_region("d_out", 2 * 1000 * 4, 0)
    hipshm.set_shared_memory_region(hin, [x])
    g = grpcclient.InferenceServerClient(gpu_server.grpc_url)
    g.register_cuda_shared_memory("d_in", hipshm.get_raw_handle(hin), 0, x.nbytes)
    g.register_cuda_shared_memory("d_out", hipshm.get_raw_handle(hout), 0, 8000)
    inp = grpcclient.InferInput("data_0", [2, 3, 224, 224], "FP32")
    inp.set_shared_memory("d_in", x.nbytes)
    out = grpcclient.InferRequestedOutput("fc6_1")
    out.set_shared_memory("d_out", 8000)
    r = g.infer("densenet_onnx", [inp], outputs=[out])
    assert r.get_output("fc6_1").parameters["shared_memory_region"].string_param == "d_out"
    got = hipshm.get_contents_as_numpy(hout, np.float32, [2, 1000])
    # the served engine is the fp32-parity one (models/densenet_fp32.py): the
    # served path (pointer table, HIP graph, K7 scatter, native front end)
    # must land within fp32-class error of the fp32 module of the same weights
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < 1e-3, rel
    # same request over HTTP with host (binary) input and output
    h = httpclient.InferenceServerClient(gpu_server.http_url)
    hi = httpclient.InferInput("data_0", [2, 3, 224, 224], "FP32")
    hi.set_data_from_numpy(x)
    res = h.infer("densenet_onnx", [hi], outputs=[httpclient.InferRequestedOutput("fc6_1")])
    host = res.as_numpy("fc6_1")
    # host-staged and zero-copy paths run the same graph: same logits
    assert np.linalg.norm(host - got) / np.linalg.norm(got) < 1e-5
    # classification extension
    res = h.infer("densenet_onnx", [hi], outputs=[httpclient.InferRequestedOutput("fc6_1", class_count=3)])
    top = res.as_numpy("fc6_1")
    assert top.shape == (2, 3)
    assert int(top[0, 0].decode().split(":")[1]) == int(got[0].argmax())
    g.unregister_cuda_shared_memory()
    hipshm.destroy_shared_memory_region(hin)
    hipshm.destroy_shared_memory_region(hout)
    g.close()
    h.close()


@pytest.mark.parametrize("dt", ["BF16", "FP16", "FP32"])
def test_infer_input_from_device_tensor(hipshm, dt):
    """InferInput.set_data_from_dlpack with a torch ROCm FP32 tensor: the
    request bytes (HTTP binary_data / gRPC raw_input_contents) must equal the
    numpy path's for the same values (BF16 by K4 truncation on the GPU)."""
    import torch

    import tritonclient.grpc as grpcclient
    import tritonclient.http as httpclient

    x = torch.randn(4, 1000, device="cuda") * 3
    xn = x.cpu().numpy()
    for mod in (httpclient, grpcclient):
        a = mod.InferInput("x", [4, 1000], dt)
        a.set_data_from_dlpack(x[:, :] if dt != "FP16" else x)
        b = mod.InferInput("x", [4, 1000], dt)
        b.set_data_from_numpy(xn.astype(np.float16) if dt == "FP16" else xn)
        get = (lambda i: i._get_binary_data()) if mod is httpclient else (lambda i: i._get_content())
        assert get(a) == get(b)
    # a BF16 device tensor goes out as-is (no conversion)
    xb = x.to(torch.bfloat16)
    c = httpclient.InferInput("x", [4, 1000], "BF16").set_data_from_dlpack(xb)
    assert c._get_binary_data() == xb.view(torch.int16).cpu().numpy().tobytes()


@pytest.mark.parametrize("n,maxlen", [(16, 30), (4000, 40), (5000, 20), (12, 9000)])
@pytest.mark.parametrize("path", ["host", "device", "auto"])
def test_bytes_host_and_device_paths_agree(hipshm, n, maxlen, path):
    """Small BYTES tensors go through the host codec (one copy of the span),
    large ones through K2 / K3; both directions, both paths, byte-identical
    region contents and round trips (the crossover: tools/bytes_crossover.py)."""
    from tritonclient.utils import serialize_byte_tensor

    rng = np.random.default_rng(n + maxlen)
    data = np.array([bytes(rng.integers(0, 256, int(rng.integers(0, maxlen)), dtype=np.uint8)) for _ in range(n)],
                    dtype=np.object_)
    want = serialize_byte_tensor(data).item()
    h = hipshm.create_shared_memory_region("bp_%s_%d" % (path, n), len(want) + 64, 0)
    try:
        hipshm.set_shared_memory_region(h, [data], serialize_bytes=True, bytes_path=path)
        assert hipshm.get_contents_as_numpy(h, np.uint8, [len(want)]).tobytes() == want
        back = hipshm.get_contents_as_numpy(h, np.object_, [n], bytes_path=path)
        assert list(back) == list(data)
        with pytest.raises(hipshm.CudaSharedMemoryException):
            hipshm.get_contents_as_numpy(h, np.object_, [n + 17], bytes_path=path)
    finally:
        hipshm.destroy_shared_memory_region(h)
