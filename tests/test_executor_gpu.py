"""GPU test of the native batch executor (csrc/runtime/graph_exec.hip): the
C++ per-batch dispatch tcserve runs for densenet_onnx (pointer table H2D,
bucket graph replay, K7 output scatter, host D2H) must give the same logits
as the engine called directly, for mixed device / host inputs and outputs."""

import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from triton_client_amd.server.gpu_models import DensenetOnnx

    m = DensenetOnnx(engine="fp32", max_batch_size=8)
    m.instance_count = 2
    m.load()
    yield m
    m.unload()


def _batch(refs_in, refs_out, rows):
    from triton_client_amd.server.native_frontend import TcBatch, TcRef

    n = len(rows)
    ins = (TcRef * n)(*[TcRef(*r) for r in refs_in])
    outs = (TcRef * n)(*[TcRef(*r) for r in refs_out])
    nrows = (ctypes.c_int32 * n)(*rows)
    timing = (ctypes.c_uint64 * 3)()
    b = TcBatch(n, sum(rows), nrows, 1, ins, 1, outs, timing)
    return b, (ins, outs, nrows, timing)


def test_executor_bound_and_exported(model):
    fn, user = model.native_executor()
    from triton_client_amd.ops import hip

    assert fn == ctypes.cast(hip.lib().tcamd_pgx_execute, ctypes.c_void_p).value
    assert user


@pytest.mark.parametrize("instance", [0, 1])
def test_executor_mixed_device_and_host_rows(model, instance):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(3 + instance)
    x = torch.randn(5, 3, 224, 224, generator=g)
    xd = x[:3].to(dev).contiguous()           # request 0: 3 rows in device memory (HIP shm)
    xh = np.ascontiguousarray(x[3:].numpy())  # request 1: 2 rows in host memory (in-band)
    out_d = torch.full((3, 1000), float("nan"), device=dev)
    out_h = np.full((2, 1000), np.nan, dtype=np.float32)
    torch.cuda.synchronize()
    b, keep = _batch([(1, 0, xd.data_ptr(), xd.numel() * 4), (0, 0, xh.ctypes.data, xh.nbytes)],
                     [(1, 0, out_d.data_ptr(), out_d.numel() * 4), (0, 0, out_h.ctypes.data, out_h.nbytes)], [3, 2])
    before = model.executor_stats()["batches"]
    model._pgx.execute(instance, ctypes.addressof(b))
    got = np.concatenate([out_d.cpu().numpy(), out_h])
    assert np.isfinite(got).all()
    # reference: the same engine called eagerly on the 5 rows (the executor ran
    # the bucket-8 graph: split-K plans differ with M, so fp32-parity, not bitwise)
    with torch.no_grad():
        ref = model._slots[instance]["net"](x.to(dev)).cpu().numpy()
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel < 1e-4, rel
    t = keep[3]
    assert t[1] > 0, "graph time missing"
    st = model.executor_stats()
    assert st["batches"] == before + 1 and st["wait_ns"] > 0


def test_native_executor_matches_python_path(model, monkeypatch):
    """TCAMD_NATIVE_EXEC=0 loads the model without the C++ executor (tcserve
    then calls the Python execute_native per batch); both give the same logits
    for the same batch."""
    from triton_client_amd.server.gpu_models import DensenetOnnx

    monkeypatch.setenv("TCAMD_NATIVE_EXEC", "0")
    py = DensenetOnnx(engine="fp32", max_batch_size=8)
    py.instance_count = 1
    py.load()
    try:
        assert py.native_executor() is None and py.executor_stats() is None
        assert model.native_executor() is not None
        dev = torch.device("cuda", 0)
        x = torch.randn(3, 3, 224, 224, generator=torch.Generator().manual_seed(11)).to(dev).contiguous()
        outs = []
        for m, run in ((model, lambda b: model._pgx.execute(0, ctypes.addressof(b))),
                       (py, lambda b: py.execute_native(0, b))):
            out = torch.full((3, 1000), float("nan"), device=dev)
            torch.cuda.synchronize()
            b, keep = _batch([(1, 0, x.data_ptr(), x.numel() * 4)], [(1, 0, out.data_ptr(), out.numel() * 4)], [3])
            run(b)
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy())
        assert np.isfinite(outs[1]).all()
        rel = np.linalg.norm(outs[0] - outs[1]) / np.linalg.norm(outs[1])
        assert rel < 2e-5, rel  # same engine and bucket graph; float-atomic ordering noise only
    finally:
        py.unload()


def test_executor_rejects_oversized_batch(model):
    x = torch.zeros(9, 3, 224, 224, device="cuda")
    out = torch.zeros(9, 1000, device="cuda")
    b, keep = _batch([(1, 0, x.data_ptr(), x.numel() * 4)], [(1, 0, out.data_ptr(), out.numel() * 4)], [9])
    with pytest.raises(RuntimeError, match="exceeds the largest bucket"):
        model._pgx.execute(0, ctypes.addressof(b))


def test_executor_rejects_short_input_buffer(model):
    x = torch.zeros(1, 3, 224, 224, device="cuda")
    out = torch.zeros(2, 1000, device="cuda")
    b, keep = _batch([(1, 0, x.data_ptr(), x.numel() * 4)], [(1, 0, out.data_ptr(), out.numel() * 4)], [2])
    with pytest.raises(RuntimeError, match="too small"):
        model._pgx.execute(0, ctypes.addressof(b))
