"""The served batch at the headline shape, with distinct data per request
(verdict r3 #3).

(a) The capacity-256 serving engine (DensenetOnnx max_batch_size 256, one
    instance) through the C++ batch executor (csrc/runtime/graph_exec.hip:
    pointer table -> bucket graph replay -> K7 output scatter) at 64, 121, 128
    and 256 rows made of distinct 8-row (and one ragged) requests.  Every
    row's logits are checked against the fp32 module on THAT row's image
    (a row mix-up gives a different image's logits, rel-L2 ~1), and two rows
    against fp64.
(b) tcserve + the native executor exactly as bench.py configures them (2
    instances, preferred 128, 2 ms queue delay, idle-aware dispatch,
    pipelined and staggered dispatch at their defaults) driven by the native
    load generator at concurrency 48, every slot with its OWN HIP-shm input
    region (K1 Philox, a different seed each) and its own output region.
    After the run every output region must hold the fp32 module's logits of
    its own input, and server stats must show batches of >= 100 rows.
"""

import ctypes
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

DEV = "cuda"
IMG = 3 * 224 * 224


def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def ref_module():
    """The fp32 module the served engine was built from (same seed, same
    calibration and folding as densenet_fp32.build)."""
    _need_gpu()
    from triton_client_amd.models import densenet

    m = densenet.DenseNet121()
    densenet.init_weights(m, 0)
    densenet.calibrate_bn(m, device="cpu")
    densenet.fold_for_inference(m)
    m.eval()
    return m


def _row_rel(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    return np.linalg.norm(got - ref, axis=-1) / np.linalg.norm(ref, axis=-1)


@pytest.fixture(scope="module")
def served256():
    _need_gpu()
    from triton_client_amd.server.gpu_models import DensenetOnnx

    m = DensenetOnnx(engine="fp32", max_batch_size=256)
    m.instance_count = 1
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


@pytest.mark.parametrize("rows", [64, 121, 128, 256])
def test_capacity256_engine_distinct_requests(served256, ref_module, rows):
    """Rows from distinct requests, each request its own device buffers: the
    executor's pointer table and scatter must keep every row with its image."""
    dev = torch.device(DEV, 0)
    sizes = [8] * (rows // 8) + ([rows % 8] if rows % 8 else [])
    g = torch.Generator(device=dev).manual_seed(1000 + rows)
    x = torch.randn(rows, 3, 224, 224, device=dev, generator=g)
    reqs = [t.clone() for t in torch.split(x, sizes)]
    outs = [torch.full((s, 1000), float("nan"), device=dev) for s in sizes]
    torch.cuda.synchronize()
    b, keep = _batch([(1, 0, r.data_ptr(), r.numel() * 4) for r in reqs],
                     [(1, 0, o.data_ptr(), o.numel() * 4) for o in outs], sizes)
    assert served256._pgx is not None, "native executor missing"
    served256._pgx.execute(0, ctypes.addressof(b))
    got = torch.cat(outs).cpu().numpy()
    assert np.isfinite(got).all()
    with torch.no_grad():
        ref = torch.cat([ref_module.to(dev).float()(c) for c in torch.split(x, 64)]).cpu().numpy()
    rel = _row_rel(got, ref)
    print("rows %d: per-row rel-L2 vs fp32 module max %.3g mean %.3g" % (rows, rel.max(), rel.mean()))
    assert rel.max() < 1e-3, (int(rel.argmax()), float(rel.max()))
    # two rows against fp64 (first and last: different requests, different halves of the batch)
    pick = [0, rows - 1]
    with torch.no_grad():
        r64 = ref_module.to("cpu").double()(x[pick].cpu().double()).numpy()
        ref_module.float()
    rel64 = _row_rel(got[pick], r64)
    print("rows %d: rel-L2 vs fp64 %s" % (rows, rel64))
    assert rel64.max() < 1e-4
    assert keep[3][1] > 0


def test_bench_configured_server_keeps_48_distinct_requests_apart(ref_module, tmp_path):
    """(b): bench.py's server configuration, concurrency 48, 48 distinct input
    and output regions; every output checked against the fp32 module."""
    _need_gpu()
    import tritonclient.grpc as grpcclient
    from tritonclient.utils import hip_shared_memory as hipshm
    from triton_client_amd.perf.harness import ServerProcess
    from triton_client_amd.perf.native import PerfSession

    conc, bs = 48, 8
    log = os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.getcwd()), "gpurun_out", "served_batch_server.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    srv = ServerProcess(device=0, models="densenet_onnx", log_path=log,
                        extra_args=["--instance-count", "2", "--max-queue-delay-us", "2000", "--idle-dispatch", "on",
                                    "--engine", "fp32", "--preferred-batch-sizes", "128"])
    regions, client = [], None
    try:
        srv.wait_ready(timeout=900, model="densenet_onnx")
        client = grpcclient.InferenceServerClient(srv.grpc_url)
        in_names, out_names, rin, rout = [], [], [], []
        for i in range(conc):
            r = hipshm.create_shared_memory_region("sb_in_%d" % i, bs * IMG * 4, 0)
            regions.append(r)
            rin.append(r)
            hipshm.fill_synthetic_data(r, "FP32", bs * IMG, "normal", 0.0, 1.0, 5000 + i)
            client.register_cuda_shared_memory("sb_in_%d" % i, hipshm.get_raw_handle(r), 0, bs * IMG * 4)
            in_names.append("sb_in_%d" % i)
            o = hipshm.create_shared_memory_region("sb_out_%d" % i, bs * 1000 * 4, 0)
            regions.append(o)
            rout.append(o)
            client.register_cuda_shared_memory("sb_out_%d" % i, hipshm.get_raw_handle(o), 0, bs * 1000 * 4)
            out_names.append("sb_out_%d" % i)
        args = ["-m", "densenet_onnx", "-i", "grpc", "-u", srv.grpc_url, "-b", bs, "--shared-memory", "hip",
                "--device", 0, "--shared-memory-input", "data_0=" + ",".join(in_names),
                "--shared-memory-output", "fc6_1=" + ",".join(out_names), "--concurrency-range", conc]
        with PerfSession([str(a) for a in args]) as s:
            assert "caller regions pinned to slots" in s.describe()
            s.run_fixed(conc, 4 * conc)  # warm-up
            st0 = s.server_stats()
            lat, _ = s.run_fixed(conc, 16 * conc)
            st1 = s.server_stats()
        assert len(lat) == 16 * conc
        reqs = st1["success_count"] - st0["success_count"]
        execs = st1["execution_count"] - st0["execution_count"]
        rows = st1["inference_count"] - st0["inference_count"]
        assert reqs == 16 * conc, (reqs, st0, st1)
        print("served: %d requests in %d batches, %.1f rows per batch" % (reqs, execs, rows / max(execs, 1)))
        stats = client.get_inference_statistics("densenet_onnx", as_json=True)
        big = sum(int(b.get("compute_infer", {}).get("count", 0)) for m in stats["model_stats"]
                  for b in m.get("batch_stats", []) if int(b["batch_size"]) >= 100)
        assert big > 0, "no batch of >= 100 rows formed"
        dev = torch.device(DEV, 0)
        worst = 0.0
        for i in range(conc):
            x = torch.from_dlpack(hipshm.as_shared_memory_tensor(rin[i], "FP32", [bs, 3, 224, 224])).clone()
            got = hipshm.get_contents_as_numpy(rout[i], np.float32, [bs, 1000])
            with torch.no_grad():
                ref = ref_module.to(dev).float()(x.to(dev)).cpu().numpy()
            rel = _row_rel(got, ref)
            worst = max(worst, float(rel.max()))
            assert rel.max() < 1e-3, (i, rel)
        print("48 distinct requests: worst per-row rel-L2 vs fp32 module %.3g" % worst)
    finally:
        if client is not None:
            try:
                client.unregister_cuda_shared_memory()
            except Exception:
                pass
            client.close()
        for r in regions:
            try:
                hipshm.destroy_shared_memory_region(r)
            except Exception:
                pass
        srv.stop()
