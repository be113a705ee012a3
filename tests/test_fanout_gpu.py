"""Fan-out of the synthetic batch on a real GPU.

* the Python X2 star (``parallel/fanout._p2p_star``): two processes on GPU 0
  in one gloo group, rank 0 fills its HIP shm region with K1 and copies it
  into rank 1's region through rank 1's IPC handle; every byte of both
  replicas is compared;
* the native perf_analyzer lanes (``csrc/cpp/perf/multigpu.cc``): two lanes on
  GPU 0 (``--devices 0,0``), the batch made once by K1 on lane 0 and copied
  into lane 1's region by the p2p star and by the host path, verified byte for
  byte before any request, then per-GPU rows against the GPU server.
"""

import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

_CHILD = r"""
import hashlib, json, os, sys
sys.path.insert(0, os.environ["REPO"])
import torch, torch.distributed as dist
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"],
                        rank=int(os.environ["RANK"]), world_size=2)
torch.cuda.set_device(0)
from tritonclient.utils import hip_shared_memory as hipshm
from triton_client_amd.parallel import fanout
rank = dist.get_rank()
n = 8 * 3 * 224 * 224  # densenet bs8 fp32: 4.8 MB
h = hipshm.create_shared_memory_region("fan%d" % rank, n * 4, 0)
m = fanout.fill_and_fanout(h, "FP32", n, seed=77, mode="normal", method="p2p")
import numpy as np
arr = hipshm.get_contents_as_numpy(h, np.float32, [n])
digests = [None, None]
dist.all_gather_object(digests, hashlib.sha256(arr.tobytes()).hexdigest())
if rank == 0:
    # the root's bytes are K1's: regenerate them independently
    ref = torch.empty(n, device="cuda", dtype=torch.float32)
    from triton_client_amd.ops import hip
    hip.synth_fill(ref.data_ptr(), n, "FP32", hip.SYNTH_NORMAL, 0.0, 1.0, seed=77)
    torch.cuda.synchronize()
    same_k1 = bool((ref.cpu().numpy() == arr).all())
    json.dump({"method": m, "digests": digests, "k1": same_k1, "finite": bool(abs(arr).max() < 100)},
              open(os.environ["OUT"], "w"))
dist.barrier()
hipshm.destroy_shared_memory_region(h)
dist.destroy_process_group()
"""


def test_python_p2p_star_two_processes_one_gpu(tmp_path):
    from triton_client_amd.perf.harness import free_port

    port = str(free_port())
    out = tmp_path / "fan.json"
    env = dict(os.environ, REPO=REPO, PORT=port, OUT=str(out), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-c", _CHILD], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(2)]
    logs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o + e)
        assert p.returncode == 0, "\n".join(logs)[-3000:]
    res = json.load(open(out))
    assert res["method"] == "p2p"
    assert res["digests"][0] == res["digests"][1], res
    assert res["k1"] and res["finite"]


@pytest.mark.parametrize("fan", ["p2p", "host"])
def test_native_perf_lanes_fanout_on_one_gpu(gpu_server, tmp_path, fan):
    from triton_client_amd.perf import native

    j = tmp_path / "lanes.json"
    r = subprocess.run([native.BIN_PATH, "-m", "densenet_onnx", "-b", "8", "-i", "grpc", "-u", gpu_server.grpc_url,
                        "--devices", "0,0", "--fanout", fan, "--shared-memory", "hip",
                        "--output-shared-memory-size", str(8 * 1000 * 4), "--concurrency-range", "8", "-p", "400",
                        "-r", "4", "-s", "30", "--json-report", str(j)],
                       capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "fanned out by %s" % fan in r.stdout and "replicas verified" in r.stdout, r.stdout[-1500:]
    assert "inputs filled on device by K1" in r.stdout
    rep = json.load(open(j))
    pt = rep["points"][0]
    assert rep["gpus"] == 2 and pt["errors"] == 0
    assert [g["load"] for g in pt["per_gpu"]] == [4, 4]
    assert all(g["throughput"] > 0 for g in pt["per_gpu"])
    print(fan, "lanes:", [round(g["throughput"]) for g in pt["per_gpu"]], "total", round(pt["throughput"]))


def test_native_rccl_fanout_reports_clean_error_or_runs(gpu_server):
    """RCCL needs distinct devices per communicator rank: on a 1-GPU box
    `--devices 0,0 --fanout rccl` must fail cleanly (no hang, a named
    error); with >= 2 GPUs it must run and verify its replicas."""
    import torch

    from triton_client_amd.perf import native

    ngpu = torch.cuda.device_count()
    devs = "0,1" if ngpu >= 2 else "0,0"
    r = subprocess.run([native.BIN_PATH, "-m", "densenet_onnx", "-b", "8", "-i", "grpc", "-u", gpu_server.grpc_url,
                        "--devices", devs, "--fanout", "rccl", "--shared-memory", "hip",
                        "--output-shared-memory-size", str(8 * 1000 * 4), "--concurrency-range", "4", "-p", "300",
                        "-r", "3", "-s", "50"], capture_output=True, text=True, timeout=90)
    if ngpu >= 2:
        assert r.returncode == 0 and "fanned out by rccl" in r.stdout and "replicas verified" in r.stdout
    else:
        assert r.returncode == 1 and "ncclCommInitAll" in r.stderr, r.stdout[-800:] + r.stderr[-800:]


def test_native_perf_bytes_packed_on_device_by_k2(gpu_server, tmp_path):
    """HIP-shm BYTES synthetic data: K1 draws the characters and K2 packs the
    length-prefixed stream on the device (nothing built on the host); the
    server parses every element of every request."""
    from triton_client_amd.perf import native

    j = tmp_path / "bytes.json"
    r = subprocess.run([native.BIN_PATH, "-m", "simple_identity", "-i", "grpc", "-u", gpu_server.grpc_url,
                        "--shape", "INPUT0:64", "--string-length", "24", "--shared-memory", "hip",
                        "--output-shared-memory-size", str(64 * 28), "--concurrency-range", "2", "-p", "300",
                        "-r", "3", "-s", "60", "--json-report", str(j)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "K2 BYTES packing" in r.stdout, r.stdout[-1500:]
    pt = json.load(open(j))["points"][0]
    assert pt["errors"] == 0 and pt["request_count"] > 0
