"""One-GPU rehearsal of the driver's multi-GPU bench launch.

``bench.py --gpus 2 --rehearse`` goes through the same path as the 8-GPU
scaling run -- torch.distributed.run child, one server per rank on HIP shm,
rank 0's K1 batch fanned out to every rank's region, replica verification,
MAX-over-ranks timing, all-gathered latency arrays, the X1/X2 fan-out timing
-- except that both ranks sit on GPU 0 over gloo (RCCL cannot put two ranks
on one device), so the fan-out is the xGMI-less p2p star (same-device IPC)
and host staging.  Not a scaling number; a launch/aggregation check.
"""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_bench_two_ranks_rehearsed_on_one_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--rehearse", "--steps", "2",
           "--warmup", "1", "--window", "4", "--no-bf16", "--instance-count", "2", "--max-batch-size", "32",
           "--preferred", "32", "--bs1-concurrency", "8"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=850, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["world_size_reported_by_process_group"] == 2
    assert res["config"]["shared_memory"] == "hip" and res["config"]["parallelism"] == "dp2"
    assert "rehearsal" in res
    fan = res["fanout"]
    assert fan["replicas_verified"] is True and fan["method"] == "p2p"
    assert fan["fanout_us"] > 0
    assert set(fan["timings"]) == {"p2p", "host"}
    assert all("us" in v for v in fan["timings"].values()), fan
    # X2 is a pull: each destination timed its own copy; both ranks share GPU 0
    assert set(fan["timings"]["p2p"]["per_peer"]) == {"1"}
    assert fan["timings"]["p2p"]["per_peer"]["1"]["us"] > 0
    assert fan["timings"]["p2p"]["peer_access"] is None
    assert res["value"] > 0 and res["p99_latency_us"] > 0
    # every p99-constrained probe says how its rows split into batches
    for p in res["p99_constrained"]["points"][1:]:
        assert sum(p["breakdown_rank0"]["batch_rows_histogram"].values()) > 0


@pytest.mark.timeout(900)
def test_bert_sweep_two_ranks_rehearsed_on_one_gpu():
    """The config-4 sweep through the multi-rank launch: both ranks' bert_large
    servers on GPU 0, the token-id region fanned out and X1/X2-timed (per-peer
    pull time), the sweep aggregated over ranks."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--rehearse", "--model", "bert_large",
           "--sweep", "1,8", "--steps", "2", "--warmup", "1", "--bert-instance-count", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=850, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and "rehearsal" in res and res["config"]["model"] == "bert_large"
    assert [p["concurrency"] for p in res["sweep"]] == [1, 8]
    assert all(p["infer_per_sec"] > 0 for p in res["sweep"])
    fan = res["fanout"]
    assert set(fan["timings"]) == {"p2p", "host"} and not fan["errors"]
    assert fan["timings"]["p2p"]["per_peer"]["1"]["us"] > 0
