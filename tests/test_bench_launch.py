"""bench.py's launch contract on CPU: ``--gpus N`` without WORLD_SIZE spawns
N ranks (torch.distributed.run as a child process), every rank runs the full
pipeline (server, fan-out of the synthetic batch, native load generator,
timed windows) and rank 0 prints ONE JSON line aggregated over the ranks.
``--cpu`` swaps the GPU pieces for the CPU frontend_sink model, system shm
and gloo, so this runs without a GPU."""

import json
import os
import subprocess
import sys

import pytest

from triton_client_amd.parallel import placement
from triton_client_amd.perf import native

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not native.available(), reason="libperfanalyzer.so not built")


def _bench(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--cpu", "--warmup", "1",
                        "--concurrency", "4", "--bs1-concurrency", "4", *args],
                       capture_output=True, text=True, timeout=timeout, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_spawns_ranks_and_aggregates(gpus):
    res, err = _bench("--gpus", str(gpus), "--steps", "5")
    assert res["n_gpus"] == gpus
    assert res["world_size_reported_by_process_group"] == gpus
    assert res["config"]["parallelism"] == "dp%d" % gpus
    assert res["steps"] == 5 and res["warmup"] == 1
    assert res["value"] > 0 and res["p99_latency_us"] >= res["p50_latency_us"] > 0
    assert len(res["window_infer_per_sec_rank0"]) == 5
    assert len(res["window_p99_latency_us_rank0"]) == 5
    assert all(p99 >= p50 > 0 for p50, p99 in zip(res["window_p50_latency_us_rank0"],
                                                   res["window_p99_latency_us_rank0"]))
    assert len(res["placement"]) == gpus and all(p["applied"] is (gpus > 1) for p in res["placement"])
    assert res["bs1"]["infer_per_sec"] > 0
    assert res["bs1"]["breakdown_rank0"]["avg_rows_per_batch"] >= 1
    if gpus > 1:
        assert "spawning %d ranks" % gpus in err
        assert "fanned out by gloo" in res["data"]


def test_bench_bs1_over_two_client_lanes():
    """--lanes 2 / --bs1-lanes 2: the headline and bs=1 concurrencies split over
    two client connections / worker threads (disjoint concurrency slots); the
    JSON says so and the breakdowns still read the server's statistics."""
    res, _ = _bench("--steps", "2", "--bs1-lanes", "2", "--lanes", "2")
    assert res["bs1"]["client_lanes"] == 2 and res["bs1"]["concurrency"] == 4
    assert res["config"]["client_lanes"] == 2 and res["value"] > 0 and len(res["window_infer_per_sec_rank0"]) == 2
    assert res["bs1"]["infer_per_sec"] > 0 and res["bs1"]["p99_latency_us"] >= res["bs1"]["p50_latency_us"] > 0
    assert res["bs1"]["breakdown_rank0"]["avg_rows_per_batch"] >= 1


@pytest.mark.slow
def test_bench_eight_ranks_on_cpu():
    """The driver's N=8 launch, rehearsed on the CPU (verdict r4 #6): 8 ranks,
    8 servers and 8 native load generators on one host, world size 8 in the
    JSON, disjoint per-rank port stripes, gloo agreement on the aggregate, and
    every rank pinned to its own CPU slice (no KFD topology here: the even
    split of the allowed CPUs)."""
    res, err = _bench("--gpus", "8", "--steps", "3", "--window", "4", timeout=900)
    assert res["n_gpus"] == 8 and res["world_size_reported_by_process_group"] == 8
    assert res["config"]["parallelism"] == "dp8" and res["value"] > 0
    pl = res["placement"]
    assert len(pl) == 8 and all(p["applied"] for p in pl), pl
    assert len({p["grpc_port"] for p in pl}) == 8
    cpus = [set(placement.parse_cpulist(p["cpulist"])) for p in pl]
    if len(os.sched_getaffinity(0)) >= 8:
        assert all(len(a & b) == 0 for i, a in enumerate(cpus) for b in cpus[i + 1:]), pl
    assert "fanned out by gloo" in res["data"]


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--cpu", "--gpus", "2"],
                       capture_output=True, text=True, timeout=60, cwd=REPO, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_bench_bert_sweep_two_ranks():
    """Config 4's path (bench.py --model bert_large): three INT32 input regions
    fanned out from rank 0, a concurrency sweep per rank, one aggregated JSON
    line with every point (CPU: the bert_sink shape model)."""
    res, err = _bench("--gpus", "2", "--steps", "3", "--model", "bert_large", "--sweep", "1,4")
    assert res["n_gpus"] == 2 and res["config"]["model"] == "bert_sink"
    assert res["config"]["seq_len"] == 384 and res["config"]["parallelism"] == "dp2"
    assert [p["concurrency"] for p in res["sweep"]] == [1, 4]
    assert all(p["infer_per_sec"] > 0 and p["p99_latency_us"] >= p["p50_latency_us"] > 0 for p in res["sweep"])
    assert res["value"] == res["sweep"][-1]["infer_per_sec"]
    assert "fanned out by gloo" in res["data"]
    assert "bert c4" in err


def test_merge_lanes_puts_lanes_on_one_clock():
    """Lanes started at different times: their completion times are shifted to
    the earliest lane's clock before the windows sort them (round-5 advisor
    finding: mixed time bases skewed the per-window statistics)."""
    import numpy as np

    import bench

    # lane 0 ran 0..1.0 s, lane 1 started 0.5 s later and ran 1.0 s
    lane0 = (np.array([5, 6], dtype=np.uint64), np.array([400_000_000, 1_000_000_000], dtype=np.uint64), 1.0)
    lane1 = (np.array([7, 8], dtype=np.uint64), np.array([100_000_000, 1_000_000_000], dtype=np.uint64), 1.0)
    lat, end, span = bench.merge_lanes([lane0, lane1], [2_000_000_000, 2_500_000_000])
    assert list(lat) == [5, 6, 7, 8]
    assert list(end) == [400_000_000, 1_000_000_000, 600_000_000, 1_500_000_000]
    assert abs(span - 1.5) < 1e-9


def test_batcher_preference_per_point():
    """The preferred batch rows bench.py sets per load point: one full group
    per instance (bs=1: concurrency / instances; bert: from --bert-preferred-from
    rows per instance, capped at the model's max batch)."""
    import bench

    assert bench.bs1_preferred_rows("auto", 64, 2) == [32]
    assert bench.bs1_preferred_rows("auto", 63, 2) is None
    assert bench.bs1_preferred_rows("none", 64, 2) is None
    assert bench.bs1_preferred_rows("16,32", 64, 2) == [16, 32]
    got = [bench.bert_point_preferred("auto", c, 2, 2) for c in (1, 4, 16, 64, 256)]
    assert got == [None, 2, 8, 32, 64]
    assert bench.bert_point_preferred("auto", 4, 2, 8) is None
    assert bench.bert_point_preferred("none", 64, 2, 2) is None
