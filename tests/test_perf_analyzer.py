"""Native perf_analyzer (csrc/cpp/perf) against the CPU test server.

Covers the perf_analyzer-equivalent of SURVEY.md Appendix D: CLI parsing,
concurrency / request-rate / fixed-count loads, sync / async / streaming
issue paths, system shared memory, sequence models, BYTES inputs, stability
windows and the CSV / JSON reports.  Everything here runs on CPU.
"""

import csv
import json
import os
import subprocess

import pytest

from triton_client_amd.perf import native

pytestmark = pytest.mark.skipif(not native.available(), reason="csrc/cpp not built")


def _pa(args, timeout=120):
    return subprocess.run([native.BIN_PATH] + [str(a) for a in args], capture_output=True, text=True,
                          timeout=timeout)


def test_help_and_bad_flags():
    r = _pa(["-h"])
    assert r.returncode == 0 and "--concurrency-range" in r.stdout
    r = _pa(["-m", "simple", "--bogus-flag"])
    assert r.returncode == 1 and "unknown" in r.stderr
    r = _pa(["-b", "2"])
    assert r.returncode == 1 and "-m <model> is required" in r.stderr
    r = _pa(["-m", "x", "--streaming"])  # streaming needs grpc
    assert r.returncode == 1 and "grpc" in r.stderr
    # a comma list with no region in it is an error, not an empty list (front() on it was UB)
    for flag in ("--shared-memory-input", "--shared-memory-output"):
        for val in ("IN=,", "IN=,,,"):
            r = _pa(["-m", "x", flag, val])
            assert r.returncode == 1 and "no region for IN" in r.stderr, (flag, val, r.stderr)


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_concurrency_sweep_csv(cpu_server, tmp_path, proto):
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    f = tmp_path / "out.csv"
    j = tmp_path / "out.json"
    r = _pa(["-m", "simple", "-i", proto, "-u", url, "-p", "300", "--concurrency-range", "1:3:2", "-f", f,
             "--json-report", j, "-r", "4"])
    assert r.returncode == 0, r.stderr
    assert "Request concurrency: 1" in r.stdout and "Request concurrency: 3" in r.stdout
    assert "Inferences/Second vs. Client Average Batch Latency" in r.stdout
    rows = list(csv.DictReader(open(f)))
    assert [row["Concurrency"] for row in rows] == ["1", "3"]
    assert all(float(row["Inferences/Second"]) > 0 for row in rows)
    assert all(float(row["p99 latency"]) >= float(row["p50 latency"]) > 0 for row in rows)
    rep = json.load(open(j))
    assert rep["model"] == "simple" and len(rep["points"]) == 2
    assert rep["points"][0]["server"]["success_count"] > 0


def test_sweep_checkpoint_and_resume(cpu_server, tmp_path):
    """The JSON report is a checkpoint: --resume skips completed points, keeps
    them in the reports, and refuses a checkpoint of a different sweep."""
    j = tmp_path / "sweep.json"
    base = ["-m", "simple", "-i", "grpc", "-u", cpu_server.grpc_url, "-p", "200", "-r", "3", "--json-report", j]
    r = _pa(base + ["--concurrency-range", "1:2:1"])
    assert r.returncode == 0, r.stderr
    first = json.load(open(j))
    assert [p["load"] for p in first["points"]] == [1, 2]
    # a sweep that died after concurrency 1
    partial = dict(first, points=first["points"][:1])
    json.dump(partial, open(j, "w"))
    f = tmp_path / "sweep.csv"
    r = _pa(base + ["--concurrency-range", "1:3:1", "--resume", "-f", f])
    assert r.returncode == 0, r.stderr
    assert "Resumed from" in r.stdout and "concurrency 1 (already measured)" in r.stdout
    assert r.stdout.count("Request concurrency: 1") == 1  # reprinted from the checkpoint, not re-measured
    assert "Request concurrency: 2" in r.stdout and "Request concurrency: 3" in r.stdout
    done = json.load(open(j))
    assert [p["load"] for p in done["points"]] == [1, 2, 3]
    assert done["points"][0]["throughput"] == pytest.approx(first["points"][0]["throughput"], rel=1e-3)
    assert [row["Concurrency"] for row in csv.DictReader(open(f))] == ["1", "2", "3"]
    # a checkpoint from another model is refused
    r = _pa(["-m", "simple_string", "-i", "grpc", "-u", cpu_server.grpc_url, "-p", "200", "--json-report", j,
             "--resume"])
    assert r.returncode == 1 and "different sweep" in r.stderr


def test_roctx_ranges_enabled_without_profiler(cpu_server):
    """TC_ROCTX=1 loads roctx and pushes ranges (perf windows, client Infer);
    without a profiler attached they are no-ops and the run is unchanged."""
    env = dict(os.environ, TC_ROCTX="1")
    r = subprocess.run([native.BIN_PATH, "-m", "simple", "-i", "grpc", "-u", cpu_server.grpc_url, "-p", "200", "-r",
                        "3", "--sync"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    assert "Request concurrency: 1" in r.stdout


def _fake_amdgpu(root, busy, watts, vram):
    dev = root / "card{}".format(len(list(root.iterdir()))) / "device"
    (dev / "hwmon" / "hwmon7").mkdir(parents=True)
    (dev / "vendor").write_text("0x1002\n")
    (dev / "gpu_busy_percent").write_text("%d\n" % busy)
    (dev / "mem_info_vram_used").write_text("%d\n" % vram)
    (dev / "hwmon" / "hwmon7" / "power1_average").write_text("%d\n" % (watts * 1000000))


def test_collect_metrics_from_amdgpu_sysfs(cpu_server, tmp_path):
    """--collect-metrics samples the amdgpu sysfs counters of --device (a fake
    tree here; /sys/class/drm on the GPU box) into stdout, CSV and JSON."""
    root = tmp_path / "drm"
    root.mkdir()
    _fake_amdgpu(root, 10, 200, 1 << 30)
    _fake_amdgpu(root, 73, 615, 3 << 30)
    (root / "card1-DP-1").mkdir()  # connectors are skipped
    f, j = tmp_path / "m.csv", tmp_path / "m.json"
    r = _pa(["-m", "simple", "-i", "grpc", "-u", cpu_server.grpc_url, "-p", "200", "-r", "3", "--collect-metrics",
             "--metrics-interval", "20", "--metrics-sysfs-root", root, "--device", "1", "-f", f, "--json-report", j])
    assert r.returncode == 0, r.stderr
    assert "GPU: utilization 73.0%, power 615.0 W, max memory used 3072 MiB" in r.stdout
    row = next(csv.DictReader(open(f)))
    assert float(row["Avg GPU Utilization"]) == pytest.approx(0.73)
    assert float(row["Avg GPU Power Usage"]) == pytest.approx(615.0)
    assert float(row["Max GPU Memory Usage"]) == 3 << 30
    assert json.load(open(j))["points"][0]["gpu"] == {"util_pct": 73.0, "power_w": 615.0, "mem_mib": 3072.0}


def test_system_shm_sync_count_windows(cpu_server):
    r = _pa(["-m", "simple", "-u", cpu_server.http_url, "--sync", "--shared-memory", "system",
             "--measurement-mode", "count_windows", "--measurement-request-count", "60",
             "--concurrency-range", "2"])
    assert r.returncode == 0, r.stderr
    assert "system shared memory" in r.stdout and "synchronous" in r.stdout
    assert "Failed requests" not in r.stdout


def test_streaming_and_sequences(cpu_server):
    r = _pa(["-m", "simple_sequence", "-i", "grpc", "-u", cpu_server.grpc_url, "--streaming", "-p", "300",
             "--sequence-length", "4", "--concurrency-range", "2", "-r", "4"])
    assert r.returncode == 0, r.stderr
    assert "streaming" in r.stdout and "Sequence model: 4 requests per sequence" in r.stdout
    assert "Failed requests" not in r.stdout


def test_request_rate_poisson(cpu_server):
    r = _pa(["-m", "simple", "-u", cpu_server.http_url, "--request-rate-range", "200",
             "--request-distribution", "poisson", "-p", "400", "-r", "3"])
    assert r.returncode == 0, r.stderr
    thr = float(r.stdout.split("Throughput: ")[1].split()[0])
    assert 100 < thr < 320  # open loop: throughput follows the offered rate


def test_request_intervals_file(cpu_server, tmp_path):
    f = tmp_path / "iv.txt"
    f.write_text("\n".join(["2000"] * 10))  # 2 ms apart -> ~500 req/s
    r = _pa(["-m", "simple", "-u", cpu_server.http_url, "--request-intervals", f, "-p", "1000", "-r", "3", "-v"])
    assert r.returncode == 0, r.stderr
    thr = float(r.stdout.split("Throughput: ")[1].split()[0])
    # the schedule is honoured: ~500/s, and well below what the same server
    # does unthrottled right now (a CPU-starved xdist host slows both)
    u = _pa(["-m", "simple", "-u", cpu_server.http_url, "--concurrency-range", "16", "-p", "1000", "-r", "3"])
    unthrottled = float(u.stdout.split("Throughput: ")[1].split()[0])
    assert 250 < thr, r.stdout + r.stderr
    if unthrottled > 1200:
        assert thr < 0.75 * unthrottled, (thr, unthrottled, r.stdout[-1500:] + r.stderr[-1500:])


def test_bytes_and_json_data(cpu_server, tmp_path):
    r = _pa(["-m", "simple_string", "-u", cpu_server.http_url, "--string-data", "12", "-p", "300", "-r", "3"])
    assert r.returncode == 0, r.stderr
    d = tmp_path / "data.json"
    d.write_text(json.dumps({"data": [{"INPUT0": list(range(16)), "INPUT1": [1] * 16}]}))
    r = _pa(["-m", "simple", "-u", cpu_server.http_url, "--input-data", d, "-p", "300", "-r", "3"])
    assert r.returncode == 0, r.stderr
    assert "json:" in r.stdout


def test_batch_limit_and_unknown_model(cpu_server):
    r = _pa(["-m", "simple", "-u", cpu_server.http_url, "-b", "4"])  # simple has max_batch_size 8? no: 0
    assert ("does not support batching" in r.stderr) or ("exceeds max_batch_size" in r.stderr) or r.returncode == 0
    r = _pa(["-m", "no_such_model", "-u", cpu_server.http_url])
    assert r.returncode == 1 and "no_such_model" in r.stderr


def test_native_session_fixed_run(cpu_server):
    with native.PerfSession(["-m", "simple", "-i", "grpc", "-u", cpu_server.grpc_url, "--shared-memory", "system",
                             "--concurrency-range", "4"]) as s:
        assert "system shared memory" in s.describe()
        st0 = s.server_stats()
        lat, el = s.run_fixed(4, 200)
        assert len(lat) == 200 and (lat > 0).all() and el > 0
        st1 = s.server_stats()
        assert st1["success_count"] - st0["success_count"] >= 200
        lat2, _ = s.run_fixed(2, 50)  # reuse the session at a different concurrency
        assert len(lat2) == 50
        p = s.profile(2)
        assert p["throughput"] > 0 and p["p99_us"] >= p["p50_us"] > 0


def test_native_session_errors():
    with pytest.raises(native.PerfError):
        native.PerfSession(["-m", "simple", "-u", "127.0.0.1:1", "--concurrency-range", "1"])
    with pytest.raises(native.PerfError):
        native.PerfSession(["--concurrency-range", "1"])


@pytest.mark.parametrize("shm", ["system", "none"])
def test_multi_lane_host_fanout_per_gpu_rows(cpu_server, tmp_path, shm):
    """--gpus 2 on CPU: two lanes (clients, worker threads, regions), the
    synthetic batch made once and host-fanned into lane 1's region (verified
    byte for byte), per-GPU rows + the aggregate in stdout / CSV / JSON."""
    f, j = tmp_path / "mg.csv", tmp_path / "mg.json"
    url = cpu_server.grpc_url
    r = _pa(["-m", "simple", "-i", "grpc", "-u", "%s,%s" % (url, url), "--gpus", "2", "--shared-memory", shm,
             "--concurrency-range", "4:6:2", "-p", "300", "-r", "4", "-s", "50", "-f", f, "--json-report", j,
             "--fanout", "host"])
    assert r.returncode == 0, r.stderr + r.stdout
    assert "2 GPUs [0,1]" in r.stdout and "load split over GPUs" in r.stdout
    if shm == "system":
        assert "fanned out by host" in r.stdout and "replicas verified" in r.stdout
    assert r.stdout.count("Per-GPU (2 lanes") == 2
    rows = list(csv.DictReader(open(f)))
    assert [x["GPU"] for x in rows] == ["all", "0", "1", "all", "0", "1"]
    for k in (0, 3):
        agg, g0, g1 = rows[k:k + 3]
        assert abs(float(agg["Inferences/Second"]) - float(g0["Inferences/Second"]) - float(g1["Inferences/Second"])) \
            < 0.02 * float(agg["Inferences/Second"]) + 1
    rep = json.load(open(j))
    assert rep["gpus"] == 2
    for p, conc in zip(rep["points"], (4, 6)):
        assert p["load"] == conc
        assert [g["gpu"] for g in p["per_gpu"]] == [0, 1]
        assert sum(g["load"] for g in p["per_gpu"]) == conc
        assert sum(g["request_count"] for g in p["per_gpu"]) == p["request_count"]


def test_multi_lane_full_load_per_gpu_and_url_count(cpu_server):
    url = cpu_server.http_url
    r = _pa(["-m", "simple", "-u", url, "--gpus", "3", "--load-per-gpu", "--concurrency-range", "2", "-p", "250",
             "-r", "3", "-s", "60"])
    assert r.returncode == 0, r.stderr
    assert "full load per GPU" in r.stdout
    assert r.stdout.count("concurrency 2,") == 3  # every lane runs the full concurrency
    r = _pa(["-m", "simple", "-u", "%s,%s" % (url, url), "--gpus", "3"])
    assert r.returncode == 1 and "2 URLs for 3 GPUs" in r.stderr


def test_json_data_multiple_entries_cycle(cpu_server, tmp_path):
    d = tmp_path / "steps.json"
    d.write_text(json.dumps({"data": [{"INPUT0": [i] * 16, "INPUT1": [1] * 16} for i in range(3)]}))
    r = _pa(["-m", "simple", "-u", cpu_server.http_url, "--input-data", d, "-p", "200", "-r", "3", "-s", "60"])
    assert r.returncode == 0, r.stderr
    assert "3 entries, cycled per request" in r.stdout


def _counters(srv):
    nf = srv.server.native_frontend
    return nf.counters() if nf is not None else None


def test_tensor_format_json_reaches_server_as_json(cpu_server):
    """--input-tensor-format / --output-tensor-format json: every request
    carries inline JSON "data" (the reference's ConvertBinaryInputToJSON path,
    http_client.cc:580-678) and asks for JSON outputs; the server counts both."""
    ws = cpu_server.server.wire_stats
    before_in, before_out = ws["json_input_tensors"], ws["json_output_tensors"]
    r = _pa(["-m", "simple", "-u", cpu_server.http_url, "--input-tensor-format", "json", "--output-tensor-format",
             "json", "--measurement-mode", "count_windows", "--measurement-request-count", "50", "-r", "3"])
    assert r.returncode == 0, r.stderr
    assert "tensors in/out as json/json" in r.stdout
    n_in, n_out = ws["json_input_tensors"] - before_in, ws["json_output_tensors"] - before_out
    assert n_in >= 2 * 50 and n_out >= 2 * 50, (n_in, n_out)  # simple: 2 inputs, 2 outputs per request
    r = _pa(["-m", "simple", "-u", cpu_server.grpc_url, "-i", "grpc", "--input-tensor-format", "json"])
    assert r.returncode == 1 and "need -i http" in r.stderr


@pytest.mark.parametrize("proto,algo", [("http", "gzip"), ("http", "deflate"), ("grpc", "gzip"), ("grpc", "deflate")])
def test_compression_reaches_server(cpu_server, proto, algo):
    """--grpc-compression-algorithm / --compression-algorithm: compressed
    request bodies (and, over HTTP, compressed responses) served on tcserve's
    native path; its counters verify what arrived."""
    c0 = _counters(cpu_server)
    if c0 is None:
        pytest.skip("native front end not built")
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    flag = "--grpc-compression-algorithm" if proto == "grpc" else "--compression-algorithm"
    r = _pa(["-m", "add_sub_batched", "-u", url, "-i", proto, flag, algo, "--measurement-mode", "count_windows",
             "--measurement-request-count", "40", "-r", "3"])
    assert r.returncode == 0, r.stderr
    assert "%s compression" % algo in r.stdout
    c1 = _counters(cpu_server)
    assert c1["inflated_requests"] - c0["inflated_requests"] >= 120
    if proto == "http":
        assert c1["compressed_responses"] - c0["compressed_responses"] >= 120
    assert c1["native_requests"] - c0["native_requests"] >= 120
    r = _pa(["-m", "simple", "--compression-algorithm", "brotli"])
    assert r.returncode == 1 and "compression" in r.stderr


@pytest.mark.parametrize("proto", ["http", "grpc"])
def test_request_parameters_reach_server(cpu_server, proto):
    """--request-parameter name:value:type (repeatable) arrives typed on every
    request (reference common.h:155-159, 230)."""
    ws = cpu_server.server.wire_stats
    url = cpu_server.http_url if proto == "http" else cpu_server.grpc_url
    args = ["-m", "simple", "-u", url, "-i", proto, "--request-parameter", "tenant:a:b:string",
            "--request-parameter", "max_tokens:42:int", "--request-parameter", "stream:true:bool",
            "--request-parameter", "temperature:0.5:double", "--measurement-mode", "count_windows",
            "--measurement-request-count", "30", "-r", "3"]
    keys = ["param:tenant:str:a:b", "param:max_tokens:int:42", "param:stream:bool:True", "param:temperature:float:0.5"]
    before = {k: ws[k] for k in keys}
    r = _pa(args)
    assert r.returncode == 0, r.stderr
    assert "4 request parameter(s)" in r.stdout
    for k in keys:
        assert ws[k] - before[k] >= 90, (k, ws[k] - before[k], dict(ws))
    for bad in ("x:1", "x:1:float", "x:maybe:bool", "x:abc:int"):
        r = _pa(["-m", "simple", "--request-parameter", bad])
        assert r.returncode == 1 and "request-parameter" in r.stderr, bad


def test_slot_pinned_caller_regions_keep_requests_apart(cpu_server):
    """--shared-memory-input NAME=R0,..,Rn / --shared-memory-output NAME=O0,..:
    concurrency slot s reads entry s % n and writes its own output region, so
    after a batched run (add_sub_batched rides the native dynamic batcher with
    batches of several requests) every output region must hold the result of
    ITS slot's inputs: a row mix-up in batch assembly or output scatter shows."""
    import numpy as np

    import tritonclient.grpc as grpcclient
    from tritonclient.utils import shared_memory as shm

    n = 6
    c = grpcclient.InferenceServerClient(cpu_server.grpc_url)
    regions, names = [], {"in0": [], "in1": [], "out0": [], "out1": []}
    try:
        for i in range(n):
            for kind in names:
                nm = "pin_%s_%d" % (kind, i)
                key = "/pin_%s_%d_%d" % (kind, i, os.getpid())
                r = shm.create_shared_memory_region(nm, key, 64)
                regions.append(r)
                names[kind].append(nm)
                if kind == "in0":
                    shm.set_shared_memory_region(r, [np.arange(16, dtype=np.int32) + 100 * i])
                elif kind == "in1":
                    shm.set_shared_memory_region(r, [np.full(16, 7 * i + 1, np.int32)])
                else:
                    shm.set_shared_memory_region(r, [np.full(16, -999, np.int32)])
                c.register_system_shared_memory(nm, key, 64)
        args = ["-m", "add_sub_batched", "-i", "grpc", "-u", cpu_server.grpc_url, "--shared-memory", "system",
                "--shared-memory-input", "INPUT0=" + ",".join(names["in0"]),
                "--shared-memory-input", "INPUT1=" + ",".join(names["in1"]),
                "--shared-memory-output", "OUTPUT0=" + ",".join(names["out0"]),
                "--shared-memory-output", "OUTPUT1=" + ",".join(names["out1"]),
                "--concurrency-range", str(n)]
        with native.PerfSession(args) as s:
            assert "caller regions pinned to slots" in s.describe()
            st0 = s.server_stats()
            lat, _ = s.run_fixed(n, 600)
            assert len(lat) == 600
            st1 = s.server_stats()
        execs = st1["execution_count"] - st0["execution_count"]
        infers = st1["inference_count"] - st0["inference_count"]
        assert infers >= 600 and infers > execs, ("no request was batched with another", infers, execs)
        byname = {nm: r for nm, r in zip([x for i in range(n) for x in (names["in0"][i], names["in1"][i],
                                                                         names["out0"][i], names["out1"][i])],
                                         regions)}
        for i in range(n):
            a = np.arange(16, dtype=np.int32) + 100 * i
            b = np.full(16, 7 * i + 1, np.int32)
            o0 = shm.get_contents_as_numpy(byname[names["out0"][i]], np.int32, [16])
            o1 = shm.get_contents_as_numpy(byname[names["out1"][i]], np.int32, [16])
            assert (o0 == a + b).all() and (o1 == a - b).all(), (i, o0, o1)
    finally:
        try:
            c.unregister_system_shared_memory()
        finally:
            for r in regions:
                shm.destroy_shared_memory_region(r)
