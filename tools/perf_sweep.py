"""Measured perf_analyzer baselines on one MI355X (BASELINE.md "Runs").

Starts the bench server on GPU 0, then runs the native perf_analyzer
(csrc/cpp/build/bin/perf_analyzer) through the BASELINE client modes:

  1. in-band binary tensors over gRPC and HTTP (the reference's data path)
  2. system shared memory
  3. HIP shared memory (zero-copy hipIpc handles, inputs filled on device by K1)

for densenet_onnx at bs=1 and bs=8 over a few concurrencies, and a bert_large
concurrency sweep over HIP shm.  Writes a markdown table + raw JSON.

  python tools/perf_sweep.py --out profiles/r1_perf_sweep.md
"""

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
PA = os.path.join(REPO, "csrc", "cpp", "build", "bin", "perf_analyzer")


def run_point(url_grpc, url_http, model, bs, proto, shm, conc, interval_ms, extra=()):
    url = url_grpc if proto == "grpc" else url_http
    out = "/tmp/pa_%d.json" % os.getpid()
    cmd = [PA, "-m", model, "-b", str(bs), "-i", proto, "-u", url, "--shared-memory", shm,
           "--concurrency-range", "%d" % conc, "-p", str(interval_ms), "-r", "6", "--json-report", out,
           "--percentile", "99"] + list(extra)
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": (r.stderr or r.stdout)[-500:], "cmd": " ".join(cmd)}
    rep = json.load(open(out))
    p = rep["points"][0]
    p["cmd"] = " ".join(os.path.relpath(c, REPO) if c.startswith(REPO) else c for c in cmd)
    p["wall_s"] = round(time.time() - t0, 1)
    p["data"] = rep["data"]
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r1_perf_sweep.md"))
    ap.add_argument("--interval-ms", type=int, default=2000)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    from triton_client_amd.perf.harness import ServerProcess

    log = os.path.join(REPO, "gpurun_out", "sweep_server.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    srv = ServerProcess(device=0, models="densenet_onnx,bert_large", log_path=log,
                        extra_args=["--instance-count", "3", "--max-queue-delay-us", "500"])
    rows = []
    try:
        srv.wait_ready(timeout=1200, model="densenet_onnx")
        srv.wait_ready(timeout=1200, model="bert_large")
        print("server ready", flush=True)
        modes = [("grpc", "none"), ("http", "none"), ("grpc", "system"), ("grpc", "hip")]
        concs = {1: [1, 16, 64], 8: [1, 16, 48]} if not a.quick else {1: [16], 8: [16]}
        for bs in (1, 8):
            for proto, shm in modes:
                for conc in concs[bs]:
                    p = run_point(srv.grpc_url, srv.http_url, "densenet_onnx", bs, proto, shm, conc, a.interval_ms)
                    p.update(model="densenet_onnx", bs=bs, proto=proto, shm=shm, conc=conc)
                    rows.append(p)
                    print(json.dumps({k: p.get(k) for k in ("model", "bs", "proto", "shm", "conc", "throughput",
                                                             "p99_us", "error")}), flush=True)
        for conc in ([1, 4, 16, 64, 256] if not a.quick else [16]):
            p = run_point(srv.grpc_url, srv.http_url, "bert_large", 1, "grpc", "hip", conc, a.interval_ms)
            p.update(model="bert_large", bs=1, proto="grpc", shm="hip", conc=conc)
            rows.append(p)
            print(json.dumps({k: p.get(k) for k in ("model", "conc", "throughput", "p99_us", "error")}), flush=True)
    finally:
        srv.stop()
    # the GPU box gets a snapshot without .git: pass the SHA in (TC_GIT_SHA=$(git rev-parse --short HEAD))
    sha = os.environ.get("TC_GIT_SHA") or subprocess.run(
        ["git", "rev-parse", "--short", "HEAD"], cwd=REPO, capture_output=True, text=True).stdout.strip() or "unknown"
    with open(a.out, "w") as f:
        f.write("# perf_analyzer sweep on 1x MI355X (measured)\n\n")
        f.write("git %s; server: `python -m triton_client_amd.server --gpu --models densenet_onnx,bert_large "
                "--instance-count 3 --max-queue-delay-us 500` (idle-aware dynamic batching; tcserve native gRPC front end, "
                "aiohttp HTTP); "
                "client: native `perf_analyzer` (csrc/cpp/perf), %d ms windows, stability on p99; synthetic data, "
                "random-init weights, bf16 compute.\n\n" % (sha, a.interval_ms))
        f.write("| model | bs | protocol | tensors | concurrency | infer/s | p50 us | p99 us | stable |\n")
        f.write("|---|---:|---|---|---:|---:|---:|---:|---|\n")
        for p in rows:
            if "error" in p:
                f.write("| %s | %d | %s | %s | %d | error | | | %s |\n" % (p["model"], p["bs"], p["proto"], p["shm"],
                                                                     p["conc"], p["error"][:80].replace("|", "/")))
                continue
            f.write("| %s | %d | %s | %s | %d | %.0f | %.0f | %.0f | %s |\n" % (
                p["model"], p["bs"], p["proto"], {"none": "in-band", "system": "system shm",
                                                   "hip": "HIP shm (K1 fill)"}[p["shm"]],
                p["conc"], p["throughput"], p["p50_us"], p["p99_us"], "yes" if p["stable"] else "no"))
        f.write("\nExample command: `%s`\n" % next((p["cmd"] for p in rows if "cmd" in p), ""))
    with open(a.out.replace(".md", ".json"), "w") as f:
        json.dump(rows, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
