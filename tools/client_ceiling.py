#!/usr/bin/env python3
"""Load-generator / client ceiling: how many requests per second each client
flavour can push when the server costs (almost) nothing, so that the
headline's load generator is shown not to be the bottleneck.

Server: the KServe-v2 test server in a child process (native tcserve front
end, CPU models only).  Models: ``add_sub_batched`` (2 x INT32[16] in/out: pure
request overhead) and ``frontend_sink`` (the densenet_onnx request shape,
FP32 [bs,3,224,224] in, [bs,1000] out, no compute) over system shared memory.

  * native C++ perf_analyzer, gRPC and HTTP, concurrency 1..256;
  * Python clients: gRPC sync, gRPC async_infer (callbacks), gRPC aio, HTTP
    sync, HTTP async_infer (connection pool), HTTP aio.

    python tools/client_ceiling.py --json profiles/r2_client_ceiling.json --md profiles/r2_client_ceiling.md
"""

import argparse
import asyncio
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def perf(url, proto, model, conc, extra=(), count=None):
    from triton_client_amd.perf import native

    j = "/tmp/ceiling_%s_%s_%d.json" % (proto, model, conc)
    cmd = [native.BIN_PATH, "-m", model, "-i", proto, "-u", url, "--concurrency-range", str(conc),
           "--measurement-mode", "count_windows", "--measurement-request-count",
           str(count or max(2000, 40 * conc)),
           "-s", "15", "-r", "6", "--json-report", j, *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode:
        return {"error": (r.stdout + r.stderr)[-400:]}
    p = json.load(open(j))["points"][0]
    return {"infer_per_sec": round(p["throughput"], 1), "p50_us": p["p50_us"], "p99_us": p["p99_us"]}


def py_clients(http_url, grpc_url, seconds=2.0):
    import numpy as np

    import tritonclient.grpc as grpcclient
    import tritonclient.grpc.aio as grpcaio
    import tritonclient.http as httpclient
    import tritonclient.http.aio as httpaio

    a = np.arange(16, dtype=np.int32).reshape(1, 16)

    def ins(mod):
        x = [mod.InferInput("INPUT0", [1, 16], "INT32"), mod.InferInput("INPUT1", [1, 16], "INT32")]
        x[0].set_data_from_numpy(a)
        x[1].set_data_from_numpy(a)
        return x

    out = {}

    def timed(fn):
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            n += fn()
        return round(n / (time.perf_counter() - t0), 1)

    g = grpcclient.InferenceServerClient(grpc_url)
    gi = ins(grpcclient)
    out["python grpc sync (1 thread)"] = timed(lambda: (g.infer("add_sub_batched", gi), 1)[1])

    def grpc_async_batch(k=64):
        done = threading.Semaphore(0)
        for _ in range(k):
            g.async_infer("add_sub_batched", gi, lambda result, error: done.release())
        for _ in range(k):
            done.acquire()
        return k
    out["python grpc async_infer (64 in flight)"] = timed(grpc_async_batch)
    g.close()

    h = httpclient.InferenceServerClient(http_url, concurrency=16)
    hi = ins(httpclient)
    out["python http sync (1 thread)"] = timed(lambda: (h.infer("add_sub_batched", hi), 1)[1])

    def http_async_batch(k=64):
        reqs = [h.async_infer("add_sub_batched", hi) for _ in range(k)]
        for r in reqs:
            r.get_result()
        return k
    out["python http async_infer (pool 16, 64 in flight)"] = timed(http_async_batch)
    h.close()

    async def aio_rate(mk, url):
        c = mk(url)
        x = ins(grpcaio if mk is grpcaio.InferenceServerClient else httpaio)
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            await asyncio.gather(*[c.infer("add_sub_batched", x) for _ in range(64)])
            n += 64
        rate = n / (time.perf_counter() - t0)
        await c.close()
        return round(rate, 1)

    out["python grpc aio (64 tasks)"] = asyncio.run(aio_rate(grpcaio.InferenceServerClient, grpc_url))
    out["python http aio (64 tasks)"] = asyncio.run(aio_rate(httpaio.InferenceServerClient, http_url))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="")
    ap.add_argument("--md", default="")
    ap.add_argument("--compression-only", action="store_true", help="only the gzip REST points")
    ap.add_argument("--target-req-per-gpu", type=float, default=34455.0 / 8,
                    help="headline request rate one GPU's load generator must sustain (infer/s / bs)")
    a = ap.parse_args()
    from triton_client_amd.perf.harness import ServerProcess

    srv = ServerProcess(gpu=False, models="add_sub_batched,frontend_sink", log_path="/tmp/ceiling_server.log",
                        extra_args=["--native-grpc", "on"])
    rows = {"perf_analyzer": {}, "python": {}}
    try:
        srv.wait_ready(timeout=120, model="add_sub_batched")
        # compressed native REST (gzip both ways, in-band bs8 zero tensors, so
        # the client's own deflate of 4.8 MB bodies stays cheap): the
        # responses are deflated on tcserve's codec pool, off the batcher threads
        for conc in (16, 64):
            k = "http frontend_sink bs8 in-band gzip c%d" % conc
            rows["perf_analyzer"][k] = perf(srv.http_url, "http", "frontend_sink", conc,
                                            ("-b", "8", "--compression-algorithm", "gzip", "--input-data", "zero"),
                                            count=400)
            print(k, rows["perf_analyzer"][k], flush=True)
        for conc in (16, 64):
            k = "http add_sub_batched gzip c%d" % conc
            rows["perf_analyzer"][k] = perf(srv.http_url, "http", "add_sub_batched", conc,
                                            ("--compression-algorithm", "gzip"))
            print(k, rows["perf_analyzer"][k], flush=True)
        if a.compression_only:
            for k, v in rows["perf_analyzer"].items():
                print(json.dumps({k: v}))
            return
        for proto, url in (("grpc", srv.grpc_url), ("http", srv.http_url)):
            for conc in (1, 16, 64, 256):
                k = "%s add_sub_batched c%d" % (proto, conc)
                rows["perf_analyzer"][k] = perf(url, proto, "add_sub_batched", conc)
                print(k, rows["perf_analyzer"][k], flush=True)
            for conc in (16, 64, 256):
                k = "%s frontend_sink bs8 system-shm c%d" % (proto, conc)
                rows["perf_analyzer"][k] = perf(url, proto, "frontend_sink", conc,
                                                ("-b", "8", "--shared-memory", "system",
                                                 "--output-shared-memory-size", str(8 * 1000 * 4)))
                print(k, rows["perf_analyzer"][k], flush=True)
        rows["python"] = py_clients(srv.http_url, srv.grpc_url)
        print(rows["python"], flush=True)
    finally:
        srv.stop()
    best_req = max(v.get("infer_per_sec", 0) for k, v in rows["perf_analyzer"].items() if "add_sub" in k)
    sink = max(v.get("infer_per_sec", 0) / 8 for k, v in rows["perf_analyzer"].items() if "frontend_sink" in k)
    rows["target_req_per_gpu"] = round(a.target_req_per_gpu, 1)
    rows["headroom_simple"] = round(best_req / a.target_req_per_gpu, 1)
    rows["headroom_headline_shape"] = round(sink / a.target_req_per_gpu, 1)
    if a.json:
        json.dump(rows, open(a.json, "w"), indent=1)
    if a.md:
        L = ["# Client / load-generator ceiling (round 2)", "",
             "`tools/client_ceiling.py`: server = the test server in a child process (native tcserve front end, "
             "CPU models, no compute); one load-generator process; measured in the 8-CPU build container (server and client share those 8 cores).  `frontend_sink` is the densenet_onnx request "
             "shape (FP32 [8,3,224,224] in, [8,1000] out) with system shared memory for both.", "",
             "| client | load | infer/s | p50 us | p99 us |", "|---|---|---:|---:|---:|"]
        for k, v in rows["perf_analyzer"].items():
            if "error" in v:
                L.append("| perf_analyzer (C++) | %s | error | | |" % k)
            else:
                L.append("| perf_analyzer (C++) | %s | %.0f | %.0f | %.0f |" % (k, v["infer_per_sec"], v["p50_us"],
                                                                           v["p99_us"]))
        for k, v in rows["python"].items():
            L.append("| %s | add_sub_batched | %.0f | | |" % (k, v))
        L += ["", "Headline request rate one GPU's load generator must sustain: %.0f req/s (the 1-GPU headline "
              "infer/s at bs 8)." % a.target_req_per_gpu,
              "Native load-generator ceiling: %.0fx that on `add_sub_batched` requests (2 x INT32[16]) and %.0fx at the headline request "
              "shape (frontend_sink, requests/s = infer/s / 8)." % (rows["headroom_simple"],
                                                                  rows["headroom_headline_shape"])]
        open(a.md, "w").write("\n".join(L) + "\n")
    print(json.dumps({k: rows[k] for k in ("target_req_per_gpu", "headroom_simple", "headroom_headline_shape")}))


if __name__ == "__main__":
    main()
