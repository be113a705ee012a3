#!/bin/bash
# Round-end style check on one GPU: full GPU test suite, smoke(), the default
# bench, and a bert_large HIP-shm concurrency sweep with the native perf_analyzer.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 400 python -u - > gpurun_out/bert_sweep.log 2>&1 <<'PY'
import json, subprocess
from triton_client_amd.perf.harness import ServerProcess
from triton_client_amd.perf import native
srv = ServerProcess(device=0, models="bert_large", log_path="gpurun_out/bert_server.log",
                    extra_args=["--instance-count", "3", "--max-queue-delay-us", "500"])
try:
    srv.wait_ready(timeout=300, model="bert_large")
    for c in (1, 16, 64, 256):
        j = "/tmp/bert_c%d.json" % c
        r = subprocess.run([native.BIN_PATH, "-m", "bert_large", "-b", "1", "-i", "grpc", "-u", srv.grpc_url,
                            "--shared-memory", "hip", "--concurrency-range", str(c), "-p", "1000", "-r", "6",
                            "--percentile", "99", "--json-report", j], capture_output=True, text=True, timeout=120)
        pt = json.load(open(j))["points"][0] if r.returncode == 0 else {"error": r.stdout[-500:] + r.stderr[-500:]}
        print(json.dumps({"conc": c, "throughput": pt.get("throughput"), "p99_us": pt.get("p99_us"),
                          "error": pt.get("error")}), flush=True)
finally:
    srv.stop()
PY
