#!/bin/bash
# default bench.py + one-forward profile at bs128
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 && tail -1 gpurun_out/bench_default.log && \
bash tools/gpu_fwd_profile.sh 128 fwd128q
