#!/bin/bash
# fp32 engine quick check: bs128 forward kernel profile and engine throughput at 1 and 3 streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
bash tools/gpu_x3_profile.sh 128 x3prof128 || exit 1
head -12 gpurun_out/x3prof128/breakdown_b128.md
timeout -k 10 300 python3 tools/fp32_engine_bench.py --batches 128 --streams 1,3 --engines fp32 --iters 20 \
  > gpurun_out/x3quick_engine.log 2>&1 || exit 1
grep engine gpurun_out/x3quick_engine.log
