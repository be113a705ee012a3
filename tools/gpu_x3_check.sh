#!/bin/bash
# fp32 engine: kernel numerics + engine parity tests, one-forward breakdown at bs128,
# and the engine-only throughput (1 and 2 streams).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/x3check_tests.log 2>&1 || exit 1
bash tools/gpu_x3_profile.sh 128 x3prof_ws || exit 1
timeout -k 10 300 python3 tools/fp32_engine_bench.py --batches 128,256 --streams 1,2 --engines fp32 --iters 20 \
  > gpurun_out/x3check_engine.log 2>&1 || exit 1
