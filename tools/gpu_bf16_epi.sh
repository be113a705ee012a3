#!/bin/bash
# bf16 engine: kernel numerics after the staged epilogue + engine throughput (bf16 and fp32)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_densenet_kernels_gpu.py tests/test_hip_shm_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/bf16_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/fp32_engine_bench.py --batches 128 --streams 1,3 --engines bf16 --iters 20 \
  > gpurun_out/bf16_engine.log 2>&1 || exit 1
