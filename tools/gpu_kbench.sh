#!/bin/bash
# Kernel numerics + per-layer sweeps on one GPU.  Usage: tools/gpu_kbench.sh [pytest -k expr] [kbench --only]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD:$PWD/tools
mkdir -p gpurun_out/kb
timeout -k 10 300 python -u -m pytest tests/test_densenet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "${1:-conv}" > gpurun_out/kb/tests.log 2>&1 && \
timeout -k 10 400 python -u tools/kbench_densenet.py --batch 128 --iters 30 --only "${2:-}" > gpurun_out/kb/kb128.log 2>&1
