#!/bin/bash
# fp32 engine at 1 and 3 streams with the persistent kernels' grid at 1x / 2x / 4x the CU count
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
for G in 1 2 4; do
  echo "== grid mult $G"
  TCAMD_X3_GRID_MULT=$G timeout -k 10 300 python3 tools/fp32_engine_bench.py --batches 128 --streams 1,3 --engines fp32 \
    --iters 20 || exit 1
done
