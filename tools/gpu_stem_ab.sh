#!/bin/bash
# stem versions (v1 LDS conv tile, v2 per-tile, v3 persistent): numerics + one-forward kernel time at bs128
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "stem or engine" > gpurun_out/stem_tests.log 2>&1 || exit 1
for V in ${STEM_VERSIONS:-2 3}; do
  TCAMD_X3_STEM=$V bash tools/gpu_x3_profile.sh 128 stem_v$V || exit 1
  grep -E "stem|one forward" gpurun_out/stem_v$V/breakdown_b128.md | head -3
done
