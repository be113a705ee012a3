#!/bin/bash
# K9x 3x3 timing at the bs128 / bs8 layer shapes (+ the fp32 numerics tests first).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
mkdir -p gpurun_out/x3s
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/x3s/tests.log 2>&1 || exit 1
for C in "56 128" "28 128" "14 128" "7 128" "56 8" "28 8" "14 8"; do
  set -- $C
  timeout -k 10 60 python3 tools/x3_kbench.py --op conv3x3 --hw $1 --imgs $2 --iters 50 2>&1 | grep -v amdgpu.ids \
    >> gpurun_out/x3s/k3.log || exit 1
done
