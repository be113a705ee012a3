#!/bin/bash
# ws 1x1 equal-tile split: numerics + timings at the bs128 layer shapes + forward profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/x3check_tests.log 2>&1 || exit 1
for K in 64:56 256:56 128:28 256:28 480:28 256:14 992:14; do
  IFS=: read KK HW <<< "$K"
  echo -n "hw=$HW k=$KK "
  timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw $HW --k $KK --imgs 128 --iters 30 2>&1 | grep conv1x1 | sed 's/conv1x1 hw=.*k=[0-9]*: //' || exit 1
done
bash tools/gpu_x3_profile.sh 128 x3prof_ws || exit 1
