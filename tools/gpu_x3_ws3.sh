#!/bin/bash
# ws 1x1 on the small layers (TCAMD_X3_WS_MIN) vs the tiled kernel + numerics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
TCAMD_X3_WS_MIN=1024 timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "conv1x1_split_out or engine" > gpurun_out/x3ws3_tests.log 2>&1 || exit 1
for K in 128:28 480:28 256:14 512:14 768:14 992:14 512:7 992:7 64:56 256:56; do
  IFS=: read KK HW <<< "$K"
  for MIN in 1000000000 1024; do
    echo -n "hw=$HW k=$KK wsmin=$MIN "
    TCAMD_X3_WS_MIN=$MIN timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw $HW --k $KK --imgs 128 --iters 30 2>&1 | grep conv1x1 | sed 's/conv1x1 hw=.*k=[0-9]*: //' || exit 1
  done
done
