#!/bin/bash
# ws 1x1: K-step rotation across blocks (dbg bit 4 = off) A/B + numerics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "conv1x1_split_out" > gpurun_out/x3ws_tests.log 2>&1 || exit 1
for K in 64 128 256 128:28 480:28 1024:7; do
  IFS=: read KK HW <<< "$K"; HW=${HW:-56}
  for DBG in 4 0 7 3; do
    echo -n "hw=$HW k=$KK dbg=$DBG "
    TCAMD_X3_WS_DBG=$DBG timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw $HW --k $KK --imgs 128 --iters 30 2>&1 | grep conv1x1 | sed 's/conv1x1 hw=.*launch, //' || exit 1
  done
done
