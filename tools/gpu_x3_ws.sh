#!/bin/bash
# fp32 1x1 numerics (incl. the warp-specialised kernel) + A/B timing at bs128 shapes:
# tiled (WS=0) vs warp-specialised PF 3 / PF 5, plus the ablations of PF 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "conv1x1_split_out" > gpurun_out/x3ws_tests.log 2>&1 || exit 1
for K in 64 128 192 256 128:28 256:28 480:28; do
  IFS=: read KK HW <<< "$K"; HW=${HW:-56}
  for V in "0 3 0" "1 3 0" "1 5 0" "1 3 1" "1 3 2" "1 3 3"; do
    read WS PF DBG <<< "$V"
    echo -n "hw=$HW k=$KK ws=$WS pf=$PF dbg=$DBG "
    TCAMD_X3_WS=$WS TCAMD_X3_WS_PF=$PF TCAMD_X3_WS_DBG=$DBG timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw $HW --k $KK --imgs 128 --iters 30 2>&1 | grep conv1x1 || exit 1
  done
done
