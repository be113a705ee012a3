#!/bin/bash
# 3x3 v2 ablation at bs128: TCAMD_X3_K9_DBG 1 no MFMA, 2 no partial exchange, 4 no operand reads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
for HW in 56 28 14; do
  for D in 0 1 2 4 3 5 6 7; do
    echo -n "hw=$HW dbg=$D "
    TCAMD_X3_K9_DBG=$D timeout -k 10 60 python3 tools/x3_kbench.py --op conv3x3 --hw $HW --imgs 128 --iters 30 2>&1 | grep conv3x3 | sed 's/conv3x3 hw=.*k=[0-9]*: //' || exit 1
  done
done
