#!/bin/bash
# 7x7 bs128 1x1 (tiled BM 32): split-K threshold A/B, plus 14x14 / 7x7 transitions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
for K in 512 640 800 992; do
  for T in 192 400 800; do
    echo -n "hw=7 k=$K splitk_below=$T "
    TCAMD_X3_SPLITK_BELOW=$T timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw 7 --k $K --imgs 128 --iters 30 2>&1 | grep conv1x1 | sed 's/conv1x1 hw=.*k=[0-9]*: //' || exit 1
  done
done
