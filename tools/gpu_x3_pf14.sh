#!/bin/bash
# ws 1x1 on the latency-bound 14x14 layers: register-ring depth 3 vs 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
for K in 256:14 512:14 992:14 128:28 480:28; do
  IFS=: read KK HW <<< "$K"
  for PF in 3 5; do
    echo -n "hw=$HW k=$KK pf=$PF "
    TCAMD_X3_WS_PF=$PF timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw $HW --k $KK --imgs 128 --iters 30 2>&1 | grep conv1x1 | sed 's/conv1x1 hw=.*k=[0-9]*: //' | cut -c1-20 || exit 1
  done
done
