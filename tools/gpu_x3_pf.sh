#!/bin/bash
# A/B of the BM-128 1x1 register-ring depth (TCAMD_X3_PF128) at the bs128 layer shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
for K in 64 128 192 256 128:28 256:28 480:28; do
  IFS=: read KK HW <<< "$K"; HW=${HW:-56}
  for PF in 1 2; do
    echo -n "hw=$HW k=$KK pf=$PF "
    TCAMD_X3_PF128=$PF timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw $HW --k $KK --imgs 128 --iters 30 || exit 1
  done
done
