#!/bin/bash
# K8x ws: X steps in flight (TCAMD_X3_WS_PF 3/5/6) with and without the MFMA/stores (dbg 3 = X read only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
for K in 128 224; do
  for D in 0 3; do
    for PF in 3 5 6; do
      echo -n "k=$K ldx=256 dbg=$D pf=$PF "
      TCAMD_X3_WS_DBG=$D TCAMD_X3_WS_PF=$PF timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw 56 --k $K --ldx 256 --imgs 128 --iters 30 2>&1 | grep conv1x1 || exit 1
    done
  done
done
