#!/bin/bash
# effective shader clock (GRBM_GUI_ACTIVE per XCD / kernel time) of the 3x3 v2 with and without MFMAs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/clk
for D in 0 1 6 7; do
  TCAMD_X3_K9_DBG=$D timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace \
    --output-format csv -d gpurun_out/clk/d$D -o p -- python3 tools/x3_kbench.py --op conv3x3 --hw 56 --imgs 128 --iters 5 \
    > gpurun_out/clk/d$D.log 2>&1 || exit 1
done
