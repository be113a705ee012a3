#!/bin/bash
# PMC passes over single fp32-parity kernels at bs128 shapes (tools/x3_kbench.py).
# Usage: tools/gpu_pmc_x3.sh "<case> ..." where case = op:hw:k  (e.g. conv3x3:56:0 conv1x1:56:224)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
mkdir -p gpurun_out/pmcx3
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
for C in $1; do
  IFS=: read OP HW K <<< "$C"
  timeout -k 10 120 python3 tools/x3_kbench.py --op $OP --hw $HW --k $K --imgs 128 --iters 50 >> gpurun_out/pmcx3/timing.log 2>&1 || exit 1
  for PASS in 1 2 3 4; do
    eval CT=\$P$PASS
    timeout -s KILL 90 rocprofv3 --pmc $CT --output-format csv -d gpurun_out/pmcx3/${OP}_${HW}_${K}_p$PASS -o p -- \
      python3 tools/x3_kbench.py --op $OP --hw $HW --k $K --imgs 128 --iters 5 > gpurun_out/pmcx3/${OP}_${HW}_${K}_p$PASS.log 2>&1 || exit 1
  done
done
