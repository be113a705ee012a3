#!/bin/bash
# PMC passes (SQ timing buckets) over K8 / K8p on one 1x1 shape.  Usage: tools/gpu_pmc_1x1.sh M K ldx "variants"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
M=$1; K=$2; LDX=$3
mkdir -p gpurun_out/pmc
for V in $4; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
    --output-format csv -d gpurun_out/pmc/v$V -o p -- python3 tools/kprobe_1x1.py --M $M --K $K --ldx $LDX --variant $V --iters 100 \
    > gpurun_out/pmc/v$V.log 2>&1 || exit 1
  echo "variant $V done"
done
