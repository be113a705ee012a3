#!/bin/bash
# Instruction mix per kernel of the fused DenseNet forward (one SQ PMC pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
B=${1:-128}
mkdir -p gpurun_out/pmcmix
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  --output-format csv -d gpurun_out/pmcmix -o p -- python3 tools/densenet_probe.py --buckets $B --stem 0 --torch 0 --iters 3 \
  > gpurun_out/pmcmix/log.txt 2>&1
