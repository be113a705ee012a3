#!/bin/bash
# Client data kernels (K1-K7): achieved GB/s vs HBM + rocprofv3 kernel table
# (LDS_Block_Size column = the LDS staging of each kernel) + an LDS counter pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
mkdir -p gpurun_out/kio
timeout -k 10 300 python3 tools/kbench_io.py --iters 20 --json gpurun_out/kio/kbench_io.json > gpurun_out/kio/kbench_io.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kio/trace -o io -- \
  python3 tools/kbench_io.py --iters 5 --sizes 4.8e6 > gpurun_out/kio/trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv \
  -d gpurun_out/kio/pmc -o io -- python3 tools/kbench_io.py --iters 2 --sizes 4.8e6 > gpurun_out/kio/pmc.log 2>&1
