#!/bin/bash
# Kernel trace of the fp32-parity DenseNet engine (K8x-K10x) at one batch size
# + the one-forward breakdown in launch order.
# Usage: tools/gpu_x3_profile.sh <batch> [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
B=${1:-128}; TAG=${2:-x3prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o probe -- \
  python3 tools/fp32_engine_bench.py --batches $B --streams 1 --engines fp32 --iters 5 > gpurun_out/$TAG/probe.log 2>&1 && \
python3 tools/forward_breakdown.py --marker x3_head_pool_kernel --order \
  $(find gpurun_out/$TAG -name '*kernel_trace.csv' | head -1) > gpurun_out/$TAG/breakdown_b$B.md
