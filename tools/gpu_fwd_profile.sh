#!/bin/bash
# Kernel trace of the fused DenseNet engine at one batch size + one-forward breakdown.
# Usage: tools/gpu_fwd_profile.sh <batch> [tag]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
B=${1:-128}; TAG=${2:-fwd}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o probe -- \
  python3 tools/densenet_probe.py --buckets $B --stem 0 --torch 0 --iters 20 > gpurun_out/$TAG/probe.log 2>&1 && \
python3 tools/forward_breakdown.py $(ls gpurun_out/$TAG/*kernel_trace.csv | head -1) > gpurun_out/$TAG/breakdown_b$B.md
