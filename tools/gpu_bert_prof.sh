#!/bin/bash
# per-kernel split of one bert_large bs64 forward
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/bertprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bertprof -o p -- \
  python3 tools/bert_probe.py --batch 64 --iters 5 > gpurun_out/bertprof/log 2>&1 || exit 1
