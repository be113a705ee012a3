#!/bin/bash
# Profile the flagship bench on the GPU box: per-kernel stats for the server
# (child process inherits the rocprofv3 preload).  Usage: tools/gpu_profile.sh [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
  python3 bench.py "$@" > gpurun_out/prof_bench.log 2>&1
