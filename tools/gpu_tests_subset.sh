#!/bin/bash
# GPU pytest subset: tools/gpu_tests_subset.sh "<pytest -k expr>" [files...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K="$1"; shift
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 180 --timeout-method thread -k "$K" \
  > gpurun_out/gpu_subset.log 2>&1
