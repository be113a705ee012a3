#!/bin/bash
# Split-K threshold A/B now that the 3x3 reduces the partials (TCAMD_X3_SPLITK_BELOW: split when fewer 1x1 tiles than this).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
for T in 192 256 400; do
  echo "== TCAMD_X3_SPLITK_BELOW=$T"
  TCAMD_X3_SPLITK_BELOW=$T bash tools/gpu_x3_profile.sh 128 thr$T || exit 1
  head -10 gpurun_out/thr$T/breakdown_b128.md
  TCAMD_X3_SPLITK_BELOW=$T timeout -k 10 200 python3 tools/fp32_engine_bench.py --batches 8,128 --streams 1,3 --engines fp32 --iters 15 2>&1 | grep engine || exit 1
done
