#!/bin/bash
# 7x7 dense-layer 1x1 tile shape with the fused split-K reduce: force the M tile (TCAMD_X3_BM) and split more
# (TCAMD_X3_SPLITK_BELOW), bs128 forward breakdown + engine throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
for BM in 64 128; do
  echo "== TCAMD_X3_BM=$BM TCAMD_X3_SPLITK_BELOW=400"
  TCAMD_X3_BM=$BM TCAMD_X3_SPLITK_BELOW=400 bash tools/gpu_x3_profile.sh 128 bm$BM || exit 1
  head -11 gpurun_out/bm$BM/breakdown_b128.md
  TCAMD_X3_BM=$BM TCAMD_X3_SPLITK_BELOW=400 timeout -k 10 200 python3 tools/fp32_engine_bench.py --batches 128 --streams 1,3 --engines fp32 --iters 15 2>&1 | grep engine || exit 1
done
