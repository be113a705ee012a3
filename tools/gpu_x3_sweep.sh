#!/bin/bash
# A/B of the K8x 1x1 tile plans on the small-M dense-layer shapes (bs128 14x14 / 7x7, bs8 56x56/28x28).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
mkdir -p gpurun_out/x3sweep
for BM in 0 32 64 128; do
  for C in "14 128 256" "14 128 640" "14 128 992" "7 128 512" "7 128 992" "56 8 224" "28 8 480"; do
    set -- $C
    TCAMD_X3_BM=$BM timeout -k 10 60 python3 tools/x3_kbench.py --op conv1x1 --hw $1 --imgs $2 --k $3 --iters 50 2>&1 \
      | grep -v amdgpu.ids | sed "s/^/bm=$BM /" >> gpurun_out/x3sweep/sweep.log || exit 1
  done
done
