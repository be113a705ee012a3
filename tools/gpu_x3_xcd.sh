#!/bin/bash
# transition 1x1s: XCD-grouped sibling N-tiles (TCAMD_X3_XCD_GROUP) numerics + pool kbench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/xcd_tests.log 2>&1 || exit 1
for C in 256:56 512:28 1024:14; do
  IFS=: read K HW <<< "$C"
  for X in 0 1; do
    echo -n "pool hw=$HW k=$K xcd=$X "
    TCAMD_X3_XCD_GROUP=$X timeout -k 10 60 python3 tools/x3_kbench.py --op pool --hw $HW --k $K --imgs 128 --iters 30 2>&1 | grep pool | sed 's/pool hw=.*k=[0-9]*: //' | cut -c1-20 || exit 1
  done
done
