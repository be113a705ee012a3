#!/bin/bash
# fp32 engine after the in-3x3 split-K reduce: kernel + engine numerics, bs1/bs8/bs128 forward profiles,
# engine throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/x3dense_tests.log 2>&1 || { tail -30 gpurun_out/x3dense_tests.log; exit 1; }
tail -2 gpurun_out/x3dense_tests.log
for B in 1 8 128; do
  bash tools/gpu_x3_profile.sh $B x3prof$B || exit 1
  head -12 gpurun_out/x3prof$B/breakdown_b$B.md
done
timeout -k 10 300 python3 tools/fp32_engine_bench.py --batches 1,8,128 --streams 1,3 --engines fp32 --iters 20 \
  > gpurun_out/x3dense_engine.log 2>&1 || exit 1
grep engine gpurun_out/x3dense_engine.log
