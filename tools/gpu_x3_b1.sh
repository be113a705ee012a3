#!/bin/bash
# fp32 engine small batches: numerics of the dense-layer path, bs1/bs8 forward profiles, engine throughput.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "dense_layer or engine" > gpurun_out/x3b1_tests.log 2>&1 || { tail -30 gpurun_out/x3b1_tests.log; exit 1; }
tail -1 gpurun_out/x3b1_tests.log
for B in 1 8; do
  bash tools/gpu_x3_profile.sh $B x3prof$B || exit 1
  head -8 gpurun_out/x3prof$B/breakdown_b$B.md
done
timeout -k 10 300 python3 tools/fp32_engine_bench.py --batches 1,8 --streams 1,3 --engines fp32 --iters 20 \
  > gpurun_out/x3b1_engine.log 2>&1 || exit 1
grep engine gpurun_out/x3b1_engine.log
