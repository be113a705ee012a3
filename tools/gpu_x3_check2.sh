#!/bin/bash
# fp32 engine: kernel numerics + end-to-end parity tests, bs1 kernel durations, bs1/bs128 forward
# profiles and the engine throughput at 1 and 3 streams.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_densenet_fp32_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/x3check2_tests.log 2>&1 || { tail -30 gpurun_out/x3check2_tests.log; exit 1; }
tail -2 gpurun_out/x3check2_tests.log
bash tools/gpu_small_m.sh > gpurun_out/smallm.txt 2>&1 || exit 1
bash tools/gpu_x3_profile.sh 1 x3prof1 && bash tools/gpu_x3_profile.sh 128 x3prof128 || exit 1
head -4 gpurun_out/x3prof1/breakdown_b1.md; head -4 gpurun_out/x3prof128/breakdown_b128.md
timeout -k 10 300 python3 tools/fp32_engine_bench.py --batches 1,8,128 --streams 1,3 --engines fp32 --iters 20 \
  > gpurun_out/x3check2_engine.log 2>&1 || exit 1
grep engine gpurun_out/x3check2_engine.log
