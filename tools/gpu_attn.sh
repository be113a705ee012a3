#!/bin/bash
# K12 attention: numerics (+ BERT layer tests) and timing vs torch SDPA at bs64 x 384 
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_bert_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/attn_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/attn_probe.py --batch 64 > gpurun_out/attn_probe.log 2>&1 && for B in 1 4 8 16; do timeout -k 10 60 python3 tools/attn_probe.py --batch $B >> gpurun_out/attn_probe.log 2>&1 || exit 1; done
timeout -k 10 200 python3 tools/bert_probe.py --batch 1 8 64 > gpurun_out/bert_probe.log 2>&1 || exit 1
