#!/bin/bash
# bert_large forward with torch TunableOp GEMM selection (hipBLASLt + rocBLAS candidates) vs default heuristics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
timeout -k 10 200 python3 tools/bert_probe.py --batch 8 64 > gpurun_out/tun_off.log 2>&1 || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 600 python3 tools/bert_probe.py --batch 8 64 > gpurun_out/tun_on.log 2>&1 || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv \
  timeout -k 10 200 python3 tools/bert_probe.py --batch 8 64 > gpurun_out/tun_use.log 2>&1 || exit 1
