#!/bin/bash
# L2<->fabric traffic of the fused DenseNet forward (two PMC passes, one per TCC budget).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=$PWD
B=${1:-128}
mkdir -p gpurun_out/pmcf
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf/fetch -o p -- \
  python3 tools/densenet_probe.py --buckets $B --stem 0 --torch 0 --iters 5 > gpurun_out/pmcf/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmcf/write -o p -- \
  python3 tools/densenet_probe.py --buckets $B --stem 0 --torch 0 --iters 5 > gpurun_out/pmcf/write.log 2>&1
