#!/bin/bash
# densenet_onnx bs=1 latency/throughput vs server queue delay (bench.py, HIP shm)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bs1
for D in ${DELAYS:-0 100 500}; do
  for C in 1 64; do
    timeout -k 10 200 python -u bench.py --batch 1 --concurrency $C --max-queue-delay-us $D --preferred "" \
      --instance-count 2 --steps 200 --warmup 20 > gpurun_out/bs1/d${D}_c${C}.log 2>&1 || exit 1
    echo "delay $D conc $C: $(tail -1 gpurun_out/bs1/d${D}_c${C}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "p50", d["p50_latency_us"], "p99", d["p99_latency_us"])')"
  done
done
