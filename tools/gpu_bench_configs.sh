#!/bin/bash
# A/B of bench.py server operating points (fp32 headline engine).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bcfg
i=0
while read -r ARGS; do
  [ -z "$ARGS" ] && continue
  i=$((i+1))
  echo "== $ARGS" >> gpurun_out/bcfg/summary.log
  timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-bf16 $ARGS > gpurun_out/bcfg/b$i.out 2> gpurun_out/bcfg/b$i.err || exit 1
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bcfg/b$i.out') if l.startswith('{')][-1]); print(d['value'], d['p50_latency_us'], d['p99_latency_us'], d['bs1']['infer_per_sec'], d['bs1']['concurrency1_p50_latency_us'])" >> gpurun_out/bcfg/summary.log
done <<< "$1"
