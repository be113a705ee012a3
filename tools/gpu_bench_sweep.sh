#!/bin/bash
# bench.py variants on one GPU: each line "conc pref delay [instances [idle [max_batch]]]" -> gpurun_out/sweep/*.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
while read -r C P D I X B; do
  I=${I:-2}; X=${X:-on}; B=${B:-0}
  [ -z "$C" ] && continue
  tag="c${C}_p${P:-none}_d${D}_i${I}_idle${X}_mb${B}"
  extra=""
  [ "$P" != "none" ] && extra="--preferred $P"
  timeout -k 10 240 python -u bench.py --steps 40 --warmup 10 --concurrency $C --max-queue-delay-us $D --instance-count $I --idle-dispatch $X --max-batch-size $B $extra \
    > gpurun_out/sweep/$tag.log 2>&1 || { echo "FAIL $tag"; exit 1; }
  echo "$tag $(tail -1 gpurun_out/sweep/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_us"], d["p99_latency_us"], d.get("server_avg_batch_rows_rank0"))')"
done < "${1:-/dev/stdin}"
