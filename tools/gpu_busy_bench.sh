#!/bin/bash
# bench.py while sampling the amdgpu busy percent of the (single visible) GPU every 50 ms.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/busy
F=$(ls /sys/class/drm/card*/device/gpu_busy_percent 2>/dev/null | head -1)
echo "busy file: $F"
for args in "--instance-count 1 --concurrency 16" "--instance-count 3 --concurrency 48"; do
  tag=$(echo $args | tr ' -' '__')
  ( while true; do cat "$F" >> gpurun_out/busy/$tag.txt 2>/dev/null; sleep 0.05; done ) &
  SAMPLER=$!
  timeout -k 10 300 python -u bench.py --steps 100 $args > gpurun_out/busy/$tag.log 2>&1
  RC=$?
  kill $SAMPLER
  [ $RC = 0 ] || exit $RC
  echo "$args: $(tail -1 gpurun_out/busy/$tag.log | cut -c60-110) busy samples: $(sort -n gpurun_out/busy/$tag.txt | uniq -c | sort -rn | head -5 | tr '\n' ' ')"
done
