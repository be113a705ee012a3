#!/bin/bash
# bert_large sweep under different server batching settings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD
mkdir -p gpurun_out/bertcfg
i=0
while read -r ARGS; do
  [ -z "$ARGS" ] && continue
  i=$((i+1))
  echo "== $ARGS" >> gpurun_out/bertcfg/summary.log
  timeout -k 10 400 python -u bench.py --model bert_large --steps 5 --warmup 1 $ARGS > gpurun_out/bertcfg/b$i.out \
    2> gpurun_out/bertcfg/b$i.err || exit 1
  grep "bert c" gpurun_out/bertcfg/b$i.err >> gpurun_out/bertcfg/summary.log
done <<< "$1"
