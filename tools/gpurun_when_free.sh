#!/bin/bash
# Run one gpurun call, re-submitting it ONLY while gpurun answers 3 ("no box
# or slot free right now", or the pod's GPU slots all busy: nothing ran, nothing
# was charged).  Any other exit
# code -- success, a failing or killed GPU step, a refusal -- ends the loop:
# a GPU step that failed is never re-run from here.
#   tools/gpurun_when_free.sh LOG TIMEOUT -- <command...>
log=$1; to=$2; shift 3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "on this pod are busy" "$log"; then break; fi
  echo "[when_free] no box (try $i); waiting" >> "$log.tries"
  sleep 150
done
echo "EXIT $rc" >> "$log"
