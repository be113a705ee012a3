#!/bin/bash
# Profile the default bench with rocprofv3: bench.py runs under the profiler and
# so does its server child process (the profiler's environment is inherited),
# where the model kernels run; one kernel_stats CSV per process.
# Usage: tools/gpu_profile.sh [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
mkdir -p gpurun_out/prof
rm -rf gpurun_out/prof/*
# MARKERS=1: also record roctx ranges (tcserve batches, model forwards; TC_ROCTX=1 turns them on)
TRACE="--kernel-trace --stats"
if [ "${MARKERS:-0}" = 1 ]; then export TC_ROCTX=1; TRACE="$TRACE --marker-trace"; fi
timeout -k 10 900 rocprofv3 $TRACE --output-format csv -d gpurun_out/prof -o bench_%pid% -- \
  python3 bench.py "$@" > gpurun_out/prof_bench.log 2>&1
RC=$?
echo "bench under rocprofv3 rc=$RC"
exit $RC
