#!/bin/bash
# Profile the bench SERVER (where the model kernels run) with rocprofv3:
# the server runs under the profiler, bench.py drives it from outside, then the
# server is stopped with SIGTERM so the profiler flushes its CSVs.
# Usage: tools/gpu_profile.sh [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
rm -f gpurun_out/prof/*.csv
# MARKERS=1: also record roctx ranges (tcserve batches, model forwards; TC_ROCTX=1 turns them on)
TRACE="--kernel-trace --stats"
if [ "${MARKERS:-0}" = 1 ]; then export TC_ROCTX=1; TRACE="$TRACE --marker-trace"; fi
timeout -k 10 900 rocprofv3 $TRACE --output-format csv -d gpurun_out/prof -o server -- \
  python3 -m triton_client_amd.server --http-port 18000 --grpc-port 18001 --gpu --models densenet_onnx \
  --instance-count ${INSTANCES:-4} --preferred-batch-sizes 128 --max-queue-delay-us 2000 --idle-dispatch off \
  > gpurun_out/prof_server.log 2>&1 &
PROF_PID=$!
timeout -k 10 600 python3 bench.py --server-url 127.0.0.1:18001 --http-url 127.0.0.1:18000 "$@" \
  > gpurun_out/prof_bench.log 2>&1
RC=$?
# stop the python server (child of rocprofv3) gracefully
# rocprofv3 may exec the program itself (then PROF_PID is the server)
SRV_PID=$(pgrep -P $PROF_PID -n python3 || true)
kill -TERM "${SRV_PID:-$PROF_PID}"
# the profiler flushes its CSVs on SIGTERM, but the server may not exit after
# that: give it 30 s, then kill the process group member by PID
for i in $(seq 30); do
  kill -0 $PROF_PID 2>/dev/null || break
  echo "waiting for profiler exit ($i s)"
  sleep 1
done
kill -KILL ${SRV_PID:-} $PROF_PID 2>/dev/null
wait $PROF_PID
echo "bench rc=$RC profiler rc=$?"
exit $RC
