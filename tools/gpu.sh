#!/bin/bash
# The one launcher for GPU-box runs (replaces the per-experiment gpu_*.sh
# scripts of rounds 1-2; their results live in profiles/):
#
#   gpurun --timeout 900 -- bash tools/gpu.sh "tests" "smoke" "bench --steps 10"
#
# Each quoted argument is one step; steps run in order, each under its own
# time limit, and the script stops at the first failing step (no retries).
#   tests [pytest args...]     GPU suite (e.g. "tests -k executor")   -> gpurun_out/gpu_tests.log
#   smoke                      __graft_entry__.smoke()                 -> gpurun_out/smoke.log
#   bench [bench.py args...]   bench.py (JSON line on stdout)          -> gpurun_out/bench<N>.log/.err
#   bert [bench.py args...]    bench.py --model bert_large             -> gpurun_out/bench_bert.log
#   py <script> [args...]      python tools/<script> (probes, kbench)  -> gpurun_out/py_<script>.log
#   prof <tag> <cmd...>        rocprofv3 --kernel-trace --stats on <cmd> -> gpurun_out/prof_<tag>/
#   pmc <tag> <counters> <cmd...>  one rocprofv3 --pmc pass (counters comma-separated)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
n_bench=0
for step in "$@"; do
  read -r -a a <<< "$step"
  name=${a[0]}
  args=("${a[@]:1}")
  echo "== step: $step ($(date +%T))"
  case "$name" in
    tests)
      [ ${#args[@]} -eq 0 ] && args=(tests)
      timeout -k 10 1000 python -u -m pytest "${args[@]}" -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
      rc=$?
      tail -3 gpurun_out/gpu_tests.log
      ;;
    smoke)
      timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?
      tail -2 gpurun_out/smoke.log
      ;;
    bench)
      n_bench=$((n_bench + 1))
      timeout -k 10 600 python -u bench.py "${args[@]}" > gpurun_out/bench${n_bench}.log 2> gpurun_out/bench${n_bench}.err
      rc=$?
      tail -1 gpurun_out/bench${n_bench}.log
      ;;
    bert)
      timeout -k 10 600 python -u bench.py --model bert_large "${args[@]}" > gpurun_out/bench_bert.log \
        2> gpurun_out/bench_bert.err
      rc=$?
      tail -1 gpurun_out/bench_bert.log
      ;;
    py)
      script=${args[0]}
      timeout -k 10 600 python -u "tools/$script" "${args[@]:1}" > "gpurun_out/py_${script%.py}.log" 2>&1
      rc=$?
      tail -5 "gpurun_out/py_${script%.py}.log"
      ;;
    prof)
      tag=${args[0]}
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null || exit 1
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_${tag}" -o run_%pid% -- "${args[@]:1}" \
        > "gpurun_out/prof_${tag}.log" 2>&1
      rc=$?
      tail -2 "gpurun_out/prof_${tag}.log"
      ;;
    pmc)
      tag=${args[0]}
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${args[1]//,/ } -d "gpurun_out/pmc_${tag}" -o run -- \
        "${args[@]:2}" > "gpurun_out/pmc_${tag}.log" 2>&1
      rc=$?
      tail -2 "gpurun_out/pmc_${tag}.log"
      ;;
    *)
      echo "unknown step: $name"
      exit 2
      ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "== step failed (rc $rc): $step"
    exit $rc
  fi
done
echo "== all steps passed"
