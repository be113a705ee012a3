set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
TC_GIT_SHA=nativehttp timeout -k 10 400 python -u tools/perf_sweep.py --quick --interval-ms 1000 --out gpurun_out/sweep_quick.md > gpurun_out/sweep_quick.log 2>&1
