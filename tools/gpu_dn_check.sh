set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_densenet_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dn_tests.log 2>&1 && \
bash tools/gpu_bench_quick.sh
