set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_densenet_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "stem or fused" > gpurun_out/stem_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/kbench_stem.py > gpurun_out/kbench_stem.log 2>&1 && \
bash tools/gpu_fwd_profile.sh 128 fwd128s
