mkdir -p gpurun_out/g9
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/g9/tests.log 2>&1 || exit 1
TCAMD_GEMM_HALF=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "matches_fp32" > gpurun_out/g9/tests_half2.log 2>&1 || exit 1
for r in 1 2; do for h in 0 1 2; do
  TCAMD_GEMM_HALF=$h timeout -k 10 200 python -u tools/gemm_probe.py --variant 6 --tokens 24576,3072 --rounds 3 >> gpurun_out/g9/probe_h$h.log 2>&1 || exit 1
done; done
