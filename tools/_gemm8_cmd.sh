mkdir -p gpurun_out/g8
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/g8/tests.log 2>&1 || exit 1
for r in 1 2; do for v in 1 6; do
  timeout -k 10 200 python -u tools/gemm_probe.py --variant $v --tokens 24576,3072 --rounds 3 >> gpurun_out/g8/probe_v$v.log 2>&1 || exit 1
done; done
