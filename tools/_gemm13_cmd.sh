mkdir -p gpurun_out/g13
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k variant > gpurun_out/g13/tests.log 2>&1 || exit 1
for r in 1 2; do for v in 6 11; do
  timeout -k 10 200 python -u tools/gemm_probe.py --variant $v --tokens 24576,3072 --rounds 3 >> gpurun_out/g13/probe_v$v.log 2>&1 || exit 1
done; done
