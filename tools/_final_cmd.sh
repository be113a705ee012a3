mkdir -p gpurun_out/fin
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/fin/gemm_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bert_probe.py --batch 8 64 --k15-ab 2048 --rounds 3 > gpurun_out/fin/bert_k15_ab.log 2>&1 || exit 1
