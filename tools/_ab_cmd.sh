mkdir -p gpurun_out/ab3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_densenet_fp32_gpu.py -k "x3_dense_small or engine" > gpurun_out/ab3/tests.log 2>&1 || exit 1
for r in 1 2; do for w in 0 1; do
  timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,512,992 --rounds 3 --wreg $w >> gpurun_out/ab3/k14_w$w.log 2>&1 || exit 1
done; done
timeout -k 10 120 python -u tools/k14x_bench.py --ks 512,992 --hw 14 --stamp --dbg 64 --rounds 1 --wreg 1 > gpurun_out/ab3/timeline_w1.log 2>&1 || exit 1
for w in 0 1 0 1; do TCAMD_X3_SMALLF_WREG=$w timeout -k 10 120 python -u tools/fp32_engine_bench.py --batches 128,64 --streams 1,2 --engines fp32 --iters 20 >> gpurun_out/ab3/eng_w$w.log 2>&1 || exit 1; done
