mkdir -p gpurun_out/ab4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_densenet_fp32_gpu.py -k "x3_dense_small or engine" > gpurun_out/ab4/tests.log 2>&1 || exit 1
for r in 1 2; do for lib in base new; do
  if [ $lib = base ]; then export TCAMD_HIP_LIB=$PWD/ab/libtcamd_hip_base.so; else unset TCAMD_HIP_LIB; fi
  timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,512,992 --rounds 3 >> gpurun_out/ab4/k14_$lib.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/fp32_engine_bench.py --batches 128,64 --streams 1,2 --engines fp32 --iters 20 >> gpurun_out/ab4/eng_$lib.log 2>&1 || exit 1
done; done
unset TCAMD_HIP_LIB
timeout -k 10 120 python -u tools/k14x_bench.py --ks 512,992 --hw 14 --stamp --dbg 64 --rounds 1 > gpurun_out/ab4/timeline.log 2>&1 || exit 1
