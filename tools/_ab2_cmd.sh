mkdir -p gpurun_out/ab5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_densenet_fp32_gpu.py > gpurun_out/ab5/tests.log 2>&1 || exit 1
for r in 1 2; do for lib in base0 base new; do
  if [ $lib = new ]; then unset TCAMD_HIP_LIB; else export TCAMD_HIP_LIB=$PWD/ab/libtcamd_hip_$lib.so; fi
  timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,992 --rounds 3 >> gpurun_out/ab5/k14_$lib.log 2>&1 || exit 1
  TCAMD_X3F_V=1 timeout -k 10 120 python -u tools/x3_pair_bench.py --hw 56 --ks 64,224 --ldx 256 --chunks "" --iters 20 >> gpurun_out/ab5/k11_$lib.log 2>&1 || exit 1
  TCAMD_X3F_V=1 timeout -k 10 120 python -u tools/x3_pair_bench.py --hw 28 --ks 128,480 --ldx 512 --chunks "" --iters 20 >> gpurun_out/ab5/k11_$lib.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/fp32_engine_bench.py --batches 128 --streams 1,2 --engines fp32 --iters 20 >> gpurun_out/ab5/eng_$lib.log 2>&1 || exit 1
done; done
