mkdir -p gpurun_out/ab6
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_densenet_fp32_gpu.py -k "block7 or dense_small or engine" > gpurun_out/ab6/tests.log 2>&1 || exit 1
for r in 1 2 3; do for b7 in 0 1; do
  TCAMD_X3_BLOCK7=$b7 timeout -k 10 120 python -u tools/fp32_engine_bench.py --batches 128 --streams 1,2 --engines fp32 --iters 20 >> gpurun_out/ab6/eng_b7$b7.log 2>&1 || exit 1
done; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab6/trace -o fwd -- python3 tools/fp32_engine_bench.py --batches 128 --streams 1 --engines fp32 --iters 5 > gpurun_out/ab6/run.log 2>&1 || exit 1
