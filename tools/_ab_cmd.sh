mkdir -p gpurun_out/fwd
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fwd/trace -o fwd -- python3 tools/fp32_engine_bench.py --batches 128 --streams 1 --engines fp32 --iters 5 > gpurun_out/fwd/run.log 2>&1 || exit 1
for r in 1 2; do for pf in 3 6; do
  timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,512,992 --rounds 3 --pf $pf >> gpurun_out/fwd/k14_pf$pf.log 2>&1 || exit 1
done; done
