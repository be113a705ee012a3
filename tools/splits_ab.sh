export PYTHONPATH=$PWD HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for ms in 0 16 8 4 2; do
  if [ $ms = 0 ]; then unset TCAMD_X3_MAX_SPLITS; else export TCAMD_X3_MAX_SPLITS=$ms; fi
  echo "== max_splits $ms" >> gpurun_out/splits_ab.log
  timeout -k 10 200 python tools/fp32_engine_bench.py --engines fp32 --batches 1,2,8 --streams 1 --iters 30 >> gpurun_out/splits_ab.log 2>&1 || exit 1
done
