mkdir -p gpurun_out/ab
for r in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export TCAMD_HIP_LIB=$PWD/ab/libtcamd_hip_base.so; else unset TCAMD_HIP_LIB; fi
    timeout -k 10 120 python -u tools/fp32_engine_bench.py --batches 128 --streams 1,2 --engines fp32 --iters 20 >> gpurun_out/ab/eng_$lib.log 2>&1 || exit 1
    TCAMD_X3F_V=1 timeout -k 10 120 python -u tools/x3_pair_bench.py --hw 56 --ks 64,224 --ldx 256 --chunks "" --iters 20 >> gpurun_out/ab/k11_$lib.log 2>&1 || exit 1
    timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,992 --rounds 3 >> gpurun_out/ab/k14_$lib.log 2>&1 || exit 1
  done
done
unset TCAMD_HIP_LIB
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/ab/pmc1 -- python3 tools/k14x_bench.py --ks 992 --hw 14 --rounds 1 --iters 5 > gpurun_out/ab/pmc1.log 2>&1 || exit 1
TCAMD_X3F_V=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/ab/pmc2 -- python3 tools/x3_pair_bench.py --hw 56 --ks 64,224 --ldx 256 --chunks "" --iters 5 > gpurun_out/ab/pmc2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/ab/pmc3 -- python3 tools/k14x_bench.py --ks 992 --hw 14 --rounds 1 --iters 5 > gpurun_out/ab/pmc3.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,992 --hw 14 --stamp --dbg 64 --rounds 1 > gpurun_out/ab/timeline.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,992 --hw 14,7 --stamp --dbg 192 --rounds 3 > gpurun_out/ab/prio.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/k14x_bench.py --ks 256,992 --hw 14,7 --stamp --dbg 64 --rounds 3 > gpurun_out/ab/noprio.log 2>&1 || exit 1
for r in 1 2; do for sg in 0 1; do
  TCAMD_X3F_V=1 TCAMD_X3F_STAGGER=$sg timeout -k 10 120 python -u tools/x3_pair_bench.py --hw 56 --ks 64,128,224 --ldx 256 --chunks "" --iters 20 >> gpurun_out/ab/stg56_$sg.log 2>&1 || exit 1
  TCAMD_X3F_V=1 TCAMD_X3F_STAGGER=$sg timeout -k 10 120 python -u tools/x3_pair_bench.py --hw 28 --ks 128,256,480 --ldx 512 --chunks "" --iters 20 >> gpurun_out/ab/stg28_$sg.log 2>&1 || exit 1
done; done
for sg in 0 1; do TCAMD_X3F_STAGGER=$sg timeout -k 10 120 python -u tools/fp32_engine_bench.py --batches 128 --streams 1,2,3 --engines fp32 --iters 20 >> gpurun_out/ab/eng_stg$sg.log 2>&1 || exit 1; done
timeout -k 10 240 python -u tools/bert_probe.py --batch 64 --iters 5 --rounds 3 --tunable gpurun_out/ab/tunableop_b64.csv > gpurun_out/ab/bert_tun.log 2>&1 || exit 1
