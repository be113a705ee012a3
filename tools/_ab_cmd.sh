mkdir -p gpurun_out/ab2
timeout -k 10 300 python -u tools/bert_probe.py --batch 1 2 4 8 16 32 64 --iters 5 --rounds 3 --tunable gpurun_out/ab2/bert_large_gfx950.csv > gpurun_out/ab2/bert_tune.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bert_probe.py --batch 1 8 64 --iters 5 --rounds 3 --tuned-table gpurun_out/ab2/bert_large_gfx950.csv > gpurun_out/ab2/bert_table.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/k14x_bench.py --ks 512,992 --hw 14 --stamp --dbg 64 --rounds 1 > gpurun_out/ab2/timeline.log 2>&1 || exit 1
