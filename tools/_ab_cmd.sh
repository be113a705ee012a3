mkdir -p gpurun_out/bert
timeout -k 10 900 python -u bench.py --model bert_large > gpurun_out/bert/bench_bert.json 2> gpurun_out/bert/bench_bert.err || exit 1
