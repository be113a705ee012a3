mkdir -p gpurun_out/bert
for t in 0 1; do
  TC_BERT_TUNED_GEMMS=$t timeout -k 10 600 python -u bench.py --model bert_large > gpurun_out/bert/bench_bert_t$t.json 2> gpurun_out/bert/bench_bert_t$t.err || exit 1
done
