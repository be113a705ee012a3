mkdir -p gpurun_out/bat
timeout -k 10 200 python -u tools/fp32_engine_bench.py --batches 128,192,256 --streams 1,2 --engines fp32 --iters 20 > gpurun_out/bat/engine.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-bf16 --steps 10 --max-batch-size 256 --preferred 256 > gpurun_out/bat/b256.json 2> gpurun_out/bat/b256.err || exit 1
timeout -k 10 400 python -u bench.py --no-bf16 --steps 10 --max-batch-size 192 --preferred 192 > gpurun_out/bat/b192.json 2> gpurun_out/bat/b192.err || exit 1
timeout -k 10 400 python -u bench.py --no-bf16 --steps 10 > gpurun_out/bat/b128.json 2> gpurun_out/bat/b128.err || exit 1
