# round check: the whole GPU suite, smoke, the default bench (each step time-limited, chained)
mkdir -p gpurun_out/rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/rc/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/rc/bench.json 2> gpurun_out/rc/bench.err || exit 1
