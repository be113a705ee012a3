#!/bin/bash
# Round-end style check: full GPU suite, smoke, default bench, bert_large sweep bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --model bert_large --steps 5 --warmup 1 > gpurun_out/bench_bert.log \
  2> gpurun_out/bench_bert.err || exit 1
