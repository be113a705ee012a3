set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 && \
bash tools/gpu_profile.sh --steps 30 --warmup 5 && \
python3 tools/summarize_prof.py gpurun_out/prof/server_kernel_stats.csv --top 20 > gpurun_out/prof_summary.md
