set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b3
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py > gpurun_out/b3/run$i.log 2>&1 || exit 1
  tail -1 gpurun_out/b3/run$i.log | cut -c1-120
done
