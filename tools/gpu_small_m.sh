#!/bin/bash
# bs1 kernel durations of the fp32 engine (rocprofv3 kernel trace, cases split by idle gaps);
# the 3x3 also with TCAMD_X3_K9_DBG ablations (1 no MFMA, 4 no LDS operand reads, 7 skeleton).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONPATH=$PWD TMPDIR=/tmp
for D in 0 7; do
  rm -rf gpurun_out/smallm_$D
  TCAMD_X3_K9_DBG=$D timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/smallm_$D -o t -- \
    python3 tools/small_m_probe.py > gpurun_out/smallm_$D.log 2>&1 || exit 1
  echo "== TCAMD_X3_K9_DBG=$D"
  python3 tools/trace_groups.py $(find gpurun_out/smallm_$D -name '*kernel_trace.csv') || exit 1
done
