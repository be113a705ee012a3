# K11w timing ablations (libraries from tools/probes/k11w_ablate.py), interleaved
# with the production build: v1 and v5 (K11w) per shape, bs128.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONPATH=$PWD
for r in 1 2; do
for v in prod ${K11W_ARMS:-noconv nomma1 no3x3}; do
  if [ $v = prod ]; then unset TCAMD_HIP_LIB; else export TCAMD_HIP_LIB=$PWD/k12ab/libtcamd_hip_k11w_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/k11x_ab.py --versions 1,5 --imgs 128 --shapes 56:64,56:224,28:480 --rounds 2 || exit 1
done
done
