set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONPATH=$PWD
for v in full stage; do
  if [ $v = stage ]; then export TCAMD_HIP_LIB=$PWD/k12ab/libtcamd_hip_k12stage.so; else unset TCAMD_HIP_LIB; fi
  for b in 1 8 64; do
    echo "== $v bs$b"; timeout -k 10 120 python -u tools/attn_probe.py --batch $b --k12-only || exit 1
  done
done
