# A/B of the production build against a scratch library in k12ab/ (built from
# another revision of a kernel source), interleaved rounds, one command:
#   bash tools/probes/lib_ab.sh <lib name in k12ab/> <python tool + args...>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONPATH=$PWD
alt=$1; shift
for r in 1 2; do
for v in prod alt; do
  if [ $v = prod ]; then unset TCAMD_HIP_LIB; else export TCAMD_HIP_LIB=$PWD/k12ab/$alt; fi
  echo "== $v"
  timeout -k 10 300 python -u "$@" || exit 1
done
done
