set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export PYTHONPATH=$PWD
for r in 1 2 3; do
  for b in 1 64; do
    for pad in 0 20 192; do
      echo "== bs$b pad$pad"; timeout -k 10 120 python -u tools/attn_probe.py --batch $b --k12-only --pad $pad || exit 1
    done
  done
done
