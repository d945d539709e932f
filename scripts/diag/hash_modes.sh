# Coarse atomic hash backward under its diagnostic modes (0 product, 1 no
# atomics, 2 plain stores, 3 no run merge): stages.py per-level timings.
set -e
cd "$GRAFT_REPO_ROOT"
for m in ${MODES:-0 1 3}; do
  echo "mode $m"
  NGP_HASH_BWD_MODE=$m PRETRAIN=1000 timeout -k 10 200 python scripts/diag/stages.py 2>/dev/null | tail -1
done
