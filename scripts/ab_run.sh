set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_abn.sh ab_seg0 3 "NGP_PREFETCH_AT=start" "NGP_PREFETCH_AT=after_seg0"
bash scripts/pmc_bench.sh 'hash|adam|field|composite|march' r2g "fetch write"
