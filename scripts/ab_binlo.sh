# A/B of the hybrid hash backward's coarse/binned level split (bench --bin-level-lo),
# two interleaved rounds per setting.  Usage: gpurun -- bash scripts/ab_binlo.sh tag "7 8 9 10"
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-abl}
mkdir -p "$OUT"
for rep in 1 2; do
  for v in ${2:-8 9}; do
    timeout -k 10 150 python3 bench.py --no-cpu-baseline --psnr-views 0 --infer-frames 0 --bin-level-lo $v \
        > "$OUT/lo${v}_r$rep.json" 2> "$OUT/lo${v}_r$rep.err"
  done
done
