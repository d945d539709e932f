# Kernel-trace profile of the timed bench region: python3 bench.py under rocprofv3 (stats per kernel).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_trace}
mkdir -p "$OUT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT" -o run -f csv -- python3 bench.py --steps 200 --warmup 10 --pretrain 2000 --psnr-views 0 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
