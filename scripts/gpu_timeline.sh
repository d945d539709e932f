# Graph-mode kernel timeline of the bench's steady-state steps.
# Usage: gpurun --timeout 600 -- bash scripts/gpu_timeline.sh tag [bench args]
# (BACKS="130 131": steps counted from the end; the last --steps steps are the stamped roofline region)
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-tl}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o run -f csv -- python3 bench.py --steps 100 --warmup 5 \
    --psnr-views 0 --no-cpu-baseline --breakdown-steps 1 "$@" > "$OUT/b.json" 2> "$OUT/b.err"
for b in ${BACKS:-10 11 12}; do python3 scripts/timeline.py "$OUT/tr/run_kernel_trace.csv" 20 $b; done > "$OUT/timeline.txt"
rm -rf "$OUT/tr"
