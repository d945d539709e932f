# One GPU-box pass: parity tests, smoke, bench line, rocprof kernel stats.
# Usage (from this container): gpurun --timeout 1100 -- bash scripts/gpu_check.sh [tag]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -f csv -- python3 bench.py --steps 100 --warmup 5 --psnr-views 0 --no-cpu-baseline --infer-frames 0 --quality-steps 0 > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.err"
python3 scripts/kstats.py "$OUT/trace/run_kernel_trace.csv" 100 "$OUT/kstats.csv" > "$OUT/kstats.txt"
