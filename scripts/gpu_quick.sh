# Quick GPU pass: GPU tests + one bench line without the CPU baseline.
# Usage: gpurun --timeout 900 -- bash scripts/gpu_quick.sh tag [extra bench args]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-quick}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --psnr-views 0 --quality-steps 0 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
