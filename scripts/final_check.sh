# Final-commit GPU check: the full GPU suite, smoke, a short bench line.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 400 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
