# Iteration check on the GPU box: selected GPU tests, then a short bench line
# with the per-kernel breakdown.  Usage: gpurun -- bash scripts/gpu_iter.sh TAG "pytest args"
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-iter}
TESTS=${2:-tests/test_field_gpu.py tests/test_trainer_gpu.py}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 400 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["ms_per_step"]):
    print(f"  {k:20s} {v['avg_launch_ms']*1e3:8.1f} us x {v['launches_per_step']:.2f}")
PY
