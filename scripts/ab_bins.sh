# A/B of the hash-backward level split and coarse-level run merging (bench lines + kernel breakdown).
# Usage: gpurun -- bash scripts/ab_bins.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
TAG=${1:-bins}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {
    name=$1; shift
    timeout -k 10 200 python -u bench.py --steps 400 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
        --infer-frames 0 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 - "$OUT/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d["kernels"]
print(f"{sys.argv[2]:24s} {d['value']/1e6:7.3f} M rays/s {d['ms_per_step']*1e3:7.1f} us/step | " +
      " ".join(f"{k}={v['avg_launch_ms']*1e3:.0f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1]['ms_per_step'])[:8]))
PY
}
for rep in 1 2; do
run default_$rep
run lo0_m8_$rep --bin-level-lo 0 --bin-merge-hi 8
run lo0_m10_$rep --bin-level-lo 0 --bin-merge-hi 10
run lo4_m8_$rep --bin-level-lo 4 --bin-merge-hi 8
run lo6_m8_$rep --bin-level-lo 6 --bin-merge-hi 8
done
