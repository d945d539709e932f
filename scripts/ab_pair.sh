# A/B: one vs two steady-state steps per graph replay, alternating (bench lines); the data-parallel
# step emulated at world 1; then a kernel timeline.  Usage: gpurun -- bash scripts/ab_pair.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-pair}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {
    name=$1; shift
    timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
        --infer-frames 0 --breakdown-steps 20 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step')" "$OUT/$name.json" "$name"
}
for rep in 1 2 3; do
run single_$rep --no-pair-steps
run pair_$rep
done
run emulate_dp_1 --emulate-dp
run emulate_dp_2 --emulate-dp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/tr" -o run -f csv -- python3 bench.py --steps 100 --warmup 5 \
    --psnr-views 0 --no-cpu-baseline --breakdown-steps 1 --quality-steps 0 --infer-frames 0 > "$OUT/b.json" 2> "$OUT/b.err"
for b in 10 11; do python3 scripts/timeline.py "$OUT/tr/run_kernel_trace.csv" 20 $b; done > "$OUT/timeline.txt"
rm -rf "$OUT/tr"
