# A/B of the run-merged binned hash backward: all levels binned, merge levels [0, m)
# vs the hybrid default. Usage: gpurun -- bash scripts/ab_merge.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-merge}
mkdir -p "$OUT"
run() {  # name env... -- bench args
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 $BARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_bwd_coarse','hash_write','hash_accum','hash_count') if n in k})"
}
BARGS="" run hybrid NGP_BIN_MERGE_HI=0
for m in 8 12 16; do BARGS="--hash-backward binned" run binned_m$m NGP_BIN_MERGE_HI=$m; done
BARGS="" run hybrid_m8 NGP_BIN_MERGE_HI=8
