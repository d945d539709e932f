# A/B of the encode's gather rounds (NGP_ENCODE_PG level pairs per round) and,
# with them, the chunk-round schedule. Usage: gpurun -- bash scripts/ab_encode_pg.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-pg}
mkdir -p "$OUT"
run() {  # name env...
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));c=d['config'];k=d['kernels'];print('$name', d['value'], d['ms_per_step'], c['field_evaluated_per_ray'], {n: (k[n]['avg_launch_ms'], k[n]['launches_per_step']) for n in ('hash_encode','field_mlp') if n in k})"
}
run pg1 NGP_ENCODE_PG=1
run pg2 NGP_ENCODE_PG=2
run pg4 NGP_ENCODE_PG=4
run pg2_r128 NGP_ENCODE_PG=2 NGP_CHUNK_ROUNDS=128
run pg4_r128 NGP_ENCODE_PG=4 NGP_CHUNK_ROUNDS=128
