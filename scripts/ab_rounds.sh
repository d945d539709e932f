# A/B of the chunked field evaluation's round bounds (NGP_CHUNK_FIRST +
# NGP_CHUNK_ROUNDS): more rounds = fewer evaluated samples, more list passes.
# Usage: gpurun -- bash scripts/ab_rounds.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-rounds}
mkdir -p "$OUT"
run() {  # name env...
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));c=d['config'];k=d['kernels'];print('$name', d['value'], d['ms_per_step'], c['field_evaluated_per_ray'], {n: k[n]['ms_per_step'] for n in ('hash_encode','field_mlp','segments','chunk_rest') if n in k})"
}
run r64 NGP_CHUNK_FIRST=64 NGP_CHUNK_ROUNDS=
run r64_128 NGP_CHUNK_FIRST=64 NGP_CHUNK_ROUNDS=128
run r32_64_128 NGP_CHUNK_FIRST=32 NGP_CHUNK_ROUNDS=64,128
run r64_96_160 NGP_CHUNK_FIRST=64 NGP_CHUNK_ROUNDS=96,160
run r48_128 NGP_CHUNK_FIRST=48 NGP_CHUNK_ROUNDS=128
