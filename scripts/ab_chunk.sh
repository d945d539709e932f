# A/B of the chunked field evaluation's first-round width (NGP_CHUNK_FIRST):
# fewer first-round samples per row = fewer evaluated samples, one more list pass.
# Usage: gpurun -- bash scripts/ab_chunk.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-chunk}
mkdir -p "$OUT"
run() {  # name env...
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));c=d['config'];k=d['kernels'];print('$name', d['value'], d['ms_per_step'], c['field_evaluated_per_ray'], {n: k[n]['ms_per_step'] for n in ('hash_encode','field_mlp','segments','chunk_rest','mlp_bwd') if n in k})"
}
for c in 64 32 16 24; do run chunk$c NGP_CHUNK_FIRST=$c; done
