# A/B: encode + MLP forward fused into one launch (NGP_FUSED_FIELD=1) vs two.
# Usage: gpurun -- bash scripts/ab_fused_field.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-ff}
mkdir -p "$OUT"
run() {  # name env...
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_encode','field_mlp','march') if n in k})"
}
for r in 1 2 3 4; do
    run split$r NGP_FUSED_FIELD=0
    run fused$r NGP_FUSED_FIELD=1
done
