# A/B of where the next batch's march is forked onto the side stream
# (NGP_PREFETCH_AT). Usage: gpurun -- bash scripts/ab_prefetch.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-pf}
mkdir -p "$OUT"
run() {  # name env...
    name=$1_$RANDOM; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('mlp_bwd','hash_encode','march','hash_write') if n in k})"
}
for p in ${PF_LIST:-after_fwd start after_composite after_mlp_bwd after_fwd}; do run $p NGP_PREFETCH_AT=$p; done
