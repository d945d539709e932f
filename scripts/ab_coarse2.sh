# A/B (fused Adam): coarse atomic levels beside the record write (default) vs
# beside the accumulation only (NGP_COARSE_AFTER_WRITE=1).
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-co2}
mkdir -p "$OUT"
run() {
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_bwd_coarse','hash_write','hash_accum','adam') if n in k})"
}
for r in 1 2 3; do run default$r NGP_COARSE_AFTER_WRITE=0; run after_write$r NGP_COARSE_AFTER_WRITE=1; done
