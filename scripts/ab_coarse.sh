# A/B of where the coarse levels' atomic hash backward overlaps: beside the
# binned record write + accumulation (default), beside the accumulation only
# (NGP_COARSE_AFTER_WRITE=1), or not at all (NGP_BWD_OVERLAP=0).
# Usage: gpurun -- bash scripts/ab_coarse.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-coarse}
mkdir -p "$OUT"
run() {  # name env...
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_bwd_coarse','hash_write','hash_accum','adam','mlp_bwd') if n in k})"
}
run default NGP_COARSE_AFTER_WRITE=0
run after_write NGP_COARSE_AFTER_WRITE=1
run serial NGP_BWD_OVERLAP=0
run after_write2 NGP_COARSE_AFTER_WRITE=1
run default2 NGP_COARSE_AFTER_WRITE=0
