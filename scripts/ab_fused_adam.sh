# A/B: FusedAdam of the binned levels inside their accumulation (default),
# + the MLP/coarse Adam on the side stream after the coarse levels
# (NGP_ADAM_SPLIT=1), and one Adam launch after the backward (NGP_FUSED_ADAM=0).
# Usage: gpurun -- bash scripts/ab_fused_adam.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-fa}
mkdir -p "$OUT"
run() {  # name env...
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_bwd_coarse','hash_write','hash_accum','adam') if n in k})"
}
run fused NGP_FUSED_ADAM=1 NGP_ADAM_SPLIT=0
run fused_split NGP_FUSED_ADAM=1 NGP_ADAM_SPLIT=1
run separate NGP_FUSED_ADAM=0 NGP_ADAM_SPLIT=0
run fused2 NGP_FUSED_ADAM=1 NGP_ADAM_SPLIT=0
run fused_split2 NGP_FUSED_ADAM=1 NGP_ADAM_SPLIT=1
