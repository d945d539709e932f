# A/B: Adam of the MLP + coarse levels on the side stream right after the
# coarse hash backward (beside the LDS-bound fine-level accumulation) vs one
# Adam after the join.  Usage: gpurun -- bash scripts/ab_adam_split.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-adam}
mkdir -p "$OUT"
run() {  # name env...
    name=$1; shift
    env "$@" timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_bwd_coarse','hash_write','hash_accum','adam') if n in k})"
}
run default NGP_ADAM_SPLIT=0
run split NGP_ADAM_SPLIT=1
run default2 NGP_ADAM_SPLIT=0
run split2 NGP_ADAM_SPLIT=1
