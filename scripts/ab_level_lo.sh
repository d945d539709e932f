# A/B of the hybrid hash backward's split level (levels < lo atomic, >= lo binned)
# with the binned levels' Adam fused into their accumulation.
# Usage: gpurun -- bash scripts/ab_level_lo.sh tag
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_${1:-lo}
mkdir -p "$OUT"
run() {  # name lo
    name=$1; lo=$2
    timeout -k 10 200 python -u bench.py --steps 600 --warmup 5 --psnr-views 0 --no-cpu-baseline \
      --infer-frames 0 --quality-steps 0 --breakdown-steps 50 --bin-level-lo $lo > "$OUT/$name.json" 2> "$OUT/$name.err"
    python3 -c "import json;d=json.load(open('$OUT/$name.json'));k=d['kernels'];print('$name', d['value'], d['ms_per_step'], {n: k[n]['ms_per_step'] for n in ('hash_bwd_coarse','hash_write','hash_accum','adam') if n in k})"
}
for r in 1 2; do for lo in 8 9 10 7; do run lo${lo}_$r $lo; done; done
