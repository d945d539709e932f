# Alternating A/B/n of bench configurations, each "lib::flags" with lib = "" (the tree's
# ar-nerf_amd/lib/libngp_amd.so), "base" (ar-nerf_amd/lib_base/libngp_amd.so, built by
# scripts/build_base_lib.sh or by hand from a variant of the sources) or another directory
# name under ar-nerf_amd/ holding a variant's libngp_amd.so.
# gpurun -- bash scripts/ab_lib.sh TAG REPS "::" "base::" "::--no-defer-color" ...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for rep in $(seq 1 $REPS); do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    lib=${cfg%%::*}; flags=${cfg#*::}
    if [ "$lib" = base ]; then LIB=ar-nerf_amd/lib_base/libngp_amd.so
    elif [ -n "$lib" ]; then LIB=ar-nerf_amd/$lib/libngp_amd.so
    else LIB=ar-nerf_amd/lib/libngp_amd.so; fi
    NGP_AMD_LIB=$PWD/$LIB timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline \
        --quality-steps 0 --no-oracle-quality --psnr-views 0 --infer-frames 0 --breakdown-steps 20 $flags \
        > "$OUT/v${i}_$rep.json" 2> "$OUT/v${i}_$rep.err"
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels',{})
print('v'+sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step |',
      ' '.join(f'{n}={v[\"avg_launch_ms\"]*1e3:.1f}' for n, v in list(k.items())[:8]))" "$OUT/v${i}_$rep.json" "$i" "[$cfg]"
  done
done
