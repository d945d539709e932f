# Alternating A/B/n of the bench under configurations "LIBDIR|ENV|FLAGS" (LIBDIR "" = ar-nerf_amd/lib,
# else ar-nerf_amd/LIBDIR; ENV = space-separated VAR=value; FLAGS = extra bench.py flags), one line per run.
# gpurun -- bash scripts/ab_env.sh TAG REPS "||" "|NGP_FEM_LDS=1|" "lib_w4||" ...
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
    lib=$(echo "$cfg" | cut -d'|' -f1); envs=$(echo "$cfg" | cut -d'|' -f2); flags=$(echo "$cfg" | cut -d'|' -f3)
    LIB=ar-nerf_amd/lib/libngp_amd.so
    [ -n "$lib" ] && LIB=ar-nerf_amd/$lib/libngp_amd.so
    env NGP_AMD_LIB=$PWD/$LIB $envs timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline \
        --quality-steps 0 --no-oracle-quality --psnr-views 0 --infer-frames 0 --dropin-steps 0 --breakdown-steps 20 $flags \
        > "$OUT/v${i}_$rep.json" 2> "$OUT/v${i}_$rep.err"
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels',{})
print('v'+sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step', 'host', round(d.get('host_enqueue_ms_per_step', 0)*1e3,1), '|',
      ' '.join(f'{n}={v[\"avg_launch_ms\"]*1e3:.1f}' for n, v in list(k.items())[:8]), '| probes', ' '.join(f'{m}={t*1e3:.1f}' for o in d.get('ops', {}).values() for m, t in o.get('kernel_ms', {}).items()))" "$OUT/v${i}_$rep.json" "$i" "[$cfg]"
  done
done
