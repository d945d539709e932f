set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/cap1; mkdir -p $OUT
for rep in 1 2; do
for cap in 0 256 512 1024; do
  if [ $cap = 0 ]; then export NGP_AMD_LIB=$PWD/ar-nerf_amd/lib/libngp_amd.so; else export NGP_AMD_LIB=$PWD/ar-nerf_amd/lib/libngp_amd_cap$cap.so; fi
  timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --breakdown-steps 20 > $OUT/c${cap}_$rep.json 2> $OUT/c${cap}_$rep.err
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print('cap', sys.argv[2], round(d['value']/1e6,3), round(d['ms_per_step']*1e3,1), 'coarse', round(k['hash_bwd_coarse']['avg_launch_ms']*1e3,1), 'write', round(k['hash_write']['avg_launch_ms']*1e3,1), 'accum', round(k['hash_accum']['avg_launch_ms']*1e3,1))" $OUT/c${cap}_$rep.json $cap
done; done
