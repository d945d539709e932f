set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r3e; mkdir -p $OUT
for v in 32 16; do
  NGP_AMD_LIB=$PWD/ar-nerf_amd/lib/libngp_amd_cs$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vren_gpu.py -k chunk_segments > $OUT/t$v.log 2>&1
  tail -1 $OUT/t$v.log
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_trainer_gpu.py tests/test_golden_gpu.py tests/test_ddp_gpu.py tests/test_occupancy_gpu.py > $OUT/t_trainer.log 2>&1
tail -1 $OUT/t_trainer.log
cp ar-nerf_amd/trainer.py $OUT/new_trainer.py
for rep in 1 2 3; do
  for v in old 64 32 16; do
    if [ $v = old ]; then cp scripts/ab_alt/trainer.py ar-nerf_amd/trainer.py; unset NGP_AMD_LIB; else cp $OUT/new_trainer.py ar-nerf_amd/trainer.py; if [ $v = 64 ]; then unset NGP_AMD_LIB; else export NGP_AMD_LIB=$PWD/ar-nerf_amd/lib/libngp_amd_cs$v.so; fi; fi
    timeout -k 10 200 python -u bench.py --steps 1000 --warmup 10 --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
        --infer-frames 0 --breakdown-steps 20 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(sys.argv[2], round(d['value']/1e6,3), 'M rays/s', round(d['ms_per_step']*1e3,1), 'us/step', 'segments', k['segments']['avg_launch_ms'], k['segments']['launches_per_step'])" $OUT/${v}_$rep.json $v
  done
done
cp $OUT/new_trainer.py ar-nerf_amd/trainer.py
