# Round 4: rehearsal of the world > 1 bench path on one GPU -- two ranks sharing the card over gloo (RCCL refuses two
# ranks on one device), torchrun as the driver launches it.  usage: gpurun -- bash scripts/gpu_r4r.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4dp2}; mkdir -p $OUT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
    --infer-frames 0 --no-oracle-quality > $OUT/dp2.json 2> $OUT/dp2.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(d['n_gpus'], d['value'], d['ms_per_step'], c['parallelism'], c['row_forward'], c['march_fork'], c['last_loss'])" $OUT/dp2.json
