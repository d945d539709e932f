# Round 6: rehearsal of the world > 1 bench path on one GPU with the round-6 tree (segmented step at world > 1,
# occupancy draws beside the step, the eager data-parallel update every 16 steps in the pretraining) -- two ranks
# sharing the card over gloo (RCCL refuses two ranks on one device), torchrun as the driver launches it.
# usage: gpurun -- bash scripts/gpu_r6dp2.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6dp2}; mkdir -p $OUT
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --no-cpu-baseline --quality-steps 0 --psnr-views 0 \
    --infer-frames 0 --no-oracle-quality --dropin-steps 0 > $OUT/dp2.json 2> $OUT/dp2.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(d['n_gpus'], d['value'], d['ms_per_step'], c.get('parallelism'), c.get('last_loss'), d.get('guard_hits'))" $OUT/dp2.json
