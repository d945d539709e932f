# Round 5: hardware queues per process (GPU_MAX_HW_QUEUES, box default 4) x the graph executor's stream pool
# (DEBUG_HIP_FORCE_GRAPH_QUEUES).  usage: gpurun -- bash scripts/gpu_r5i.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5i}
mkdir -p gpurun_out/$T
bash scripts/ab_env.sh $T/ab 2 "||--steps 300" "|DEBUG_HIP_FORCE_GRAPH_QUEUES=3|--steps 300" \
    "|GPU_MAX_HW_QUEUES=3|--steps 300" "|GPU_MAX_HW_QUEUES=2|--steps 300" \
    "|GPU_MAX_HW_QUEUES=3 DEBUG_HIP_FORCE_GRAPH_QUEUES=2|--steps 300" "|GPU_MAX_HW_QUEUES=2 DEBUG_HIP_FORCE_GRAPH_QUEUES=1|--steps 300"
for f in gpurun_out/$T/ab/v*_1.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value']); [print(f'  {k:18s} {v[0]:7.1f} {v[1]:7.1f}') for k, v in d['probe_timeline_us'].items()]" $f
done
