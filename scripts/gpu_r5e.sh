# Round 5: HIP graph queue mapping knobs of the runtime torch ships (cross-queue edges cost ~10 us each on the
# step's critical path, probe timeline r5d): default vs DEBUG_HIP_FORCE_GRAPH_QUEUES=1/2/3 and graph packet capture.
# usage: gpurun -- bash scripts/gpu_r5e.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-r5e}
bash scripts/ab_env.sh $T/ab 1 "||--steps 300" "|DEBUG_HIP_FORCE_GRAPH_QUEUES=1|--steps 300" \
    "|DEBUG_HIP_FORCE_GRAPH_QUEUES=2|--steps 300" "|DEBUG_HIP_FORCE_GRAPH_QUEUES=3|--steps 300" \
    "|DEBUG_CLR_GRAPH_PACKET_CAPTURE=1|--steps 300" "|DEBUG_CLR_GRAPH_PACKET_CAPTURE=0|--steps 300"
for f in gpurun_out/$T/ab/v*_1.json; do
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['probe_step_gaps_us']['gaps']); [print(f'  {k:18s} {v[0]:7.1f} {v[1]:7.1f}') for k, v in d['probe_timeline_us'].items()]" $f
done
