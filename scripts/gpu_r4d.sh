# Round 4: graph structure costs, per-step unit drift, and an A/B of every round-4 change against the
# round-3-equivalent configuration.  usage: gpurun -- bash scripts/gpu_r4d.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4d}; mkdir -p $OUT
timeout -k 10 120 python -u scripts/diag/graph_split_cost.py 20000 > $OUT/graph_split.json 2> $OUT/graph_split.err && cat $OUT/graph_split.json
timeout -k 10 120 python -u scripts/diag/graph_split_cost.py 2000 > $OUT/graph_split_short.json 2> $OUT/graph_split_short.err && cat $OUT/graph_split_short.json
timeout -k 10 300 python -u scripts/diag/units_drift.py > $OUT/units_drift.json 2> $OUT/units_drift.err
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); [print(w) for w in d['windows_20_steps_marched_composited_active_evaluated_loss']]" $OUT/units_drift.json
R3="NGP_FEM_LDS=1 NGP_STEP_TICKET=0 NGP_FUSED_COARSE=0"
bash scripts/ab_env.sh ${1:-r4d}/ab 2 "lib_r3|$R3|" "|NGP_FUSED_COARSE=0|" "lib_nr|NGP_FUSED_COARSE=0|" "lib_nm|NGP_FUSED_COARSE=0|" "lib_r3|NGP_FEM_LDS=1 NGP_FUSED_COARSE=0|" "lib_r3|NGP_STEP_TICKET=0 NGP_FUSED_COARSE=0|" "lib_b12|NGP_FUSED_COARSE=0|"
