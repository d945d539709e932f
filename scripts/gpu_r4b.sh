# Round 4: parity of the changed kernels + counters, the bench unit check, A/B of the new forms, graph join costs.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4b}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_field_gpu.py tests/test_vren_gpu.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 2 $OUT/pytest.log
# the 12-wave MLP backward variant: its parity tests
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_b12/libngp_amd.so timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py -x -q -k "backward" --timeout 120 --timeout-method thread > $OUT/pytest_b12.log 2>&1
tail -n 1 $OUT/pytest_b12.log
Q="--no-cpu-baseline --quality-steps 0 --psnr-views 0 --infer-frames 0 --no-oracle-quality"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $Q > $OUT/bench20.json 2> $OUT/bench20.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r['frac'], r['ms_per_step'], json.dumps(r['units_check']))" $OUT/bench20.json
timeout -k 10 120 python -u scripts/diag/graph_join_cost.py 20000 > $OUT/graph_join.json 2> $OUT/graph_join.err && cat $OUT/graph_join.json
timeout -k 10 120 python -u scripts/diag/graph_join_cost.py 2000 > $OUT/graph_join_short.json 2> $OUT/graph_join_short.err && cat $OUT/graph_join_short.json
bash scripts/ab_env.sh ${1:-r4b}/ab 2 "||" "|NGP_FUSED_COARSE=0|" "lib_b12||" "|NGP_STEP_TICKET=0|" "|NGP_FEM_LDS=1|" "lib_fl4||" "lib_fl8||"
