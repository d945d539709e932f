# Round 6 (third session): the trainer step's gradient against the oracle with and without the fp16
# gradient-storage model (calibration); the binned tile scan in one pass (v2, the tree) vs HEAD (v1).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6af
timeout -k 10 300 python -u scripts/diag/grad16_trainer.py > gpurun_out/r6af/grad16_trainer.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_field_gpu.py tests/test_trainer_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6af/pytest.log 2>&1
timeout -k 10 700 bash scripts/ab_lib.sh r6af 4 "base::" "::" > gpurun_out/r6af/ab.txt 2>&1
