set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/pmc
PRETRAIN=200 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex march_slots_wave -d gpurun_out/pmc/a -o run -f csv -- python3 scripts/diag/march_rpw.py > gpurun_out/pmc/a.log 2>&1
