# Round 6: instruction mix of the MLP backward / forward kernels and the march (SQ_INSTS_VALU / MFMA / LDS, wave
# cycles) on the final tree
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/pmc_bench.sh 'field_bwd_mlp|field_first_chunk|field_encode_mlp_reg|march_slots|composite_loss' r6pmc "sqw lds"
cat gpurun_out/pmc_r6pmc/sqw.txt | cut -c1-220
cat gpurun_out/pmc_r6pmc/lds.txt | cut -c1-220
