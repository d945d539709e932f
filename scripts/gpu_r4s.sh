# Round 4: PMC of the MLP backward (SQ instruction mix and wait cycles), the round-3 form (lib_bwd3: no lane
# rematerialisation, unmasked exponents) and the round-4 default, one counter pass each (MI355X_MICROARCH.md).
# usage: gpurun -- bash scripts/gpu_r4s.sh TAG
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
NGP_AMD_LIB=$PWD/ar-nerf_amd/lib_bwd3/libngp_amd.so bash scripts/pmc_bench.sh 'field_bwd_mlp' ${1:-r4mlp}_r3 "sqw"
bash scripts/pmc_bench.sh 'field_bwd_mlp' ${1:-r4mlp}_r4 "sqw"
cat gpurun_out/pmc_${1:-r4mlp}_r3/sqw.txt; cat gpurun_out/pmc_${1:-r4mlp}_r4/sqw.txt
