set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/pmc_bench.sh 'field_encode|hash|field_bwd|adam|composite|march|segments' r3 "fetch write enc"
python3 scripts/pmc_traffic.py gpurun_out/pmc_r3 gpurun_out/pmc_r3/pmc_traffic.json
cat gpurun_out/pmc_r3/enc.txt | head -30
