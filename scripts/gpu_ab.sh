# A/B of bench.py under two environment settings, alternated (box noise).
# Usage: gpurun --timeout 900 -- bash scripts/gpu_ab.sh tag "ENV_A=.." "ENV_B=.." [rounds]
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; N=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/ab.txt"
for r in $(seq 1 "$N"); do
  for cfg in "$A" "$B"; do
    env $cfg timeout -k 10 200 python -u bench.py --no-cpu-baseline --psnr-views 0 --breakdown-steps 5 > "$OUT/one.json" 2> "$OUT/one.err"
    python3 -c "import json,sys; d=json.load(open('$OUT/one.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" "$cfg" >> "$OUT/ab.txt"
  done
done
