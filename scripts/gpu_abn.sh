# A/B/n of bench.py over several configurations, alternated (box noise).
# Each configuration: "ENV=.. ENV2=.. [:: bench args]".
# Usage: gpurun --timeout 900 -- bash scripts/gpu_abn.sh tag rounds "cfg1" "cfg2" ...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/ab.txt"
for r in $(seq 1 "$N"); do
  i=0
  for cfg in "$@"; do
    envs=${cfg%%::*}; args=""
    [[ "$cfg" == *::* ]] && args=${cfg#*::}
    env $envs timeout -k 10 200 python -u bench.py --no-cpu-baseline --psnr-views 0 --breakdown-steps 5 $args > "$OUT/one$i.json" 2> "$OUT/one$i.err"
    python3 -c "import json,sys; d=json.load(open('$OUT/one$i.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" "$cfg" >> "$OUT/ab.txt"
    i=$((i+1))
  done
done
