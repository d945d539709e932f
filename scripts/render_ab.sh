# A/B of the test-time march's wave-mode threshold (NGP_RENDER_WAVE_NS) on the
# same trained model state (fixed seeds): frame time per setting.
# Usage: gpurun -- bash scripts/render_ab.sh tag "16 8 4 2"
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-rab}
mkdir -p "$OUT"
for v in ${2:-16 8 4}; do
    NGP_RENDER_WAVE_NS=$v timeout -k 10 120 python3 scripts/render_profile.py --frames 20 > "$OUT/ns_$v.txt" 2> "$OUT/ns_$v.err"
done
