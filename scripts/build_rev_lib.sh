# Build libngp_amd.so from the sources of git revision REV into ar-nerf_amd/lib_NAME/ (A/B against an
# earlier tree; CPU side).  usage: bash scripts/build_rev_lib.sh NAME REV
set -e
NAME=$1; REV=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cd "$ROOT"
git archive "$REV" ar-nerf_amd/csrc include | tar -x -C "$T"
cd "$T/ar-nerf_amd"
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
      -munsafe-fp-atomics -c "$f" -o "$T/$(basename "$f" .hip).o" &
done
wait
mkdir -p "$ROOT/ar-nerf_amd/lib_$NAME"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/ar-nerf_amd/lib_$NAME/libngp_amd.so" "$T"/*.o
rm -rf "$T"
echo "built ar-nerf_amd/lib_$NAME/libngp_amd.so from $REV"
