# Build libngp_amd.so from the tree's sources with -D defines into ar-nerf_amd/lib_NAME/ (A/B variants;
# CPU side).  usage: bash scripts/build_variant.sh NAME "-DNGP_FEM2_WAVES=4 ..."
set -e
NAME=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$(mktemp -d)
cd "$ROOT/ar-nerf_amd"
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-function \
      -munsafe-fp-atomics $DEFS -c "$f" -o "$B/$(basename "$f" .hip).o" &
done
wait
mkdir -p "lib_$NAME"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "lib_$NAME/libngp_amd.so" "$B"/*.o
rm -rf "$B"
echo "built ar-nerf_amd/lib_$NAME/libngp_amd.so ($DEFS)"
