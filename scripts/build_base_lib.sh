# Build libngp_amd.so from a git revision's csrc/ (default HEAD) into ar-nerf_amd/lib_base/, for
# A/B runs of a kernel change against it (scripts/ab_lib.sh).  CPU side: run here, not on the box.
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
mkdir -p "$TMP/ar-nerf_amd/csrc" "$TMP/include"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" ar-nerf_amd/csrc/); do git -C "$ROOT" show "$REV:$f" > "$TMP/$f"; done
git -C "$ROOT" show "$REV:include/ngp_amd.h" > "$TMP/include/ngp_amd.h"
git -C "$ROOT" show "$REV:ar-nerf_amd/Makefile" > "$TMP/ar-nerf_amd/Makefile"
make -s -C "$TMP/ar-nerf_amd" -j8
mkdir -p "$ROOT/ar-nerf_amd/lib_base"
cp "$TMP/ar-nerf_amd/lib/libngp_amd.so" "$ROOT/ar-nerf_amd/lib_base/libngp_amd.so"
rm -rf "$TMP"
echo "built $REV -> ar-nerf_amd/lib_base/libngp_amd.so"
