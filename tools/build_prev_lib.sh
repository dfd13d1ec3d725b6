# Build libgasfm.so of a git revision (default HEAD) into gasfm_amd/libgasfm_<tag>.so, for same-box
# A/Bs of the working tree against it (tools/gpu_ab_libs.sh).  usage: tools/build_prev_lib.sh [rev] [tag]
set -e
REV=${1:-HEAD}; TAG=${2:-prev}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" gasfm_amd/csrc include | tar -x -C "$TMP"
OBJS=()
for src in "$TMP"/gasfm_amd/csrc/*.hip "$TMP"/gasfm_amd/csrc/*.cpp; do
  obj="$TMP/$(basename "$src").o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -c "$src" -o "$obj" &
  OBJS+=("$obj")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/gasfm_amd/libgasfm_$TAG.so" "${OBJS[@]}"
rm -rf "$TMP"
echo "$ROOT/gasfm_amd/libgasfm_$TAG.so"
