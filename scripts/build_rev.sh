#!/usr/bin/env bash
# Same-box A/B timing (measurement only, never the product): build libstein_hip.so from a git revision's
# csrc/ + include/ into ab/<name>/ (git-ignored, shipped to the GPU box), one object per source in
# parallel like __graft_entry__.build(); load it in a GPU call with ST_HIP_LIB=ab/<name>/libstein_hip.so.
set -eu
REV=${1:-HEAD}
NAME=${2:-$REV}
cd "$(dirname "$0")/.."
OUT=ab/$NAME
SRC=$OUT/src
rm -rf "$OUT" && mkdir -p "$SRC/pkg/csrc" "$SRC/include" "$OUT/obj"
for f in $(git ls-tree --name-only "$REV" gradient-free-mcmc-postprocessing_amd/csrc/); do
  git show "$REV:$f" > "$SRC/pkg/csrc/$(basename "$f")"
done
git show "$REV:include/stein_thinning_hip.h" > "$SRC/include/stein_thinning_hip.h"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
objs=()
pids=()
for f in "$SRC"/pkg/csrc/*.hip "$SRC"/pkg/csrc/*.cpp; do
  o="$OUT/obj/$(basename "${f%.*}").o"
  objs+=("$o")
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -c -o "$o" "$f" &
  pids+=($!)
done
for j in "${pids[@]}"; do wait "$j"; done
$HIPCC --offload-arch=gfx950 -fPIC -shared -o "$OUT/libstein_hip.so" "${objs[@]}"
rm -rf "$OUT/obj" "$SRC"
echo "built ab/$NAME/libstein_hip.so from $REV"
