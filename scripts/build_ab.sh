#!/usr/bin/env bash
# A/B baseline for kernel experiments (measurement only, never the product): builds the library and
# tools/probe from a git revision's sources (default HEAD) into tools/_diag/ab/, so one GPU call can
# time the committed kernel and the working tree's side by side on the same box.
set -eu
REV=${1:-HEAD}
cd "$(dirname "$0")/.."
OUT=tools/_diag/ab
SRC=$OUT/src
PK=$SRC/gradient-free-mcmc-postprocessing_amd
rm -rf "$OUT" && mkdir -p "$PK/csrc" "$SRC/include" "$SRC/tools"
for f in $(git ls-tree --name-only "$REV" gradient-free-mcmc-postprocessing_amd/csrc/); do
  git show "$REV:$f" > "$PK/csrc/$(basename "$f")"
done
git show "$REV:include/stein_thinning_hip.h" > "$SRC/include/stein_thinning_hip.h"
git show "$REV:tools/probe.hip" > "$SRC/tools/probe.hip"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CS=$PK/csrc
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -o $OUT/libstein_hip.so \
  $CS/capi.hip $CS/greedy.hip $CS/persistent.hip $CS/pairwise.hip $CS/proxy.hip $CS/kde.hip $CS/lv.hip $CS/host_prep.cpp
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -I"$SRC/include" -o $OUT/probe "$SRC/tools/probe.hip" -L$OUT -lstein_hip -Wl,-rpath,'$ORIGIN'
echo "built A/B baseline from $REV"
