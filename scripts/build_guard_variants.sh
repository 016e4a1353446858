#!/usr/bin/env bash
# Measurement builds (never the product): the working tree's library with the persistent-kernel TUs recompiled
# under -D flags, into ab/<name>/libstein_hip.so; the other objects come from __graft_entry__.build().
# Usage: scripts/build_guard_variants.sh name:"-DFOO=1 -DBAR=2" ...
set -eu
cd "$(dirname "$0")/.."
CS=gradient-free-mcmc-postprocessing_amd/csrc
OBJ=gradient-free-mcmc-postprocessing_amd/build/obj
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
TUS="persistent persistent_guard persistent_small"
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p ab/$name/obj
  for tu in $TUS; do
    [[ -f $CS/$tu.hip ]] || continue
    $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC $flags -c -o ab/$name/obj/$tu.o $CS/$tu.hip &
    pids+=($!)
  done
done
for j in "${pids[@]}"; do wait "$j"; done
for spec in "$@"; do
  name=${spec%%:*}
  objs=()
  for o in $OBJ/*.o; do
    b=$(basename $o .o)
    if [[ -f ab/$name/obj/$b.o ]]; then objs+=(ab/$name/obj/$b.o); else objs+=($o); fi
  done
  $HIPCC --offload-arch=gfx950 -fPIC -shared -o ab/$name/libstein_hip.so "${objs[@]}"
  rm -rf ab/$name/obj
  echo "built ab/$name"
done
