#!/usr/bin/env bash
# Build stamped diagnostic variants of the persistent kernel (measurement only, never the product
# library): tools/_diag/v_<name>/{libstein_hip.so,probe_stamps}, one per "name:-Dflags" argument.
#   bash scripts/build_variants.sh "k1:-DST_POLL_DEPTH=1" "k2:-DST_POLL_DEPTH=2 -DST_POLL_SPACING=70"
set -eu
cd "$(dirname "$0")/.."
CS=gradient-free-mcmc-postprocessing_amd/csrc
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FL="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -DST_PERSIST_STAMPS"
OBJ=tools/_diag/obj
mkdir -p $OBJ
for s in capi greedy pairwise proxy kde lv; do
  [[ $OBJ/$s.o -nt $CS/$s.hip ]] || $HIPCC $FL -c -o $OBJ/$s.o $CS/$s.hip &
done
[[ $OBJ/host_prep.o -nt $CS/host_prep.cpp ]] || $HIPCC $FL -c -o $OBJ/host_prep.o $CS/host_prep.cpp &
wait
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  D=tools/_diag/v_$name
  mkdir -p $D
  ( $HIPCC $FL $flags -c -o $D/persistent.o $CS/persistent.hip &&
    $HIPCC --offload-arch=gfx950 -shared -fPIC -o $D/libstein_hip.so $D/persistent.o $OBJ/*.o &&
    $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -DST_PERSIST_STAMPS -o $D/probe_stamps tools/probe.hip \
      -L$D -lstein_hip -Wl,-rpath,'$ORIGIN' ) &
done
wait
echo built "$@"
