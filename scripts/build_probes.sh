#!/usr/bin/env bash
# Build the measurement probes (not product code): tools/probe against the product library, and
# ab/diag/probe_stamps against a diagnostic copy of the library built with -DST_PERSIST_STAMPS (ab/ ships
# to the GPU box; it is git-ignored).
set -eu
cd "$(dirname "$0")/.."
LIB=gradient-free-mcmc-postprocessing_amd/stein_thinning/_lib
CS=gradient-free-mcmc-postprocessing_amd/csrc
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe tools/probe.hip -L$LIB -lstein_hip -Wl,-rpath,'$ORIGIN/../'$LIB
OUT=ab/diag
mkdir -p $OUT/obj
pids=()
for f in $CS/*.hip $CS/*.cpp; do
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -DST_PERSIST_STAMPS ${STAMP_FLAGS:-} \
    -c -o $OUT/obj/$(basename ${f%.*}).o $f &
  pids+=($!)
done
for j in "${pids[@]}"; do wait "$j"; done
$HIPCC --offload-arch=gfx950 -fPIC -shared -o $OUT/libstein_hip.so $OUT/obj/*.o
rm -rf $OUT/obj
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -DST_PERSIST_STAMPS -o $OUT/probe_stamps tools/probe.hip \
  -L$OUT -lstein_hip -Wl,-rpath,'$ORIGIN'
echo built
