#!/usr/bin/env bash
# Product-code variants of the persistent kernel for same-box timing (measurement only, never the
# product library): tools/_diag/pv_<name>/libstein_hip.so = the working tree's persistent.hip built
# with extra -D flags + the product objects of the other translation units
# (gradient-free-mcmc-postprocessing_amd/build/obj, from __graft_entry__.build()).  No stamps.
#   bash scripts/build_pvariants.sh "base:" "il4:-DST_ROW_IL=4"
# Time them with scripts/pv_run.sh (LD_LIBRARY_PATH selects the library tools/probe loads).
set -eu
cd "$(dirname "$0")/.."
CS=gradient-free-mcmc-postprocessing_amd/csrc
OBJ=gradient-free-mcmc-postprocessing_amd/build/obj
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FL="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC"
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  D=tools/_diag/pv_$name
  mkdir -p $D
  ( $HIPCC $FL $flags -c -o $D/persistent.o $CS/persistent.hip &&
    $HIPCC --offload-arch=gfx950 -shared -fPIC -o $D/libstein_hip.so $D/persistent.o \
      $(ls $OBJ/*.o | grep -v /persistent.o) ) &
done
wait
echo built "$@"
