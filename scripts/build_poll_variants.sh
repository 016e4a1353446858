#!/usr/bin/env bash
# Build A/B libraries of the persistent kernels with other poll grids (ST_POLL_SYNC, s_memrealtime ticks of
# 10 ns; default 45) into tools/ab/ps<N>/ -- every other object from the product build.
set -eu
cd "$(dirname "$0")/.."
CS=gradient-free-mcmc-postprocessing_amd/csrc
O=gradient-free-mcmc-postprocessing_amd/build/obj
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FL="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall"
for ps in "$@"; do
  D=tools/ab/ps$ps; mkdir -p $D/obj
  for f in persistent persistent_guard persistent_small persistent_cmp; do
    $HIPCC $FL -DST_POLL_SYNC=$ps -c -o $D/obj/$f.o $CS/$f.hip &
  done
done
wait
for ps in "$@"; do
  D=tools/ab/ps$ps
  $HIPCC --offload-arch=gfx950 -fPIC -shared -o $D/libstein_hip.so $O/capi.o $O/dedup.o $O/precon.o $O/greedy.o \
    $D/obj/persistent.o $D/obj/persistent_guard.o $D/obj/persistent_small.o $D/obj/persistent_cmp.o $O/pairwise.o $O/proxy.o $O/kde.o $O/lv.o \
    $O/host_prep.o $O/prep_upload.o
  rm -rf $D/obj
done
echo built
