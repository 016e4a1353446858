#!/usr/bin/env bash
# Build the measurement probes (not product code): tools/probe against the product library, and
# tools/_diag/probe_stamps against a diagnostic copy of the library built with -DST_PERSIST_STAMPS.
set -eu
ONLY=${1:-all}
cd "$(dirname "$0")/.."
LIB=gradient-free-mcmc-postprocessing_amd/stein_thinning/_lib
CS=gradient-free-mcmc-postprocessing_amd/csrc
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe tools/probe.hip -L$LIB -lstein_hip -Wl,-rpath,'$ORIGIN/../'$LIB
mkdir -p tools/_diag
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -DST_PERSIST_STAMPS \
  -o tools/_diag/libstein_hip.so $CS/capi.hip $CS/dedup.hip $CS/precon.hip $CS/greedy.hip $CS/persistent.hip \
  $CS/persistent_guard.hip $CS/persistent_small.hip $CS/persistent_cmp.hip $CS/pairwise.hip $CS/proxy.hip $CS/kde.hip $CS/lv.hip $CS/host_prep.cpp $CS/prep_upload.cpp
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -DST_PERSIST_STAMPS -o tools/_diag/probe_stamps tools/probe.hip \
  -Ltools/_diag -lstein_hip -Wl,-rpath,'$ORIGIN'
echo built
# proxy kernel probe: one binary per ST_PROXY_DIAG level (0 full, 1 no MFMA, 2 no grad stores, 3 neither)
for lv in 0 1 2 3; do
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DST_PROXY_DIAG=$lv -o tools/_diag/proxy_probe_$lv \
    tools/proxy_probe.cpp $CS/proxy.hip
done
echo built proxy probes
