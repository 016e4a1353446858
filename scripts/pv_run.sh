#!/usr/bin/env bash
# Same-box timing of the product-code variants built by scripts/build_pvariants.sh: tools/probe's
# quick mode (q: the default persistent configuration, m = 1000) per variant, interleaved over two
# rounds, at n = 2e6 (config 4) and n = 2.5e5 (one rank of an 8-GPU config-4 run); PV_NS overrides.
#   bash scripts/pv_run.sh base il4 ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in ${PV_ROUNDS:-1 2}; do
  for n in ${PV_NS:-2000000 250000}; do
    for v in "$@"; do
      echo "## $v n=$n round $r"
      LD_LIBRARY_PATH=tools/_diag/pv_$v timeout -k 10 120 ./tools/probe $n q || exit 1
    done
  done
done
