#!/usr/bin/env bash
# Same-box A/B of the persistent kernel: A = tools/_diag/ab/probe (scripts/build_ab.sh), B = the
# working tree's tools/probe; mode r (record layouts, m = 1000) interleaved A B A B at n = 2e6, then
# A B at n = 2.5e5.  Output: gpurun_out/ab_{A,B}_{1,2,s}.log and a summary on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 ./tools/_diag/ab/probe 2000000 r > gpurun_out/ab_A_$r.log 2>&1 || exit 1
  timeout -k 10 120 ./tools/probe 2000000 r > gpurun_out/ab_B_$r.log 2>&1 || exit 1
done
timeout -k 10 120 ./tools/_diag/ab/probe 250000 r > gpurun_out/ab_A_s.log 2>&1 || exit 1
timeout -k 10 120 ./tools/probe 250000 r > gpurun_out/ab_B_s.log 2>&1 || exit 1
for f in ab_A_1 ab_B_1 ab_A_2 ab_B_2 ab_A_s ab_B_s; do
  echo "## $f"; grep -h "replicas=16\|replicas= 1 " gpurun_out/$f.log
done
