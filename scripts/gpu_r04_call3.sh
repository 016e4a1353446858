# Round 4 call 3: config-4 A/B (committed vs working tree: streamed rows' sums in LDS, own record
# region for the gated kernel), the full GPU suite (+ the LV call-shape and KSD per-pair tests), the
# stamps breakdown of the small-shard step, and the config-4 PMC traffic of the new kernel.
set -o pipefail
mkdir -p gpurun_out/r04
bash scripts/gpu_r04_c4_ab.sh || exit 1
bash scripts/gpu_r04_suite.sh || exit 1
for n in 200000 250000 2000000; do
  timeout -k 10 120 ./tools/_diag/probe_stamps $n p > gpurun_out/r04/stamps_$n.log 2>&1 || { echo "stamps $n failed"; tail gpurun_out/r04/stamps_$n.log; exit 1; }
done
grep -h "stamps\|sweep\|publish split\|compute split\|speculation" gpurun_out/r04/stamps_*.log
PMC_SOURCE="round 4 call 3 (streamed sums in LDS), scripts/pmc_workloads.sh c4_persistent" \
  bash scripts/pmc_workloads.sh c4_persistent > gpurun_out/r04/pmc_c4.log 2>&1; rc=$?; tail -n 20 gpurun_out/r04/pmc_c4.log; exit $rc
