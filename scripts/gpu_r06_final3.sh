# Round 6 final measurements (third pass: bounds slots + streamed sums in LDS under the guard): full GPU suite + smoke, the headline bench and its rocprofv3 kernel stats,
# the config-4 PMC traffic, and the thin workloads' bench lines (configs 2 / 3 / 5, one 8-GPU rank's shard,
# the LV call shape, the 5 LV chains).  Every GPU step has its own limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out/r06g3
export TMPDIR=/tmp
if [[ -z "$SKIP_SUITE" ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r06g3/gpu_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06g3/gpu_tests.log; [[ $rc == 0 ]] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06g3/smoke.log 2>&1; rc=$?
  tail -n 2 gpurun_out/r06g3/smoke.log; [[ $rc == 0 ]] || exit $rc
fi
step() {   # step <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/r06g3/$name.json" 2> "gpurun_out/r06g3/$name.err"
  local rc=$?
  [[ $rc == 0 ]] || { echo "$name rc=$rc"; tail -n 20 "gpurun_out/r06g3/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/r06g3/$name.json" | cut -c1-200
}
[[ -n "$SKIP_C4" ]] || step bench_c4 400 python3 bench.py
[[ -n "$SKIP_C4" ]] || step bench_c4_under_rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/r06g3/prof_c4 -o trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
[[ -n "$SKIP_PMC" ]] || PMC_STEPS=5 PMC_WARMUP=1 PMC_SOURCE="round 6 final run (scripts/gpu_r06_final.sh), 5 timed + 1 warm-up thin per pass" \
  bash scripts/pmc_workloads.sh ${PMC_KEYS:-c4_persistent} > gpurun_out/r06g3/pmc.log 2>&1 || { tail -n 30 gpurun_out/r06g3/pmc.log; exit 1; }
step bench_c2 300 python3 bench.py --config c2 --steps 20 --warmup 3
step bench_c3 300 python3 bench.py --config c3 --steps 20 --warmup 3
step bench_c4r8 300 python3 bench.py --config c4r8 --steps 10 --warmup 2
step bench_c5 400 python3 bench.py --config c5 --steps 3 --warmup 1
step bench_lv_call 400 python3 bench.py --config lv --steps 5 --warmup 1
step bench_chains 400 python3 bench.py --workload chains
echo "=== done"
