# Round 4 final measurements (after the repeated-row path, the device-side standardisation and the two-chain LDS
# chunks): full GPU suite + smoke, the headline bench and its rocprofv3 kernel stats, the config-4 PMC traffic, and
# the other workloads' bench lines.  Every GPU step has its own limit; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out/r04f gpurun_out/r04d
export TMPDIR=/tmp
[[ -n "$SKIP_SUITE" ]] || bash scripts/gpu_r04_suite.sh || exit 1
step() {   # step <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/r04f/$name.json" 2> "gpurun_out/r04f/$name.err"
  local rc=$?
  [[ $rc == 0 ]] || { echo "$name rc=$rc"; tail -n 20 "gpurun_out/r04f/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/r04f/$name.json" | cut -c1-300
}
[[ -n "$SKIP_C4" ]] || step bench_c4 400 python3 bench.py
cd /tmp && cd "$GRAFT_REPO_ROOT"
[[ -n "$SKIP_C4" ]] || step bench_c4_under_rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f/prof_c4 -o trace -- \
  python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
[[ -n "$SKIP_PMC" ]] || PMC_SOURCE="round 4 final run (scripts/gpu_r04_final.sh): default kernel, 8 replicas, first-poll delay 10, two-chain LDS chunks" \
  bash scripts/pmc_workloads.sh ${PMC_KEYS:-c4_persistent energy lv2} > gpurun_out/r04f/pmc.log 2>&1 || { tail -n 30 gpurun_out/r04f/pmc.log; exit 1; }
[[ -n "$SKIP_C23" ]] || step bench_c2 300 python3 bench.py --config c2 --steps 20 --warmup 3
[[ -n "$SKIP_C23" ]] || step bench_c3 300 python3 bench.py --config c3 --steps 20 --warmup 3
step bench_c5 400 python3 bench.py --config c5 --steps 3 --warmup 1
step bench_lv_call 400 python3 bench.py --config lv --steps 5 --warmup 1
step bench_energy 400 python3 bench.py --workload energy
step bench_lv 400 python3 bench.py --workload lv
step bench_ksd_full 600 python3 bench.py --workload ksd --ksd-full --steps 2 --warmup 1 --no-cpu-baseline
step bench_proxy 300 python3 bench.py --workload proxy
echo "=== done"
