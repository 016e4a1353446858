#!/usr/bin/env bash
# Profiling session: bench (full, with CPU baseline) -> kernel trace/stats -> PMC passes (one counter group each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-c4}
# run <name> <timeout> <cmd...>; rocprofv3 on this image may SIGSEGV in its own teardown after the
# output files are written (rc 139): accepted for profiler steps whose CSV exists (checked by the
# caller), any other failure stops the script.
run() {
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [[ $rc == 139 && $1 == rocprofv3 ]] && grep -q "Opened result file" "gpurun_out/$name.log"; then return 0; fi
  [[ $rc == 0 ]] || exit $rc
}
if [[ ${2:-full} == full ]]; then
  run bench_$CFG 900 python bench.py --config $CFG --steps 5 --warmup 2
fi
run trace_$CFG 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o trace -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline
run pmc_fetch_$CFG 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$CFG -o pmc -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing
run pmc_write_$CFG 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$CFG -o pmc -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing
echo "=== done"
