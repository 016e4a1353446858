#!/usr/bin/env bash
# Profiling session: [bench] -> rocprofv3 kernel trace/stats of the timed bench -> PMC passes (one
# counter group each).  Every step must exit 0 (bench.py runs with faulthandler on, so a crash
# leaves its Python stack in the step's log); the first failure ends the script.
#   bash scripts/gpu_prof.sh <config> [full|trace|pmc] [extra bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${1:-c4}
MODE=${2:-full}
shift $(( $# > 2 ? 2 : $# ))
EXTRA=("$@")
run() {   # run <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  [[ $rc == 0 ]] || exit $rc
}
if [[ $MODE == full ]]; then
  run bench_$CFG 600 python3 bench.py --config $CFG --steps 5 --warmup 2 "${EXTRA[@]}"
fi
if [[ $MODE == full || $MODE == trace ]]; then
  run trace_$CFG 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$CFG -o trace -- \
    python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline "${EXTRA[@]}"
fi
if [[ $MODE == full || $MODE == pmc ]]; then
  run pmc_fetch_$CFG 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$CFG -o pmc -- \
    python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing "${EXTRA[@]}"
  run pmc_write_$CFG 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$CFG -o pmc -- \
    python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing "${EXTRA[@]}"
fi
echo "=== done"
