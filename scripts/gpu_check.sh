#!/usr/bin/env bash
# One GPU session: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel trace.
# Every GPU step runs under its own time limit; a crash / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|5) return 0 ;;            # pass / test failures / no tests: keep going
    *) echo "fatal rc=$rc in $name: stopping"; exit $rc ;;
  esac
}
MODE=${1:-all}
if [[ $MODE == all || $MODE == test ]]; then
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
fi
if [[ $MODE == ab ]]; then   # same-box A/B of the persistent kernel (scripts/build_ab.sh first)
  step ab 900 bash scripts/ab_run.sh
fi
if [[ $MODE == files ]]; then   # gpu_check.sh files <pytest args...>
  shift
  step pytest_files 1100 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread "$@"
fi
if [[ $MODE == all || $MODE == bench ]]; then
  step bench 900 python bench.py --steps 3 --warmup 1
fi
if [[ $MODE == all || $MODE == prof ]]; then
  step rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
fi
echo "=== done"
