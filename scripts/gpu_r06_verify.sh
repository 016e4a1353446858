# Round 6: the shipped tree as the driver runs it -- GPU suite, smoke, and bench.py with no flags
set -o pipefail
mkdir -p gpurun_out/r06v
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r06v/gpu_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/r06v/gpu_tests.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06v/smoke.log 2>&1; rc=$?
tail -n 1 gpurun_out/r06v/smoke.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/r06v/bench.json 2> gpurun_out/r06v/bench.err; rc=$?
tail -n 1 gpurun_out/r06v/bench.json | cut -c1-400; exit $rc
