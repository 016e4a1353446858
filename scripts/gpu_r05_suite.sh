# Round 5: the new GPU tests first (fail fast), the whole GPU suite, then one default bench line
set -o pipefail
mkdir -p gpurun_out/r05s
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_device_tensors.py tests/test_gpu_near_tie.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r05s/new_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r05s/new_tests.log; [[ $rc == 0 ]] || exit $rc
if [[ -z "$SKIP_SUITE" ]]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05s/gpu_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r05s/gpu_tests.log; [[ $rc == 0 ]] || exit $rc
fi
timeout -k 10 600 python3 bench.py > gpurun_out/r05s/bench.json 2> gpurun_out/r05s/bench.err; rc=$?; tail -c 600 gpurun_out/r05s/bench.json; exit $rc
