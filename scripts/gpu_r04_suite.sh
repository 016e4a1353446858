# full GPU test suite (one process), then smoke
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/gpu_tests.log 2>&1; rc=$?
tail -n 5 gpurun_out/r04/gpu_tests.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1; rc=$?; tail -n 2 gpurun_out/r04/smoke.log; exit $rc
