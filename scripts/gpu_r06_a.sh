# Round 6, first GPU call: the new / changed guard tests (fail fast), the multi-process file, one bench line
set -o pipefail
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_near_tie.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06a/near_tie.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06a/near_tie.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_multiprocess.py -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r06a/multiprocess.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06a/multiprocess.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err; rc=$?; tail -c 400 gpurun_out/r06a/bench.json; exit $rc
