# Repeated-row path: the GPU dedup tests, the config-4 full-length parity test (now also through
# dedup), the multi-process sharded thins, then config 4 / 2 bench lines carrying the "dedup" object.
set -o pipefail
mkdir -p gpurun_out/r04d
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread ${DEDUP_TESTS:-tests/test_gpu_dedup.py "tests/test_gpu_parity.py::test_config4_full_length_bit_exact" tests/test_gpu_multiprocess.py} \
  > gpurun_out/r04d/tests.log 2>&1 || { tail -n 40 gpurun_out/r04d/tests.log; exit 1; }
tail -n 3 gpurun_out/r04d/tests.log
step() {   # step <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$tmo" "$@" > "gpurun_out/r04d/$name.json" 2> "gpurun_out/r04d/$name.err"
  local rc=$?
  [[ $rc == 0 ]] || { echo "$name rc=$rc"; tail -n 20 "gpurun_out/r04d/$name.err"; exit $rc; }
  tail -n 1 "gpurun_out/r04d/$name.json" | cut -c1-300
}
step bench_c4 400 python3 bench.py --no-cpu-baseline
step bench_c2 300 python3 bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline
echo "=== done"
