# Round 5: the near-tie guard -- its GPU tests, the full GPU suite, then a same-box A/B of the headline and
# config-2 thins against the round-4 library (tools/ab/r04, built from HEAD~ sources; guard off there).
set -o pipefail
mkdir -p gpurun_out/r05g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_near_tie.py ${EXTRA_TESTS} -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r05g/near_tie_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r05g/near_tie_tests.log; [[ $rc == 0 ]] || exit $rc
if [[ -z "$SKIP_SUITE" ]]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05g/gpu_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r05g/gpu_tests.log; [[ $rc == 0 ]] || exit $rc
fi
ab() {   # ab <tag> <config> <steps>
  local tag=$1 cfg=$2 steps=$3
  for r in 1 2; do
    ST_NEAR_TIE=${GUARD_A:-0} ST_HIP_LIB=${AB_LIB:-tools/ab/r04/libstein_hip.so} timeout -k 10 300 python3 bench.py --config $cfg \
      --steps $steps --warmup 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/r05g/${tag}_A$r.json 2> gpurun_out/r05g/${tag}_A$r.err || return 1
    ST_NEAR_TIE=${GUARD_B:-1} timeout -k 10 300 python3 bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline --no-kernel-timing \
      > gpurun_out/r05g/${tag}_B$r.json 2> gpurun_out/r05g/${tag}_B$r.err || return 1
  done
  for f in ${tag}_A1 ${tag}_B1 ${tag}_A2 ${tag}_B2; do
    python3 -c "import json; d=json.loads(open('gpurun_out/r05g/$f.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', round(d['ms_per_step'],4), r.get('kernel_median_us'), (d.get('dedup') or {}).get('near_tie_step'), (d.get('dedup') or {}).get('thin_s'), (d.get('end_to_end') or {}).get('thin_host_arrays_s'))"
  done
}
for spec in ${AB:-c4:20 c2:30}; do ab ${spec%%:*} ${spec%%:*} ${spec##*:} || exit 1; done
echo done
