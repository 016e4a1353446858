# Round 6: the near-tie bounds' per-block atomics spread over 16 slots (ST_BOUNDS_SLOTS) against all on one
# address (ab/s0): the guard's fixed cost per launch (tools/guard_fixed_cost.py), its near-tie tests, and the
# bench legs
set -o pipefail
mkdir -p gpurun_out/r06h
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_near_tie.py tests/test_gpu_multiprocess.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r06h/tests.log 2>&1 || { echo "FAIL tests"; tail -30 gpurun_out/r06h/tests.log; exit 1; }
tail -n 1 gpurun_out/r06h/tests.log
timeout -k 10 300 env ST_HIP_LIB=ab/s0/libstein_hip.so python3 tools/guard_fixed_cost.py c2 c4r8 > gpurun_out/r06h/fixed_s0.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/guard_fixed_cost.py c2 c4r8 > gpurun_out/r06h/fixed_s16.log 2>&1 || exit 1
grep -E "^c" gpurun_out/r06h/fixed_s0.log | sed 's/^/s0  /'; grep -E "^c" gpurun_out/r06h/fixed_s16.log | sed 's/^/s16 /'
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06h/$name.json 2> gpurun_out/r06h/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06h/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06h/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'))"
}
for rep in 1 2; do
  for cfg in c2 c4r8 c4; do
    run ${cfg}_s0_$rep ST_HIP_LIB=ab/s0/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_s16_$rep python3 bench.py --config $cfg $B
  done
done
