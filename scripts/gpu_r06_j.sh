# Round 6: streamed rows' sums in LDS automatically under the near-tie guard (st_tune key 15 = -1) -- the
# parity and near-tie suites on it, then same-box A/B against HEAD (ab/s16: sums in HBM), with 9 register rows
# on top (key 12 = 9), guarded all-row config 4 as the timed leg; the multi-rank bounds pre-pass (slots) rides
# along in the multiprocess tests
set -o pipefail
mkdir -p gpurun_out/r06j
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_near_tie.py tests/test_gpu_multiprocess.py tests/test_gpu_parity.py \
    tests/test_gpu_golden_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06j/tests.log 2>&1 \
    || { echo "FAIL tests"; tail -30 gpurun_out/r06j/tests.log; exit 1; }
tail -n 1 gpurun_out/r06j/tests.log
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e --headline-guard"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06j/$name.json 2> gpurun_out/r06j/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06j/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06j/$name.json').read().strip().splitlines()[-1]); d=L.get('dedup') or {}; print('$name', round(L['ms_per_step'],4), 'dedup', d.get('thin_s'), 'same', d.get('same_indices_as_timed_run'))"
}
for rep in 1 2; do
  run c4g_head_$rep ST_HIP_LIB=ab/s16/libstein_hip.so python3 bench.py --config c4 $B
  run c4g_cur_$rep python3 bench.py --config c4 $B
  run c4g_rt9_$rep ST_TUNE=12=9 python3 bench.py --config c4 $B
  run c4g_nosal_$rep ST_TUNE=15=0 python3 bench.py --config c4 $B
done
