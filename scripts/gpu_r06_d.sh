# Round 6: the guarded mid-size plan restored (compact-only kernel, 4 register rows, guard only) -- its
# near-tie tests, the LV call's guarded all-row thin against vr (pre-pruning library), and the multi-rank
# guard rehearsal (ranks sharing one GPU: config 4 on 2 and 4 ranks, guard off / on)
set -o pipefail
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_near_tie.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r06d/near_tie_tests.log 2>&1 || { echo "FAIL near-tie tests"; tail -30 gpurun_out/r06d/near_tie_tests.log; exit 1; }
tail -3 gpurun_out/r06d/near_tie_tests.log
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06d/$name.json 2> gpurun_out/r06d/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06d/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06d/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'), 'kernel', L['roofline']['kernel'] if L.get('roofline') else None)"
}
for rep in 1 2; do
  run lv_vr_$rep ST_HIP_LIB=ab/vr/libstein_hip.so python3 bench.py --config lv $B
  run lv_cur_$rep python3 bench.py --config lv $B
done
R="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e --no-config5 --no-chains"
for g in 2 4; do
  for rep in 1 2; do
    run c4_share${g}_g0_$rep ST_BENCH_SHARE_DEVICE=1 python3 bench.py --config c4 --gpus $g $R
    run c4_share${g}_g1_$rep ST_BENCH_SHARE_DEVICE=1 python3 bench.py --config c4 --gpus $g $R --headline-guard
  done
done
