# Round 6: guard register pressure (duplicate tests one field at a time, row ibk in SGPRs, the winner's |g|^2
# from the sweep's winner row instead of four serial global loads; guarded general kernel at 4 register rows)
# -- near-tie tests, then same-box A/B against HEAD (ab/head) and the 2-rank rehearsal
set -o pipefail
mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_near_tie.py tests/test_gpu_multiprocess.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r06e/tests.log 2>&1 || { echo "FAIL tests"; tail -30 gpurun_out/r06e/tests.log; exit 1; }
tail -2 gpurun_out/r06e/tests.log
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06e/$name.json 2> gpurun_out/r06e/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06e/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06e/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'))"
}
for rep in 1 2; do
  for cfg in c4 c2 c4r8 lv; do
    run ${cfg}_head_$rep ST_HIP_LIB=ab/head/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
  done
done
R="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e --no-config5 --no-chains"
run c4_share2_g0 ST_BENCH_SHARE_DEVICE=1 python3 bench.py --config c4 --gpus 2 $R
run c4_share2_g1 ST_BENCH_SHARE_DEVICE=1 python3 bench.py --config c4 --gpus 2 $R --headline-guard
run c4_share2_g1_head ST_HIP_LIB=ab/head/libstein_hip.so ST_BENCH_SHARE_DEVICE=1 python3 bench.py --config c4 --gpus 2 $R --headline-guard
