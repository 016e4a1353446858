# Round 6, second A/B: the lazy duplicate test + the winner's |g|^2 from the step's row (no load in the late
# check) against the round-5 library on the drop-in legs; the guarded all-row config 4 at 8 (default) and
# 9 (forced, st_tune key 12) register rows; then a 2-rank shared-GPU rehearsal of the N > 1 line
# (chains_over_gpus, rank_hop)
set -o pipefail
mkdir -p gpurun_out/r06ab2
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06ab2/$name.json 2> gpurun_out/r06ab2/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06ab2/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06ab2/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; e=L.get('exact_arithmetic') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'), d.get('near_tie_step'), 'exact', e.get('ms_per_thin'))"
}
for rep in 1 2; do
  run c4_cur_$rep python3 bench.py --config c4 $B
  run c4_rt9g_$rep ST_TUNE=12=9 python3 bench.py --config c4 $B
  for cfg in c2 c4r8 lv; do
    run ${cfg}_r05_$rep ST_HIP_LIB=ab/r05/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
  done
done
ST_BENCH_SHARE_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-config5 \
  > gpurun_out/r06ab2/rehearsal_n2.json 2> gpurun_out/r06ab2/rehearsal_n2.err; rc=$?
python3 -c "import json; L=json.loads(open('gpurun_out/r06ab2/rehearsal_n2.json').read().strip().splitlines()[-1]); print('n2', L['ms_per_step'], L['exchange'], L['rank_hop'] and L['rank_hop']['us_per_step'], L['chains_over_gpus'])" || tail -20 gpurun_out/r06ab2/rehearsal_n2.err
exit $rc
