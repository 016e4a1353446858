# Round 6, fifth A/B: the pruned plan set (mid-size compact-only, two-block, 10-row, 256-thread 8 / 16-row and
# 512-thread 6-row plans removed) against vr (the same guard code before pruning) and the round-5 library
set -o pipefail
mkdir -p gpurun_out/r06ab5
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06ab5/$name.json 2> gpurun_out/r06ab5/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06ab5/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06ab5/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; e=L.get('exact_arithmetic') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'), d.get('near_tie_step'), 'exact', e.get('ms_per_thin'))"
}
for rep in 1 2; do
  for cfg in lv c4 c2 c4r8; do
    run ${cfg}_r05_$rep ST_HIP_LIB=ab/r05/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_vr_$rep ST_HIP_LIB=ab/vr/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
  done
done
for c in 5 2; do   # the chains workload (batch launches of the LV chains' run starts)
  timeout -k 10 300 python3 bench.py --workload chains --chains $c --steps 3 --warmup 1 > gpurun_out/r06ab5/chains${c}_cur.json 2>/dev/null || exit 1
  timeout -k 10 300 env ST_HIP_LIB=ab/vr/libstein_hip.so python3 bench.py --workload chains --chains $c --steps 3 --warmup 1 > gpurun_out/r06ab5/chains${c}_vr.json 2>/dev/null || exit 1
  python3 -c "import json; [print('chains$c', v, json.loads(open(f'gpurun_out/r06ab5/chains${c}_{v}.json').read().strip().splitlines()[-1])['side_by_side_ms']) for v in ('cur','vr')]"
done
