# Round 6, fourth A/B: the guard stores moved after the publish record, the winner g row prefetched at the start of
# wave 1s chain -- the round-5 library, va (the previous step), the product build, and vr (+ the rows that repeat
# their predecessor skipped in the duplicate test)
set -o pipefail
mkdir -p gpurun_out/r06ab4
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06ab4/$name.json 2> gpurun_out/r06ab4/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06ab4/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06ab4/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'), d.get('near_tie_step'))"
}
for rep in 1 2; do
  for cfg in c2 c4r8 lv c4; do
    run ${cfg}_r05_$rep ST_HIP_LIB=ab/r05/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
    run ${cfg}_va_$rep ST_HIP_LIB=ab/va/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_vr_$rep ST_HIP_LIB=ab/vr/libstein_hip.so python3 bench.py --config $cfg $B
  done
done
