# Round 6, third A/B: where the guarded small-shard plans lost 3-5 % -- the round-5 library, the product build
# (the winner's |g|^2 recorded at the step start by wave 1; wave 1 keeps only its register rows in the rescan),
# va (|g|^2 loaded in the late check as round 5 did) and vb (va, and wave 1 rescans LDS / streamed rows too)
set -o pipefail
mkdir -p gpurun_out/r06ab3
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06ab3/$name.json 2> gpurun_out/r06ab3/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06ab3/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06ab3/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'), d.get('near_tie_step'))"
}
for rep in 1 2; do
  for cfg in c2 c4r8 lv c4; do
    run ${cfg}_r05_$rep ST_HIP_LIB=ab/r05/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
    run ${cfg}_va_$rep ST_HIP_LIB=ab/va/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_vb_$rep ST_HIP_LIB=ab/vb/libstein_hip.so python3 bench.py --config $cfg $B
  done
done
