# Round 6: same-box A/B of the guard rework -- the round-5 library (ab/r05, scripts/build_rev.sh) against
# the working tree's, alternating, on the bench legs (all rows unguarded = value, all rows guarded, the
# drop-in's run starts, exact); plus the unguarded 8-register-row compact-only kernel and the exact
# general kernel at 6 register rows
set -o pipefail
mkdir -p gpurun_out/r06ab
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06ab/$name.json 2> gpurun_out/r06ab/$name.err || { echo "FAIL $name"; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06ab/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; e=L.get('exact_arithmetic') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'), d.get('near_tie_step'), 'exact', e.get('ms_per_thin'))"
}
for rep in 1 2; do
  for cfg in c4 lv c2 c4r8; do
    run ${cfg}_r05_$rep ST_HIP_LIB=ab/r05/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
  done
done
run c4_cur_rt8 ST_TUNE=12=8 python3 bench.py --config c4 $B
run c4_cur_gen6 ST_TUNE=3=6 python3 bench.py --config c4 $B
run c4_cur_gen4 ST_TUNE=3=4 python3 bench.py --config c4 $B
