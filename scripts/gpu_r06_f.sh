# Round 6: which of the guard's register-pressure changes cost time (call E: guarded config 4 10.57 -> 11.02 ms)
# -- same-box A/B of HEAD~1 (ab/head), the product (field-wise duplicate tests + |g_j|^2 from the sweep's row),
# each change alone (f1w0 / f0w1), neither (f0w0), and the product with the rescan loops unrolled 4x (u4)
set -o pipefail
mkdir -p gpurun_out/r06f_ab
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e"
run() {  # name, env..., then args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06f_ab/$name.json 2> gpurun_out/r06f_ab/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06f_ab/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06f_ab/$name.json').read().strip().splitlines()[-1]); g=L.get('near_tie_guard') or {}; d=L.get('dedup') or {}; print('$name', round(L['ms_per_step'],4), 'guard', g.get('ms_per_thin'), g.get('first_flagged_step'), 'dedup', d.get('thin_s'))"
}
for rep in 1 2; do
  for cfg in c4 c2 c4r8; do
    run ${cfg}_head_$rep ST_HIP_LIB=ab/head/libstein_hip.so python3 bench.py --config $cfg $B
    for v in f0w0 f1w0 f0w1 u4; do
      run ${cfg}_${v}_$rep ST_HIP_LIB=ab/$v/libstein_hip.so python3 bench.py --config $cfg $B
    done
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
  done
done
