# Round 6: the guard's rescan layout now that the streamed sums are in LDS under the guard -- LDS / streamed
# rows rescanned by waves 1.. (rw1) or 3.. (rw3) instead of 2..; their loops unrolled 2x / 4x (u2 / u4); hsal =
# HEAD (91c955a), cur = the product (HEAD + unroll pragma 1).  Guarded all-row config 4 / config 2 / one rank.
set -o pipefail
mkdir -p gpurun_out/r06k
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e --headline-guard"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06k/$name.json 2> gpurun_out/r06k/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06k/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06k/$name.json').read().strip().splitlines()[-1]); print('$name', round(L['ms_per_step'],4))"
}
for rep in 1 2; do
  for cfg in c4 c4r8; do
    run ${cfg}_hsal_$rep ST_HIP_LIB=ab/hsal/libstein_hip.so python3 bench.py --config $cfg $B
    run ${cfg}_cur_$rep python3 bench.py --config $cfg $B
    for v in rw1 rw3 u2 u4; do
      run ${cfg}_${v}_$rep ST_HIP_LIB=ab/$v/libstein_hip.so python3 bench.py --config $cfg $B
    done
  done
done
