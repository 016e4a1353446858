# Round 6: the guarded all-row config-4 thin under the persistent kernel's run-time knobs (st_tune via ST_TUNE):
# streamed rows' sums in LDS (15=1), first-poll delay (16), the compact-only kernel's register rows (12=9),
# record replicas (10) -- timed as the headline leg (--headline-guard), two repetitions, one box
set -o pipefail
mkdir -p gpurun_out/r06i
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e --headline-guard"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/r06i/$name.json 2> gpurun_out/r06i/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/r06i/$name.err; exit 1; }
  python3 -c "import json,sys; L=json.loads(open('gpurun_out/r06i/$name.json').read().strip().splitlines()[-1]); print('$name', round(L['ms_per_step'],4), L['roofline']['kernel'])"
}
for rep in 1 2; do
  run base_$rep python3 bench.py --config c4 $B
  run sal1_$rep ST_TUNE=15=1 python3 bench.py --config c4 $B
  run delay0_$rep ST_TUNE=16=0 python3 bench.py --config c4 $B
  run delay20_$rep ST_TUNE=16=20 python3 bench.py --config c4 $B
  run rt9_$rep ST_TUNE=12=9 python3 bench.py --config c4 $B
  run rep16_$rep ST_TUNE=10=16 python3 bench.py --config c4 $B
  run rep4_$rep ST_TUNE=10=4 python3 bench.py --config c4 $B
done
