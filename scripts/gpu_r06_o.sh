# Round 6: guarded all-row config 4 with one LDS-row chain at a time (st_tune key 19 = 0) against the default
# two chains -- the guard's register pressure might favour the leaner form; one box, three repetitions
set -o pipefail
mkdir -p gpurun_out/r06o
export TMPDIR=/tmp
B="--steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-e2e --headline-guard"
for rep in 1 2 3; do
  for v in "" "19=0"; do
    timeout -k 10 300 env ${v:+ST_TUNE=$v} python3 bench.py --config c4 $B > gpurun_out/r06o/c4.json 2>/dev/null || exit 1
    python3 -c "import json; L=json.loads(open('gpurun_out/r06o/c4.json').read().strip().splitlines()[-1]); print('c4 guarded key', '${v:-default}', round(L['ms_per_step'],4))"
  done
done
