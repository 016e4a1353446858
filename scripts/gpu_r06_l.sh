# Round 6: config 3 (gradient-free) -- the guard's fixed / per-step split, and the guarded thin with 2 register
# rows per thread (st_tune key 3 = 2: the rest of the 782 rows per block in LDS)
set -o pipefail
mkdir -p gpurun_out/r06l
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/guard_fixed_cost.py c3 c2 > gpurun_out/r06l/fixed.log 2>&1 || { tail -5 gpurun_out/r06l/fixed.log; exit 1; }
grep -E "^c" gpurun_out/r06l/fixed.log
B="--steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-e2e --headline-guard"
for rep in 1 2; do
  for v in "" "3=2" "3=1"; do
    timeout -k 10 300 env ${v:+ST_TUNE=$v} python3 bench.py --config c3 $B > gpurun_out/r06l/c3_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; L=json.loads(open('gpurun_out/r06l/c3_$rep.json').read().strip().splitlines()[-1]); print('c3 guarded key', '${v:-auto}', round(L['ms_per_step'],4), L['roofline']['kernel'])"
  done
done
