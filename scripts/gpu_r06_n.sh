# Round 6: the 256-thread guarded kernels' wave-0 rescan after the pick instead of inside the first poll
# (ab/w0after, ST_LANES_W0_IN_POLL=0) against the product -- guarded tests on the variant, then the guard's
# fixed / per-step split and the guarded legs of configs 2 / 3 and one 8-GPU rank
set -o pipefail
mkdir -p gpurun_out/r06n
export TMPDIR=/tmp
timeout -k 10 600 env ST_HIP_LIB=ab/w0after/libstein_hip.so python -u -m pytest tests/test_gpu_near_tie.py \
    tests/test_gpu_small_shard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06n/tests.log 2>&1 \
    || { echo "FAIL tests"; tail -30 gpurun_out/r06n/tests.log; exit 1; }
tail -n 1 gpurun_out/r06n/tests.log
timeout -k 10 300 env ST_HIP_LIB=ab/w0after/libstein_hip.so python3 tools/guard_fixed_cost.py c2 c3 c4r8 > gpurun_out/r06n/fixed_w0after.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/guard_fixed_cost.py c2 c3 c4r8 > gpurun_out/r06n/fixed_cur.log 2>&1 || exit 1
grep -E "^c" gpurun_out/r06n/fixed_w0after.log | sed 's/^/w0after /'; grep -E "^c" gpurun_out/r06n/fixed_cur.log | sed 's/^/cur     /'
B="--steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-e2e --headline-guard"
for rep in 1 2; do
  for cfg in c2 c3 c4r8; do
    for v in cur w0after; do
      if [[ $v == cur ]]; then E="X=1"; else E="ST_HIP_LIB=ab/w0after/libstein_hip.so"; fi
      timeout -k 10 300 env $E python3 bench.py --config $cfg $B > gpurun_out/r06n/${cfg}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; L=json.loads(open('gpurun_out/r06n/${cfg}_$v.json').read().strip().splitlines()[-1]); print('${cfg}_${v}_$rep guarded', round(L['ms_per_step'],4))"
    done
  done
done
