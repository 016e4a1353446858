# Round 6: the guard's launch tail -- the bounds written back by block 0's step-0 check instead of at the end,
# the last step's winner row from the pick's scratch instead of global loads.  Guarded suites, then the fixed /
# per-step split against HEAD (ab/hsal) and the guarded bench legs of configs 2 / 3 / one rank
set -o pipefail
mkdir -p gpurun_out/r06m
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_near_tie.py tests/test_gpu_multiprocess.py tests/test_gpu_parity.py \
    tests/test_gpu_small_shard.py tests/test_gpu_golden_configs.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r06m/tests.log 2>&1 || { echo "FAIL tests"; tail -30 gpurun_out/r06m/tests.log; exit 1; }
tail -n 1 gpurun_out/r06m/tests.log
timeout -k 10 300 env ST_HIP_LIB=ab/hsal/libstein_hip.so python3 tools/guard_fixed_cost.py c2 c3 c4r8 > gpurun_out/r06m/fixed_hsal.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/guard_fixed_cost.py c2 c3 c4r8 > gpurun_out/r06m/fixed_cur.log 2>&1 || exit 1
grep -E "^c" gpurun_out/r06m/fixed_hsal.log | sed 's/^/hsal /'; grep -E "^c" gpurun_out/r06m/fixed_cur.log | sed 's/^/cur  /'
B="--steps 20 --warmup 3 --no-cpu-baseline --no-kernel-timing --no-e2e --headline-guard"
for rep in 1 2; do
  for cfg in c2 c3 c4r8; do
    for v in hsal cur; do
      if [[ $v == hsal ]]; then E="ST_HIP_LIB=ab/hsal/libstein_hip.so"; else E="X=1"; fi
      timeout -k 10 300 env $E python3 bench.py --config $cfg $B > gpurun_out/r06m/${cfg}_$v.json 2>/dev/null || exit 1
      python3 -c "import json; L=json.loads(open('gpurun_out/r06m/${cfg}_$v.json').read().strip().splitlines()[-1]); print('${cfg}_${v}_$rep guarded', round(L['ms_per_step'],4))"
    done
  done
done
