# Round 5: mid-size compact-only plans (persistent_cmp.hip) -- their GPU tests, the plan-sensitive suites,
# then a same-box A/B against the library before the change (tools/ab/r05d).
set -o pipefail
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mid_compact.py tests/test_gpu_parity.py tests/test_gpu_batch.py \
  tests/test_gpu_near_tie.py tests/test_gpu_small_shard.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05m/tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r05m/tests.log; [[ $rc == 0 ]] || exit $rc
SKIP_SUITE=1 EXTRA_TESTS= GUARD_A=1 GUARD_B=1 AB_LIB=tools/ab/r05d/libstein_hip.so AB="c4:20 lv:5 c4r8:20" \
  bash scripts/gpu_r05_guard.sh > gpurun_out/r05m/ab.log 2>&1; rc=$?; cat gpurun_out/r05m/ab.log; [[ $rc == 0 ]] || exit $rc
for r in 1 2; do
  ST_HIP_LIB=tools/ab/r05d/libstein_hip.so timeout -k 10 300 python3 bench.py --workload chains --steps 5 --warmup 1 \
    --no-cpu-baseline > gpurun_out/r05m/chains_A$r.json 2>/dev/null || exit 1
  timeout -k 10 300 python3 bench.py --workload chains --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/r05m/chains_B$r.json 2>/dev/null || exit 1
done
for f in A1 B1 A2 B2; do python3 -c "import json; d=json.loads(open('gpurun_out/r05m/chains_$f.json').read().strip().splitlines()[-1]); print('chains_$f', round(d['ms_per_step'],3))"; done
echo done
