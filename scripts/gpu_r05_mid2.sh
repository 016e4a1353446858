# Round 5: mid-size compact-only register-row rule (4 up to 2 560 rows per block, else 6) -- the row probe,
# the plan-sensitive GPU tests, then the LV call / config-4 A/B against the library before mid-size plans.
set -o pipefail
mkdir -p gpurun_out/r05m
export TMPDIR=/tmp
PYTHONPATH=.:gradient-free-mcmc-postprocessing_amd timeout -k 10 300 python3 tools/mid_rows_probe.py \
  > gpurun_out/r05m/mid_rows_probe.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r05m/mid_rows_probe.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_mid_compact.py tests/test_gpu_parity.py tests/test_gpu_batch.py \
  tests/test_gpu_near_tie.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r05m/tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r05m/tests.log; [[ $rc == 0 ]] || exit $rc
SKIP_SUITE=1 EXTRA_TESTS= GUARD_A=1 GUARD_B=1 AB_LIB=tools/ab/r05d/libstein_hip.so AB="lv:5 c4:10" \
  bash scripts/gpu_r05_guard.sh > gpurun_out/r05m/ab.log 2>&1; rc=$?; cat gpurun_out/r05m/ab.log; [[ $rc == 0 ]] || exit $rc
echo done
