# Round 4 call 5: first-poll delay sweep (st_tune key 16) on the product library at the 512-thread
# shard sizes, the new GPU tests (margins, key 15), the LV call-shape bench line, and the same-device
# rank rehearsal at one 8-GPU rank's per-CU load (c4r8).
set -o pipefail
mkdir -p gpurun_out/r04
: > gpurun_out/r04/sweep_delay.log
for rep in 1 2; do
  for c in c4 c4@1000000 c4@400000; do
    timeout -k 10 300 python tools/tune_sweep.py $c "16=0" "16=5" "16=10" "16=15" "16=20" "16=25" >> gpurun_out/r04/sweep_delay.log 2>&1 \
      || { tail gpurun_out/r04/sweep_delay.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r04/sweep_delay.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_margins.py "tests/test_gpu_parity.py::test_streamed_sums_in_lds_option" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r04/new_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r04/new_tests.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python bench.py --config lv --steps 5 --warmup 1 > gpurun_out/r04/bench_lv.json 2> gpurun_out/r04/bench_lv.err || { tail gpurun_out/r04/bench_lv.err; exit 1; }
tail -n 1 gpurun_out/r04/bench_lv.json | cut -c1-600
bash scripts/rehearse.sh c4r8 1 2 4 8 > gpurun_out/r04/rehearse_c4r8.log 2>&1; rc=$?; cat gpurun_out/r04/rehearse_c4r8.log; [[ $rc == 0 ]] || exit $rc
# LV phase B: per-step pieces (key 17 = 1) vs balanced pieces (2), kernel durations from rocprofv3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/prof_lv$v -o run -- python3 bench.py --workload lv --lv-dense $v \
    --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r04/bench_lv_dense$v.json 2> gpurun_out/r04/bench_lv_dense$v.err || { tail gpurun_out/r04/bench_lv_dense$v.err; exit 1; }
  f=$(find gpurun_out/r04/prof_lv$v -name '*kernel_stats.csv' | head -n 1); grep -h "lv_dense" "$f" | cut -c1-200
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_lv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/lv_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/r04/lv_tests.log; exit $rc
