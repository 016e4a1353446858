# Round 4 call 4: first-poll delay variants (tools/_diag/pv_*), the new GPU tests (margins, key 15),
# the LV call-shape bench line, and the same-device rank rehearsal at one 8-GPU rank's per-CU load
# (c4r8: 2.5e5 rows over N processes sharing the GPU, 256/N CUs each).
set -o pipefail
mkdir -p gpurun_out/r04
PV_NS="200000 250000 2000000" bash scripts/pv_run.sh base fd15 fd30 fd45 fd70 > gpurun_out/r04/pv_first_delay.log 2>&1 || { tail gpurun_out/r04/pv_first_delay.log; exit 1; }
grep -h "##\|quick" gpurun_out/r04/pv_first_delay.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_margins.py "tests/test_gpu_parity.py::test_streamed_sums_in_lds_option" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r04/new_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r04/new_tests.log; [[ $rc == 0 ]] || exit $rc
timeout -k 10 300 python bench.py --config lv --steps 5 --warmup 1 > gpurun_out/r04/bench_lv.json 2> gpurun_out/r04/bench_lv.err || { tail gpurun_out/r04/bench_lv.err; exit 1; }
tail -n 1 gpurun_out/r04/bench_lv.json | cut -c1-600
bash scripts/rehearse.sh c4r8 1 2 4 8 > gpurun_out/r04/rehearse_c4r8.log 2>&1; rc=$?; cat gpurun_out/r04/rehearse_c4r8.log; exit $rc
