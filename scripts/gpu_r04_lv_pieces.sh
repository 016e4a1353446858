# Round 4: LV phase B with 1 / 2 / 3 observation pieces per lane (st_tune key 18), alternating twice:
# rocprofv3 kernel stats of bench.py --workload lv, then the LV GPU tests
set -o pipefail
mkdir -p gpurun_out/r04d
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
for v in 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04d/prof_lvp${v}_$rep -o run -- python3 bench.py --workload lv \
    --lv-pieces $v --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r04d/bench_lvp${v}_$rep.json 2> gpurun_out/r04d/bench_lvp${v}_$rep.err \
    || { tail gpurun_out/r04d/bench_lvp${v}_$rep.err; exit 1; }
  f=$(find gpurun_out/r04d/prof_lvp${v}_$rep -name '*kernel_stats.csv' | head -n 1); echo "== pieces=$v rep $rep"; grep -h "lv_" "$f" | cut -c1-160
done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_lv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04d/lv_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/r04d/lv_tests.log; exit $rc
