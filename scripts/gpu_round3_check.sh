set -o pipefail
for v in 1 2 3 4 5; do
  timeout -k 10 180 python bench.py --workload energy --energy-variant $v --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r03_energy_v$v.json 2> gpurun_out/r03_energy_v$v.err || exit $?
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests_head.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || exit $?
timeout -k 10 240 python bench.py > gpurun_out/r03_bench_head.json 2> gpurun_out/r03_bench_head.err
