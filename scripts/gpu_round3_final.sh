# round-3 closing run: full GPU suite, smoke, headline bench, energy bench + its rocprofv3 kernel stats
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests_final.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_final.log 2>&1 || exit $?
timeout -k 10 240 python bench.py > gpurun_out/r03_bench_c4_final.json 2> gpurun_out/r03_bench_c4_final.err || exit $?
timeout -k 10 240 python bench.py --workload energy > gpurun_out/r03_bench_energy_final.json 2> gpurun_out/r03_bench_energy_final.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_energy -o run -- python3 bench.py --workload energy --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/r03_bench_energy_under_rocprof.json 2> gpurun_out/r03_energy_rocprof.err
