# energy kernel A/B on one box: variant 1 (fmin zero-distance form) vs 6 (round-2 select form), twice
# each, alternating; then the energy and KSD GPU tests
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_energy.py tests/test_gpu_parity.py -k "energy or curve or distance" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_energy_tests.log 2>&1 || exit $?
for v in 1 6 1 6; do
  timeout -k 10 180 python bench.py --workload energy --energy-variant $v --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/r03_energy_fmin_ab.jsonl 2>> gpurun_out/r03_energy_fmin_ab.err || exit $?
done
