# Round 4: energy kernel work-unit A/B (st_tune key 14) on one box after the stall pass showed ~3
# waves per SIMD on average: old target 2048 against 8192 / 16384 / 32768, variants 1 (4 blocks per
# CU) and 3 (8 blocks per CU), alternating twice; then the energy + KSD GPU tests.
set -o pipefail
mkdir -p gpurun_out/r04
out=gpurun_out/r04/energy_units_ab.jsonl
: > $out
for rep in 1 2; do
  for cfg in "1 2048" "1 8192" "1 16384" "1 32768" "3 16384" "3 32768"; do
    set -- $cfg
    timeout -k 10 180 python bench.py --workload energy --energy-variant $1 --energy-units $2 --steps 5 --warmup 1 \
      --no-cpu-baseline >> $out 2>> gpurun_out/r04/energy_units_ab.err || exit $?
  done
done
python - <<'PY'
import json
for l in open('gpurun_out/r04/energy_units_ab.jsonl'):
    if not l.startswith('{'): continue
    r = json.loads(l); rf = r['roofline']
    print(rf.get('kernel', ''), rf['step_median_us'], rf.get('frac'))
PY
timeout -k 10 400 python -u -m pytest tests/test_gpu_energy.py tests/test_gpu_ksd.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r04/energy_ksd_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r04/energy_ksd_tests.log; exit $rc
