# Round 4 call 6: flat multi-rank sweep probe (exchange floor for R x 256 records), the single-poll
# row-prefetch variant A/B (tools/_diag/pv_{base,frl}), and the config-4 / config-2 bench lines with
# the first-poll delay default.
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 120 ./tools/flat_sweep_probe 2000 > gpurun_out/r04/flat_sweep.log 2>&1; rc=$?; cat gpurun_out/r04/flat_sweep.log; [[ $rc == 0 ]] || exit $rc
PV_NS="200000 250000 2000000" bash scripts/pv_run.sh base frl > gpurun_out/r04/pv_frl.log 2>&1 || { tail gpurun_out/r04/pv_frl.log; exit 1; }
grep -h "##\|quick" gpurun_out/r04/pv_frl.log | paste - -
for c in c4 c2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04/bench_$c.json 2> gpurun_out/r04/bench_$c.err || { tail gpurun_out/r04/bench_$c.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r04/bench_$c.json') if l.startswith('{')][-1]); print('$c', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_median_us'])"
done
