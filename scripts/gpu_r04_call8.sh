# Round 4 call 8: full GPU suite + smoke on the working tree (8 replicas, first-poll delay), then the
# config-4 / config-2 / config-3 bench lines
set -o pipefail
mkdir -p gpurun_out/r04
bash scripts/gpu_r04_suite.sh || exit 1
for c in c4 c2 c3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04/bench8_$c.json 2> gpurun_out/r04/bench8_$c.err || { tail gpurun_out/r04/bench8_$c.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/r04/bench8_$c.json') if l.startswith('{')][-1]); print('$c', d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_median_us'])"
done
