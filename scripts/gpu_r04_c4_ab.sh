# Round 4: same-box A/B of config 4 (bench.py, one GPU): A = the committed library (scripts/build_ab.sh
# HEAD -> tools/_diag/ab/libstein_hip.so), B = the working tree's; alternating three times, then
# config 2 and the 2.5e5-row shard (one rank of an 8-GPU config-4 run) through tools/tune_sweep.py.
set -o pipefail
mkdir -p gpurun_out/r04
out=gpurun_out/r04/c4_ab
: > $out.jsonl
for r in 1 2 3; do
  for lib in A B; do
    L=""; [[ $lib == A ]] && L="tools/_diag/ab/libstein_hip.so"
    ST_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-kernel-timing \
      > $out.$lib$r.json 2> $out.$lib$r.err || { echo "bench $lib$r failed"; tail -n 20 $out.$lib$r.err; exit 1; }
    python - "$lib$r" "$out.$lib$r.json" >> $out.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
print(json.dumps({'run': sys.argv[1], 'ms_per_thin': round(d['ms_per_step'], 4),
                  'kernel_median_us': d['roofline']['kernel_median_us'], 'frac': d['roofline']['frac'],
                  'first_indices': d['config']['first_indices']}))
PY
  done
done
cat $out.jsonl
