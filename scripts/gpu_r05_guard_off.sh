set -o pipefail
mkdir -p gpurun_out/r05h
for cfg in c2 c4; do
 for r in 1 2; do
  for v in off on; do
   if [[ $v == off ]]; then export ST_NEAR_TIE=0; else unset ST_NEAR_TIE; fi
   timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --no-kernel-timing > gpurun_out/r05h/${cfg}_${v}$r.json 2>/dev/null || exit 1
   python3 -c "import json; d=json.loads(open('gpurun_out/r05h/${cfg}_${v}$r.json').read().strip().splitlines()[-1]); print('${cfg}_${v}$r', round(d['ms_per_step'],4), d['roofline'].get('kernel_median_us'))"
  done
 done
done
