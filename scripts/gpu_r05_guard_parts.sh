# Round 5: where the near-tie guard's cost goes -- the headline (c4) and config-2 thins with parts of the
# guard switched off (st_tune key 21, measurement only; key 20 = 0: no guard at all)
set -o pipefail
mkdir -p gpurun_out/r05p
for cfg in ${CFGS:-c4 c2}; do
  for v in ${VARIANTS:-"20=0" "21=7" "21=1" "21=2" "21=4" "21=0" "12=0"}; do
    ST_TUNE=$v timeout -k 10 300 python3 bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --no-kernel-timing \
      > gpurun_out/r05p/${cfg}_${v}.json 2> gpurun_out/r05p/${cfg}_${v}.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r05p/${cfg}_${v}.json').read().strip().splitlines()[-1]); print('${cfg} ${v}', round(d['ms_per_step'],4), d['roofline'].get('kernel_median_us'), (d.get('dedup') or {}).get('thin_s'))"
  done
done
