# Round 5: the drop-in's repeated-row thins (dedup object) of the small configs in each arithmetic,
# unguarded (ST_NEAR_TIE=0) and guarded: what a small shard's NumPy-equivalent selection costs either way
set -o pipefail
mkdir -p gpurun_out/r05a
for cfg in ${CFGS:-c2 c4r8 lv}; do
  for ar in compact exact; do
    for gd in 0 1; do
      ST_NEAR_TIE=$gd timeout -k 10 300 python3 bench.py --config $cfg --steps 5 --warmup 1 --arith $ar --no-cpu-baseline \
        --no-kernel-timing > gpurun_out/r05a/${cfg}_${ar}_g${gd}.json 2> gpurun_out/r05a/${cfg}_${ar}_g${gd}.err || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/r05a/${cfg}_${ar}_g${gd}.json').read().strip().splitlines()[-1]); print('$cfg $ar guard=$gd', round(d['ms_per_step'],4), (d.get('dedup') or {}).get('thin_s'), (d.get('dedup') or {}).get('near_tie_step'), (d.get('dedup') or {}).get('rows_kept'))"
    done
  done
done
