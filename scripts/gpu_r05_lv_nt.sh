# Round 5: the LV call shape (n = 5e5, 1 953 rows per block) on 512- vs 256-thread blocks (st_tune key 4)
set -o pipefail
mkdir -p gpurun_out/r05lv
for r in 1 2; do
  for v in default "4=256"; do
    tag=${v//=/_}
    ST_TUNE=$([[ $v == default ]] || echo $v) timeout -k 10 300 python3 bench.py --config lv --steps 5 --warmup 1 --no-cpu-baseline \
      --no-kernel-timing > gpurun_out/r05lv/lv_${tag}_$r.json 2> gpurun_out/r05lv/lv_${tag}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r05lv/lv_${tag}_$r.json').read().strip().splitlines()[-1]); print('lv $v $r', round(d['ms_per_step'],3), (d.get('dedup') or {}).get('thin_s'), (d.get('near_tie_guard') or {}).get('ms_per_thin'))"
  done
done
