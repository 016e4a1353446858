# Round 5: record replicas (st_tune key 10) on the small shards' run starts, alternating, twice
set -o pipefail
mkdir -p gpurun_out/r05k2
for r in 1 2; do
  for cfg in c2 c4r8; do
    for v in none "10=4" "10=2" "10=1"; do
      tag=${v//=/_}
      ST_TUNE=$([[ $v == none ]] || echo $v) timeout -k 10 300 python3 bench.py --config $cfg --steps 10 --warmup 2 \
        --no-cpu-baseline --no-kernel-timing > gpurun_out/r05k2/${cfg}_${tag}_$r.json 2> gpurun_out/r05k2/${cfg}_${tag}_$r.err || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/r05k2/${cfg}_${tag}_$r.json').read().strip().splitlines()[-1]); print('$cfg $v $r', round(d['ms_per_step'],4), (d.get('dedup') or {}).get('thin_s'))"
    done
  done
done
