# Round 5: the persistent kernel's tuning keys re-checked with the round-5 build (ST_TUNE, bench.py):
# first-poll delay (16), record replicas (10), two-chain LDS chunks (19), streamed sums in LDS (15)
set -o pipefail
mkdir -p gpurun_out/r05k
for cfg in c4 c4r8; do
  for v in none "16=0" "16=5" "16=20" "10=4" "10=16" "19=0" "15=0"; do
    tag=${v//=/_}
    ST_TUNE=$([[ $v == none ]] || echo $v) timeout -k 10 300 python3 bench.py --config $cfg --steps 10 --warmup 2 \
      --no-cpu-baseline --no-kernel-timing > gpurun_out/r05k/${cfg}_$tag.json 2> gpurun_out/r05k/${cfg}_$tag.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r05k/${cfg}_$tag.json').read().strip().splitlines()[-1]); print('$cfg $v', round(d['ms_per_step'],4), (d.get('dedup') or {}).get('thin_s'))"
  done
done
