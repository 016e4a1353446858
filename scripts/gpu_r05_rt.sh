# Round 5: the compact-only kernel's register rows at config 4 (st_tune key 12: 8 / 9 / 10), alternating twice
set -o pipefail
mkdir -p gpurun_out/r05rt
for r in 1 2; do
  for v in none "12=8" "12=10"; do
    tag=${v//=/_}
    ST_TUNE=$([[ $v == none ]] || echo $v) timeout -k 10 300 python3 bench.py --config c4 --steps 10 --warmup 2 \
      --no-cpu-baseline --no-kernel-timing > gpurun_out/r05rt/c4_${tag}_$r.json 2> gpurun_out/r05rt/c4_${tag}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r05rt/c4_${tag}_$r.json').read().strip().splitlines()[-1]); print('c4 $v $r', round(d['ms_per_step'],4), d['roofline']['kernel'][:60])"
  done
done
