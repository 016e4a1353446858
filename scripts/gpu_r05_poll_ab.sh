# Round 5: poll-grid A/B (ST_POLL_SYNC 38 / 45 / 52 ticks; scripts/build_poll_variants.sh), the drop-in
# defaults (guard on): all-row thin (ms_per_step) and the run starts (dedup.thin_s) of configs 4 / 2 / c4r8
set -o pipefail
mkdir -p gpurun_out/r05ps
for cfg in c4 c2 c4r8; do
  for r in 1 2; do
    for v in default ps38 ps52; do
      lib=""; [[ $v == default ]] || lib=tools/ab/$v/libstein_hip.so
      ST_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline \
        --no-kernel-timing > gpurun_out/r05ps/${cfg}_${v}_$r.json 2> gpurun_out/r05ps/${cfg}_${v}_$r.err || exit 1
      python3 -c "import json; d=json.loads(open('gpurun_out/r05ps/${cfg}_${v}_$r.json').read().strip().splitlines()[-1]); print('$cfg $v $r', round(d['ms_per_step'],4), (d.get('dedup') or {}).get('thin_s'))"
    done
  done
done
