# Round 5: the LV chains' batch launch (5 chains, run starts, ~2 300 rows per block) on the general kernel
# (st_tune key 12 = 0, the default for batches) against the compact-only kernel forced to 4 / 6 / 8 register rows.
set -o pipefail
mkdir -p gpurun_out/r05c
export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 4 6 8; do
    ST_TUNE=12=$v timeout -k 10 300 python3 bench.py --workload chains --steps 5 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r05c/chains_k$v.$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r05c/chains_k$v.$r.json').read().strip().splitlines()[-1]); print('chains key12=$v run $r', round(d['ms_per_step'],3))"
  done
done
echo done
