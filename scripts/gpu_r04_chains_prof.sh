#!/bin/bash
# rocprofv3 kernel trace of the chains workload (the batch launch of 8 LV-shape chains).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04d_prof
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o chains -- \
    python3 bench.py --workload chains --steps 3 --warmup 1 > $OUT/chains.json 2> $OUT/chains.err
