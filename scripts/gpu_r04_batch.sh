#!/bin/bash
# Batch launch (st_greedy_batch): GPU tests, the default bench (headline kernel unchanged?) and the
# chains workload (batch vs streams).
set -o pipefail
OUT=gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batch.py \
    > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --workload chains > $OUT/chains.json 2> $OUT/chains.err &&
timeout -k 10 300 python bench.py --workload chains --batch 4 > $OUT/chains_b4.json 2> $OUT/chains_b4.err
