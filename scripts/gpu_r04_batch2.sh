#!/bin/bash
# After the 256-thread batch kernels: the full GPU suite + smoke, the default bench and the chains bench.
set -o pipefail
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --workload chains > $OUT/chains.json 2> $OUT/chains.err &&
timeout -k 10 300 python bench.py --workload chains --chains 2 > $OUT/chains2.json 2> $OUT/chains2.err
