# one rocprofv3 --pmc pass over the energy workload: where the SIMD cycles of dist_colsum_kernel go
# (8 SQ counters, the per-pass SQ limit); summary: gpurun_out/valu/energy_stall.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
CTRS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
out=gpurun_out/valu/energy_stall
timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $out -o pmc -- \
  python3 bench.py --workload energy --steps 1 --warmup 0 --no-cpu-baseline > $out.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 1 $out.log | cut -c1-200
[[ $rc == 0 ]] || exit $rc
f=$(find $out -name '*counter_collection.csv' | head -n 1)
cp "$f" gpurun_out/valu/energy_stall.csv
