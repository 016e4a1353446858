# one rocprofv3 --pmc pass over the LV gradient workload: where lv_dense_kernel's cycles go
# (8 SQ counters + 2 TA counters, within the per-pass limits); summary: gpurun_out/r04/lv_stall.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum"
out=gpurun_out/r04/lv_stall
timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $out -o pmc -- \
  python3 bench.py --workload lv --steps 1 --warmup 0 --no-cpu-baseline > $out.log 2>&1
rc=$?
echo "rc=$rc"; tail -n 1 $out.log | cut -c1-200
[[ $rc == 0 ]] || exit $rc
f=$(find $out -name '*counter_collection.csv' | head -n 1)
cp "$f" gpurun_out/r04/lv_stall.csv
