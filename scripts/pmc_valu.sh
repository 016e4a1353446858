#!/usr/bin/env bash
# VALU issue counters (rocprofv3 --pmc, ONE pass per workload: 8 SQ counters + GRBM_GUI_ACTIVE, within
# one pass's limits) for the dominant kernel of the energy, KSD and config-4 thin workloads;
# summarised by tools/summarize_valu.py (instructions per pair, VALU busy, effective clock).
#   bash scripts/pmc_valu.sh [key ...]      keys: energy ksd_c2 c4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
CTRS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
declare -A ARGS=( [energy]="--workload energy" [ksd_c2]="--workload ksd" [c4]="--config c4 --no-kernel-timing" )
KEYS=("$@")
[[ ${#KEYS[@]} -gt 0 ]] || KEYS=(energy ksd_c2 c4)
for key in "${KEYS[@]}"; do
  out=gpurun_out/valu/$key
  echo "=== $key ($(date +%T))"
  timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $out -o pmc -- \
    python3 bench.py ${ARGS[$key]} --steps 1 --warmup 0 --no-cpu-baseline > $out.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -n 1 $out.log | cut -c1-200
  [[ $rc == 0 ]] || exit $rc
  f=$(find $out -name '*counter_collection.csv' | head -n 1)
  cp "$f" gpurun_out/valu/${key}_valu.csv
done
echo "=== done"
