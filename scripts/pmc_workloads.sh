#!/usr/bin/env bash
# HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE, one counter per pass, each pass its own run) of
# every bench workload's dominant kernel; summarised per launch into profiles/pmc_traffic.json by
# tools/summarize_pmc.py (gfx950 FETCH_SIZE x2 correction).  Any failing pass ends the script.
#   bash scripts/pmc_workloads.sh [key ...]      keys: energy ksd_c2 proxy_gauss proxy_t lv lv2 c4_persistent chains_batch
#                                                 c4_dropin (the guarded thin of config 4's run starts)
# PMC_SOURCE (environment) labels the records (round, commit).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
declare -A ARGS=( [energy]="--workload energy" [ksd_c2]="--workload ksd" [proxy_gauss]="--workload proxy"
                  [proxy_t]="--workload proxy --proxy-kind t" [lv]="--workload lv"
                  [c4_persistent]="--config c4 --no-kernel-timing" [lv2]="--workload lv"
                  [chains_batch]="--workload chains" [c4_dropin]="--config c4 --no-kernel-timing" )
declare -A KERN=( [energy]="dist_colsum_kernel" [ksd_c2]="ksd_colsum_kernel" [proxy_gauss]="proxy_mfma_buf_kernel"
                  [proxy_t]="proxy_mfma_buf_kernel" [lv]="lv_kernel<10>"
                  [c4_persistent]="greedy_persistent<4, false, 9, 512, 1, true, false, st::PersistArgs, false>" [lv2]="lv_dense_kernel"
                  [chains_batch]="st::BatchArgs, " [c4_dropin]="greedy_persistent<4, false, 4, 512, 1, true, true, st::PersistArgs, true>" )
declare -A EXCL=( [c4_persistent]="@none@" [lv2]="@none@" [chains_batch]="@none@" [c4_dropin]="@none@" )
KEYS=("$@")
[[ ${#KEYS[@]} -gt 0 ]] || KEYS=(energy ksd_c2 proxy_gauss proxy_t lv)
for key in "${KEYS[@]}"; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    out=gpurun_out/pmc/${key}_${ctr}
    echo "=== $key $ctr ($(date +%T))"
    timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $out -o pmc -- \
      python3 bench.py ${ARGS[$key]} --steps ${PMC_STEPS:-1} --warmup ${PMC_WARMUP:-0} --no-cpu-baseline > $out.log 2>&1
    rc=$?
    echo "rc=$rc"; tail -n 2 $out.log
    [[ $rc == 0 ]] || exit $rc
  done
  f=$(find gpurun_out/pmc/${key}_FETCH_SIZE -name '*counter_collection.csv' | head -n 1)
  w=$(find gpurun_out/pmc/${key}_WRITE_SIZE -name '*counter_collection.csv' | head -n 1)
  cp "$f" gpurun_out/pmc/${key}_fetch_size.csv && cp "$w" gpurun_out/pmc/${key}_write_size.csv
  python3 tools/summarize_pmc.py "$f" "$w" "$key" --kernel "${KERN[$key]}" --exclude "${EXCL[$key]:-, true, }" \
    --source "${PMC_SOURCE:-scripts/pmc_workloads.sh}" --out gpurun_out/pmc/pmc_traffic_new.json || exit 1
done
echo "=== done"
