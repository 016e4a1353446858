# Round 4, first GPU call: the energy stall pass (committed in round 3, never run), a persistent
# grid-size sweep with the round-3 kernel at the small-shard sizes (configs 2 / 3 and one rank of an
# 8-GPU config-4 run), and the config-2 bench line.  Every GPU step has its own time limit and the
# steps are chained: the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04
export TMPDIR=/tmp
bash scripts/pmc_energy_stall.sh > gpurun_out/r04/stall.txt 2>&1 || { echo "stall pass failed"; cat gpurun_out/r04/stall.txt; exit 1; }
echo "stall pass done"
: > gpurun_out/r04/sweep_grid.log
for c in c2 c3 c4@250000; do
  timeout -k 10 240 python tools/tune_sweep.py $c "5=256" "5=192" "5=160" "5=128" "5=96" "5=64" \
    >> gpurun_out/r04/sweep_grid.log 2>&1 || { echo "sweep $c failed"; tail -n 20 gpurun_out/r04/sweep_grid.log; exit 1; }
  echo "sweep $c done"
done
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 > gpurun_out/r04/bench_c2.json 2> gpurun_out/r04/bench_c2.err \
  || { echo "bench c2 failed"; tail -n 20 gpurun_out/r04/bench_c2.err; exit 1; }
cat gpurun_out/r04/sweep_grid.log
tail -n 1 gpurun_out/r04/bench_c2.json | cut -c1-400
