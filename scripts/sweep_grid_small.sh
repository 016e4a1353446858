# Persistent grid size (st_tune key 5) x threads per block (key 4) for small shards (tools/tune_sweep.py)
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep_grid.log
for n in 1e5 2.5e5 5e5; do
  timeout -k 10 200 python tools/tune_sweep.py c4@$n "5=256" "5=192" "5=128" "5=96" "5=64" "5=128,4=512" "5=64,4=512" >> gpurun_out/sweep_grid.log 2>&1
done
