# Round 4 call 7: record replicas (st_tune key 10) and 512-thread blocks (key 4) at the small shard
# sizes with the round-4 kernel (the flat-sweep probe found 8 replicas faster than 16 without compute)
set -o pipefail
mkdir -p gpurun_out/r04
: > gpurun_out/r04/sweep_rep_nt.log
for rep in 1 2; do
  for c in c2 c4@250000 c4; do
    timeout -k 10 300 python tools/tune_sweep.py $c "10=16" "10=8" "10=4" "10=32" "4=512" "4=512,10=8" >> gpurun_out/r04/sweep_rep_nt.log 2>&1 \
      || { tail gpurun_out/r04/sweep_rep_nt.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/r04/sweep_rep_nt.log
