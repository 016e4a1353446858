# NT=256 (one wave per SIMD) vs NT=512 dynamic-chunk persistent kernel across n (tools/tune_sweep.py)
set -e
mkdir -p gpurun_out
: > gpurun_out/sweep_n.log
for n in 2.5e5 5e5 1e6 1.2e6 1.5e6 3e6; do
  timeout -k 10 200 python tools/tune_sweep.py c4@$n "9=256" "4=512,3=8,9=256" >> gpurun_out/sweep_n.log 2>&1
done
for n in 1e6 2e6; do
  timeout -k 10 200 python tools/tune_sweep.py c3@$n "9=256" "4=512,3=8,9=256" >> gpurun_out/sweep_n.log 2>&1
done
