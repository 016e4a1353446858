#!/usr/bin/env bash
# Same-box A/B of the persistent kernel: A = tools/_diag/ab/probe (scripts/build_ab.sh), B = the
# working tree's tools/probe; mode r (record layouts, m = 1000) interleaved A B A B at n = 2e6, then
# A B at n = 2.5e5.  Output: gpurun_out/ab_{A,B}_{1,2,s}.log and a summary on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [[ -z ${1:-} ]]; then
for r in 1 2; do
  timeout -k 10 120 ./tools/_diag/ab/probe 2000000 r > gpurun_out/ab_A_$r.log 2>&1 || exit 1
  timeout -k 10 120 ./tools/probe 2000000 r > gpurun_out/ab_B_$r.log 2>&1 || exit 1
done
timeout -k 10 120 ./tools/_diag/ab/probe 250000 r > gpurun_out/ab_A_s.log 2>&1 || exit 1
timeout -k 10 120 ./tools/probe 250000 r > gpurun_out/ab_B_s.log 2>&1 || exit 1
for f in ab_A_1 ab_B_1 ab_A_2 ab_B_2 ab_A_s ab_B_s; do
  echo "## $f"; grep -h "replicas=16\|replicas= 1 " gpurun_out/$f.log
done
fi
# mode 2 (ab_run.sh step): the launch-per-step kernels -- bench config 5 (d = 50 step kernel) through
# either library (ST_HIP_LIB), and the d = 4 step-kernel sweep of tools/probe
if [[ ${1:-} == step ]]; then
  for r in 1 2; do
    ST_HIP_LIB=tools/_diag/ab/libstein_hip.so timeout -k 10 300 python3 bench.py --config c5 --steps 3 --warmup 1 \
      --no-cpu-baseline > gpurun_out/ab_c5_A_$r.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c5_B_$r.log 2>&1 || exit 1
  done
  timeout -k 10 200 ./tools/_diag/ab/probe 2000000 > gpurun_out/ab_step_A.log 2>&1 || exit 1
  timeout -k 10 200 ./tools/probe 2000000 > gpurun_out/ab_step_B.log 2>&1 || exit 1
  for f in ab_c5_A_1 ab_c5_B_1 ab_c5_A_2 ab_c5_B_2; do
    echo "## $f"; python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$f.log') if l.startswith('{')][-1]); print(d['ms_per_step'], json.dumps(d.get('roofline'))[:400])"
  done
  for f in ab_step_A ab_step_B; do echo "## $f"; grep -h "greedy blocks" gpurun_out/$f.log; done
fi
# mode 3 (ab_run.sh proxy): the proxy producers through either library, Gaussian and Student-t
if [[ ${1:-} == proxy ]]; then
  for r in 1 2; do
    for k in gauss t; do
      ST_HIP_LIB=tools/_diag/ab/libstein_hip.so timeout -k 10 300 python3 bench.py --workload proxy --proxy-kind $k \
        --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_px_A_${k}_$r.log 2>&1 || exit 1
      timeout -k 10 300 python3 bench.py --workload proxy --proxy-kind $k --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/ab_px_B_${k}_$r.log 2>&1 || exit 1
    done
  done
  for f in gpurun_out/ab_px_[AB]_*.log; do
    echo "## $f"; python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print(d['ms_per_step'], r.get('kernel_avg_us'), r.get('frac'))"
  done
fi
# mode 4 (ab_run.sh energy): the energy-distance curve through either library
if [[ ${1:-} == energy ]]; then
  for r in 1 2; do
    ST_HIP_LIB=tools/_diag/ab/libstein_hip.so timeout -k 10 300 python3 bench.py --workload energy --steps 5 --warmup 1 \
      --no-cpu-baseline > gpurun_out/ab_en_A_$r.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py --workload energy --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_en_B_$r.log 2>&1 || exit 1
  done
  for f in gpurun_out/ab_en_[AB]_*.log; do
    echo "## $f"; python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print(d['ms_per_step'], r.get('step_median_us'), r.get('frac'))"
  done
fi
# mode 5 (ab_run.sh ksd): full-sample KSD column sums, config 2 (n = 2e5) through either library
if [[ ${1:-} == ksd || ${1:-} == ksdfull ]]; then
  KF=""; [[ ${1:-} == ksdfull ]] && KF="--ksd-full"
  for r in 1 2; do
    ST_HIP_LIB=tools/_diag/ab/libstein_hip.so timeout -k 10 300 python3 bench.py --workload ksd $KF --steps 2 --warmup 1 \
      --no-cpu-baseline > gpurun_out/ab_ks_A_$r.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py --workload ksd $KF --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_ks_B_$r.log 2>&1 || exit 1
  done
  for f in gpurun_out/ab_ks_[AB]_*.log; do
    echo "## $f"; python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print(d['ms_per_step'], r.get('kernel_avg_us'), r.get('frac'))"
  done
fi
# mode 6 (ab_run.sh lv): the LV gradient batch through either library
if [[ ${1:-} == lv ]]; then
  for r in 1 2; do
    ST_HIP_LIB=tools/_diag/ab/libstein_hip.so timeout -k 10 300 python3 bench.py --workload lv --steps 5 --warmup 1 \
      --no-cpu-baseline > gpurun_out/ab_lv_A_$r.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py --workload lv --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/ab_lv_B_$r.log 2>&1 || exit 1
  done
  for f in gpurun_out/ab_lv_[AB]_*.log; do
    echo "## $f"; python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']; print(d['ms_per_step'], r.get('kernel_avg_us'), r.get('frac'))"
  done
fi
# mode 7 (ab_run.sh ranks): same-device rehearsal of the multi-rank engine (2 and 4 processes on
# the one GPU, ST_BENCH_SHARE_DEVICE=1) through either library
if [[ ${1:-} == ranks ]]; then
  for r in 1 2; do
    for w in 2 4; do
      ST_BENCH_SHARE_DEVICE=1 ST_HIP_LIB=$PWD/tools/_diag/ab/libstein_hip.so timeout -k 10 300 python3 bench.py --gpus $w \
        --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_rk_A_${w}_$r.log 2>&1 || exit 1
      ST_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python3 bench.py --gpus $w --steps 5 --warmup 2 --no-cpu-baseline \
        > gpurun_out/ab_rk_B_${w}_$r.log 2>&1 || exit 1
    done
  done
  for f in gpurun_out/ab_rk_[AB]_*.log; do
    echo "## $f"; python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print(d['n_gpus'], d['ms_per_step'], d['config']['parallelism'], d.get('degraded'))"
  done
fi
