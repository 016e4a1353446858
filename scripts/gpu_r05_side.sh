# Round 5: the side workloads' bench lines on the final build (energy curve, LV inputs, full-sample KSD, proxy)
set -o pipefail
mkdir -p gpurun_out/r05side
step() {
  local name=$1 tmo=$2; shift 2
  timeout -k 10 "$tmo" "$@" > "gpurun_out/r05side/$name.json" 2> "gpurun_out/r05side/$name.err" || { echo "$name failed"; tail -5 "gpurun_out/r05side/$name.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r05side/$name.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$name', round(d['ms_per_step'],4), d['unit'], r.get('frac'))"
}
step bench_energy 300 python3 bench.py --workload energy
step bench_lv 300 python3 bench.py --workload lv
step bench_ksd_full 600 python3 bench.py --workload ksd --ksd-full --steps 2 --warmup 1 --no-cpu-baseline
step bench_proxy 300 python3 bench.py --workload proxy
