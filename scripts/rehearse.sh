# Same-device rehearsal of the N > 1 bench flow (ST_BENCH_SHARE_DEVICE=1: every rank on cuda:0, gloo
# group, persistent grids capped to co-reside): bash scripts/rehearse.sh <config> <N>...
set -o pipefail
mkdir -p gpurun_out
export ST_BENCH_SHARE_DEVICE=1
CFG=${1:-c4}; shift
port=29611
for N in "${@:-1 2}"; do
  if [[ $N == 1 ]]; then
    timeout -k 10 300 python bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/rh_${CFG}_n1.log 2>&1 || exit $?
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $N --config $CFG --steps 5 --warmup 1 --no-cpu-baseline --no-kernel-timing \
      > gpurun_out/rh_${CFG}_n$N.log 2>&1 || exit $?
  fi
  port=$((port + 1))
  echo "== N=$N"; grep -o '"ms_per_step": [0-9.]*\|"parallelism": "[^"]*"\|"kernel": "[^"]*"' gpurun_out/rh_${CFG}_n$N.log
done
