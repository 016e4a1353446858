set -o pipefail
mkdir -p gpurun_out
export ST_BENCH_SHARE_DEVICE=1
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_n1.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_n2.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_n4.log 2>&1
rc=$?
for f in gpurun_out/c5_n*.log; do echo "== $f"; grep -o '"ms_per_step": [0-9.]*\|"parallelism": "[^"]*"' $f; done
exit $rc
