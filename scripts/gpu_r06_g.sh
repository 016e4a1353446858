# Round 6: the N > 1 bench line as the driver runs it (torch.distributed.run, one rank per GPU), rehearsed with
# the ranks sharing this box's one GPU (ST_BENCH_SHARE_DEVICE=1): config5_sharded, rank_hop and the new
# chains_over_gpus object; then configs 2 / 3 again (drop_in_takes_it now follows the drop-in's own rule)
set -o pipefail
mkdir -p gpurun_out/r06g
export TMPDIR=/tmp
for g in 2 4; do
  timeout -k 10 600 env ST_BENCH_SHARE_DEVICE=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $g \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $g --steps 3 --warmup 1 \
    > gpurun_out/r06g/rehearsal_n$g.json 2> gpurun_out/r06g/rehearsal_n$g.err || { echo "FAIL n$g"; tail -20 gpurun_out/r06g/rehearsal_n$g.err; exit 1; }
  tail -n 1 gpurun_out/r06g/rehearsal_n$g.json | cut -c1-300
done
for c in c2 c3; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 > gpurun_out/r06g/bench_$c.json 2> gpurun_out/r06g/bench_$c.err || { echo "FAIL $c"; tail -5 gpurun_out/r06g/bench_$c.err; exit 1; }
  tail -n 1 gpurun_out/r06g/bench_$c.json | cut -c1-200
done
