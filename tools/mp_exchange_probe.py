"""Measurement probe (not product code): the multi-rank persistent kernel with W processes sharing
the one GPU of a gpurun box (IPC mailboxes, gloo for setup), each rank capped at 256 / W blocks.

At n = 2e6 / 8 * W rows the per-CU load equals the 8-GPU config-4 case (2.5e5 rows per rank on
256 CUs), so the per-step time is what one rank of an 8-GPU run spends on compute + exchange
(same-device IPC instead of xGMI for the rank hop).

usage: python tools/mp_exchange_probe.py [W] [n] [m] [reps]
"""
import os
import socket
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd')]


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def worker(rank, world, port, n, m, reps, grid):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import bench
    from stein_thinning import _native as nat
    from stein_thinning import distributed as sd
    from stein_thinning import thinning as st
    nat.lib().st_tune(5, grid)
    x, g, _, _ = bench.lv_surrogate(n, 12345)
    integrand = st._make_stein_integrand(x, g, preconditioner='med')
    mb = sd.peer_mailboxes()
    assert mb.ok, mb.error
    runner = sd.PersistentShardedGreedy(integrand, rank, world, m, mb)
    ref = runner.run()
    assert runner.completed(ref)
    times = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runner.launch()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        assert np.array_equal(runner.indices(), ref)
    if rank == 0:
        med = float(np.median(times))
        print(f'W={world} n={n} m={m} grid/rank={grid}: thin {med * 1e3:.3f} ms (median of {reps}), '
              f'{med / m * 1e6:.2f} us/step, first idx {ref[:4].tolist()}', flush=True)
    dist.destroy_process_group()


def single(n, m, reps, grid):
    """W = 1: the single-device persistent kernel on `grid` blocks (no rank exchange)."""
    import torch
    import bench
    from stein_thinning import _native as nat
    from stein_thinning import thinning as st
    nat.lib().st_tune(5, grid)
    x, g, _, _ = bench.lv_surrogate(n, 12345)
    prob = st._make_stein_integrand(x, g, preconditioner='med').device_problem()
    idx, a, ws = prob.greedy_buffers(m)
    prob.greedy_launch(m, idx, a, ws)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        prob.greedy_launch(m, idx, a, ws)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    med = float(np.median(times))
    print(f'W=1 n={n} m={m} grid={grid}: thin {med * 1e3:.3f} ms, {med / m * 1e6:.2f} us/step, '
          f'first idx {idx[:4].cpu().numpy().view(np.uint32).tolist()}', flush=True)


def main():
    import torch.multiprocessing as mp
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 2_000_000 // 8 * W
    m = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    grid = int(sys.argv[5]) if len(sys.argv) > 5 else 256 // W
    if W == 1:
        single(n, m, reps, grid)
        return
    mp.spawn(worker, args=(W, _port(), n, m, reps, grid), nprocs=W, join=True)


if __name__ == '__main__':
    main()
