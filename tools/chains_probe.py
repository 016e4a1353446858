"""Measurement probe (not product code): several independent thins on ONE GPU at once -- the reference's
per-chain workload (Stein_thinning.ipynb thins every RW-MH chain separately, n ~ 5e5, m = 10 000;
its fan-out is code/src/utils/parallel.py:48-52) -- against one after the other.

Each chain's persistent launch gets its own stream and a grid of CUs / C blocks (st_tune key 5),
C = chains in flight; the launches queue on the device's hardware queues.

    python tools/chains_probe.py [chains] [n] [m] [C ...]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    from stein_thinning import _native as nat
    from stein_thinning import thinning as st
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 500_000
    m = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000
    conc = [int(c) for c in sys.argv[4:]] or [2, 4, 8]
    probs = []
    for k in range(K):
        x, g = bench.lv_call_shape(n, 20_000 + k, 'exp')
        prob = st._make_stein_integrand(x, g, preconditioner='med').device_problem()
        view = prob.dedup_view()
        probs.append(view.problem if view is not None else prob)
    print(f'{K} chains, n = {n}, m = {m}, run starts {[p.n for p in probs]}', flush=True)
    L = nat.lib()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    bufs = [p.greedy_buffers(m) for p in probs]
    pool = [torch.cuda.Stream() for _ in range(max([1] + [int(c) for c in sys.argv[4:]] + [8]))]
    # reference: one after the other on the current stream, full grid
    ref = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for p, (idx, a, ws) in zip(probs, bufs):
        p.greedy_launch(m, idx, a, ws)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ref = [b[0].cpu().numpy().view(np.uint32).copy() for b in bufs]
    print(f'one after the other (grid {cus} blocks): {1e3 * dt:8.2f} ms for {K} thins, {1e3 * dt / K:6.2f} ms per thin',
          flush=True)
    for c in conc:
        G = max(1, cus // c)
        assert L.st_tune(5, G if c > 1 else -1) == 0
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i, (p, (idx, a, ws)) in enumerate(zip(probs, bufs)):
                with torch.cuda.stream(pool[i % c]):   # c streams, as device.greedy_concurrent
                    p.greedy_launch(m, idx, a, ws)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            got = [b[0].cpu().numpy().view(np.uint32).copy() for b in bufs]
            bad = sum(int(g.max()) >= p.n for g, p in zip(got, probs))
            same = all(np.array_equal(a, b) for a, b in zip(got, ref))
            print(f'in flight {c} (grid {G} blocks each): {1e3 * dt:8.2f} ms for {K} thins, '
                  f'{1e3 * dt / K:6.2f} ms per thin, poisoned {bad}, same indices {same}', flush=True)
    L.st_tune(5, -1)
    # the product call on the full (not yet compacted) problems: run detection + the concurrent thins
    from stein_thinning.device import greedy_concurrent
    full = [st._make_stein_integrand(*bench.lv_call_shape(n, 20_000 + k, 'exp'), preconditioner='med').device_problem()
            for k in range(K)]
    ref_full = None
    for c in (1, 2, 4):
        for rep in range(2):
            for f in full:
                f._dedup = False   # detection timed too
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            got = greedy_concurrent(full, m, in_flight=c)
            dt = time.perf_counter() - t0
            if ref_full is None:
                ref_full = got   # in_flight = 1: p.greedy one after the other
            print(f'greedy_concurrent(in_flight={c}) on the full problems: {1e3 * dt:8.2f} ms for {K} thins '
                  f'(run detection included), same indices as in_flight=1 '
                  f'{all(np.array_equal(a, b) for a, b in zip(got, ref_full))}', flush=True)


if __name__ == '__main__':
    main()
