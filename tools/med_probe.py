"""Measurement probe (not product code): the 'med' preconditioner's pieces on the GPU box's host
(scipy pdist of the 1 000-row subsample, np.median), and whether a small upload + sort on a side
stream completes while a config-4-sized page-locked upload is in flight on the main stream."""
import time

import numpy as np
import torch
from scipy.spatial.distance import pdist


def main():
    rng = np.random.default_rng(0)
    sub = rng.normal(size=(1000, 4))
    for name, f in [('pdist', lambda: pdist(sub)), ('median', None)]:
        D = pdist(sub)
        ts = []
        for _ in range(20):
            t = time.perf_counter()
            f() if f else np.median(D)
            ts.append(time.perf_counter() - t)
        print(f'{name}: {1e3 * np.median(ts):.3f} ms', flush=True)
    dev = torch.device('cuda')
    big = torch.empty(2 * 2_000_000 * 4, dtype=torch.float64).pin_memory()
    side = torch.cuda.Stream()
    Dd = torch.from_numpy(pdist(sub))
    for rep in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = big.to(dev, non_blocking=True)
        e_big = torch.cuda.Event()
        e_big.record()
        t1 = time.perf_counter()
        with torch.cuda.stream(side):
            s = torch.from_numpy(sub).to(dev, non_blocking=True)
            v, _ = torch.sort(Dd.to(dev, non_blocking=True))
            pick = v[249749:249751].cpu()
        t2 = time.perf_counter()
        e_big.synchronize()
        t3 = time.perf_counter()
        print(f'rep {rep}: enqueue big {1e3 * (t1 - t0):.3f} ms, side upload+sort+readback done at '
              f'{1e3 * (t2 - t0):.3f} ms, big upload done at {1e3 * (t3 - t0):.3f} ms', flush=True)
    del g, s, pick


if __name__ == '__main__':
    main()
