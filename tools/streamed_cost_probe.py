"""What the streamed rows cost the config-4 persistent kernel: thin time per step for row counts per
block around the point where the register (9 x 512) and LDS rows (2 240 at d = 4) are full, on
prefixes of the config-4 sample (same data, same kernel: compact-only, 512 threads, RT 9).  The slope
past the knee is the per-row cost of a streamed row, against the slope below it (LDS rows)."""
import time

import numpy as np
import torch

import bench
from stein_thinning import _native as nat


def main():
    nat.set_near_tie_guard(False)
    cfg = dict(bench.CONFIGS['c4'])
    integrand, _, _ = bench.make_integrand(cfg)
    full = integrand.device_problem()
    m = 1000
    stream = torch.cuda.current_stream()
    rows_per_block = [4608, 5600, 6400, 6848, 7100, 7400, 7700, 7813]
    prev = None
    for rpb in rows_per_block:
        n = 256 * rpb
        prob = full.subset(np.arange(min(n, full.n)))
        idx, a, ws = prob.greedy_buffers(m)
        prob.greedy_launch(m, idx, a, ws)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for e0, e1 in evs:
            e0.record(stream)
            prob.greedy_launch(m, idx, a, ws)
            e1.record(stream)
        torch.cuda.synchronize()
        ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in evs]))
        streamed = max(0, rpb - 9 * 512 - 2240)
        line = f'rows/block {rpb:5d}  streamed/block {streamed:4d}  {ms:7.3f} ms  {ms:6.3f} us/step'
        if prev is not None:
            line += f'  slope {(ms - prev[1]) / (rpb - prev[0]) * 1e3:6.2f} ns/row-per-block per step'
        print(line, flush=True)
        prev = (rpb, ms)
        del prob, idx, a, ws


if __name__ == '__main__':
    main()
