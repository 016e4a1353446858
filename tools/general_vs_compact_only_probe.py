"""The 512-thread general kernel (what every rank of a multi-GPU run uses) against the single-device
compact-only kernel at the size where the plan switches (4 096 rows per block on 256 blocks): config-4
prefixes of 256 x 4 095 rows (general, 8 register rows) and 256 x 4 096 rows (compact-only, 8 rows),
near-tie guard off, m = 1000, median of 5."""
import numpy as np
import torch

import bench
from stein_thinning import _native as nat


def main():
    nat.set_near_tie_guard(False)
    integrand, _, _ = bench.make_integrand(dict(bench.CONFIGS['c4']))
    full = integrand.device_problem()
    m = 1000
    for rpb in (4095, 4096, 4200):
        prob = full.subset(np.arange(256 * rpb))
        idx, a, ws = prob.greedy_buffers(m)
        prob.greedy_launch(m, idx, a, ws)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for e0, e1 in evs:
            e0.record()
            prob.greedy_launch(m, idx, a, ws)
            e1.record()
        torch.cuda.synchronize()
        ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in evs]))
        print(f'rows/block {rpb}  {ms:.3f} ms  {ms:.3f} us/step  ({"compact-only" if rpb >= 4096 else "general"})',
              flush=True)


if __name__ == '__main__':
    main()
