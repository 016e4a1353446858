"""Register rows of the mid-size compact-only kernel (persistent_cmp.hip): config-4 prefixes of 256 x R
rows for R from 1 900 to 3 900 rows per block, on the general kernel (st_tune key 12 = 0) and the
compact-only kernel forced to 4 / 6 / 8 register rows (the rest of a block in LDS); near-tie guard off,
m = 1000, median of 5 launches.  Empty register slots are swept like full ones, so the fewest rows that
hold the block are not always the fastest."""
import numpy as np
import torch

import bench
from stein_thinning import _native as nat


def main():
    nat.set_near_tie_guard(False)
    integrand, _, _ = bench.make_integrand(dict(bench.CONFIGS['c4']))
    full = integrand.device_problem()
    L = nat.lib()
    m = 1000
    for rpb in (1900, 2300, 2700, 3100, 3500, 3900):
        prob = full.subset(np.arange(256 * rpb))
        out = []
        for key in (-1, 0, 4, 6, 8):
            nat.check(L.st_tune(12, key), 'st_tune')
            try:
                idx, a, ws = prob.greedy_buffers(m)
                prob.greedy_launch(m, idx, a, ws)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
                for e0, e1 in evs:
                    e0.record()
                    prob.greedy_launch(m, idx, a, ws)
                    e1.record()
                torch.cuda.synchronize()
            finally:
                L.st_tune(12, -1)
            out.append(float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])))
        print(f'rows/block {rpb}  auto {out[0]:.3f}  general {out[1]:.3f}  cmp4 {out[2]:.3f}  cmp6 {out[3]:.3f}  '
              f'cmp8 {out[4]:.3f} ms', flush=True)


if __name__ == '__main__':
    main()
