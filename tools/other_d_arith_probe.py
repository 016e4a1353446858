"""The launch-per-step kernels (d outside {2, 4}) in each arithmetic: under the near-tie guard the drop-in
runs these d in the exact arithmetic; this prints what that costs against the compact one (n = 5e5,
m = 200, d = 1 / 3 / 8 / 16, Langevin 'id', HIP events around DeviceProblem.greedy_launch, median of 5)."""
import numpy as np
import torch

from stein_thinning import _native as nat
from stein_thinning import thinning as st


def main():
    m = 200
    for d in (1, 3, 8, 16):
        rng = np.random.default_rng(d)
        x = rng.normal(size=(500_000, d))
        integrand = st._make_stein_integrand(x, -x)
        prob = integrand.device_problem()
        out = []
        for ar in ('compact', 'exact'):
            with nat.arithmetic_override(ar):
                idx, a, ws = prob.greedy_buffers(m)
                prob.greedy_launch(m, idx, a, ws)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
                for e0, e1 in evs:
                    e0.record()
                    prob.greedy_launch(m, idx, a, ws)
                    e1.record()
                torch.cuda.synchronize()
                out.append((ar, float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])),
                            idx.cpu().numpy().copy()))
        same = np.array_equal(out[0][2], out[1][2])
        print(f'd={d:2d}  compact {out[0][1]:8.3f} ms  exact {out[1][1]:8.3f} ms  ratio {out[1][1] / out[0][1]:5.3f}'
              f'  same indices {same}', flush=True)


if __name__ == '__main__':
    main()
