"""How evenly the LV phase-B kernels spread a parameter point's observation points over a wave's 64
lanes (measurement aid, host only): scipy's RK45 steps (the reference's solver, the same accepted
steps the kernel's phase A records) at the bench's parameter points, then per point the busiest
lane's share against a perfect split of the t_n observation points.

* per-step pieces (lv_dense_kernel): the smallest P with
  sum_s ceil(len_s / P) <= 64, one piece per lane;
* balanced pieces: P = ceil(t_n / 64) across step bounds (round 4's lv_dense_bal_kernel, which switched
  step records inside a piece: measured slower and removed, profiles/r04_lv_balanced_pieces_rejected.log);
* K pieces dealt longest-first to 64 lanes (for reference).

    python tools/lv_piece_balance.py [points]
"""
import os
import sys

import numpy as np
from scipy.integrate import solve_ivp

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd'))

from oracle import lv_numpy as ol  # noqa: E402
from stein_thinning import lotka_volterra as lv  # noqa: E402


def main():
    npts = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    data = lv.reference_data()
    t, _, s = lv._settings(data, lv.RTOL, lv.ATOL)
    rng = np.random.default_rng(12350)   # bench.py main_lv's parameter draw
    eff = {'per-step': [], 'balanced': [], 'lpt128': [], 'lpt256': []}
    steps = []
    for _ in range(npts):
        theta = np.exp(np.log(lv.THETA) + 0.05 * rng.normal(size=4))
        sol = solve_ivp(ol.lotka_volterra_sensitivity, (s[0], s[1]), np.concatenate([[s[2], s[3]], np.zeros(8)]),
                        args=(theta,), dense_output=True, rtol=s[4], atol=s[5])
        lens = np.histogram(t, bins=sol.t)[0]
        steps.append(lens.size)
        P = max(1, (t.size + 63) // 64)
        while np.sum(np.ceil(lens / P)) > 64:
            P += 1
        eff['per-step'].append(t.size / (64 * P))
        eff['balanced'].append(t.size / (64 * ((t.size + 63) // 64)))
        for K, key in ((128, 'lpt128'), (256, 'lpt256')):
            P = 1
            while np.sum(np.ceil(lens / P)) > K:
                P += 1
            pieces = sorted((min(P, L - j * P) for L in lens for j in range(int(np.ceil(L / P)))), reverse=True)
            load = np.zeros(64)
            for p in pieces:
                load[np.argmin(load)] += p
            eff[key].append(t.size / (64 * load.max()))
    print(f't_n = {t.size}, {npts} points, accepted steps per point {np.mean(steps):.1f}')
    for k, v in eff.items():
        print(f'{k:9s}: busiest-lane efficiency mean {np.mean(v):.3f}, min {np.min(v):.3f}')


if __name__ == '__main__':
    main()
