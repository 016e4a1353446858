"""Stress of the persistent kernels' exchange and the near-tie guard's late check: many back-to-back runs
of the same problems (1 .. 256 blocks, every plan: 1 / 2 / 4-row 256-thread, 512-thread compact-only and
general, batch), each compared with the first run's indices, running sums, guard verdict and final guard
state -- a timing-dependent race shows up as a run that differs.  Prints one line per problem."""
import sys
import time

import numpy as np
import torch

from stein_thinning import _native as nat
from stein_thinning import thinning as st
from stein_thinning.device import greedy_concurrent
from tests import margins_ref as mr

BOUNDS = 1088 // 8


def run(prob, m):
    idx, a, ws = prob.greedy_buffers(m)
    prob.greedy_launch(m, idx, a, ws)
    torch.cuda.synchronize()
    return (idx.cpu().numpy().copy(), a[:prob.n].cpu().numpy().copy(), nat.near_tie_step(ws),
            ws[BOUNDS:BOUNDS + 5].cpu().numpy().copy())


def main(reps):
    cases = [(60, 50), (300, 200), (700, 300), (5000, 300), (70_000, 200), (130_000, 200), (600_000, 100),
             (2_100_000, 40)]
    bad = 0
    for n, m in cases:
        X, G, _ = mr.near_tie_twins(7, n=n)
        prob = st._make_stein_integrand(X, G).device_problem()
        ref = run(prob, m)
        t0 = time.perf_counter()
        diffs = 0
        for _ in range(reps):
            got = run(prob, m)
            same = (np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]) and got[2] == ref[2]
                    and np.array_equal(got[3], ref[3]))
            diffs += not same
        bad += diffs
        print(f'n={n:8d} m={m:4d} reps={reps}  differing runs {diffs}  flag {ref[2]}  '
              f'{(time.perf_counter() - t0) / reps * 1e3:.2f} ms per run', flush=True)
    # batch launch: 4 chains side by side, repeated
    probs = []
    for k, n in enumerate((40_000, 41_000, 47_000, 60_000)):
        X, G, _ = mr.near_tie_twins(20 + k, n=n)
        probs.append(st._make_stein_integrand(X, G).device_problem())
    first = greedy_concurrent(probs, 100, dedup=False, guard=True)
    diffs = 0
    for _ in range(max(1, reps // 4)):
        got = greedy_concurrent(probs, 100, dedup=False, guard=True)
        diffs += sum(not np.array_equal(a, b) for a, b in zip(first, got))
    bad += diffs
    print(f'batch of 4  differing results {diffs}', flush=True)
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main(int(sys.argv[1]) if len(sys.argv) > 1 else 50))
