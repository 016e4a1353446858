"""NumPy restatement of stein_thinning.diagnostics.greedy_margins over the C bit model (test
infrastructure): per step, the running sums A of the bit model (oracle/stein_ref.c, the kernels'
arithmetic) -> winner, runner-up, margin in ulps, and the error band of the module's definition."""
import numpy as np

from stein_thinning.diagnostics import BAND_ULPS_PER_TERM
from tests import oracle_c


def near_tie_twins(seed: int = 0, n: int = 400, nudge: int = 4, steps=(8, 9, 10, 11, 12)):
    """Bivariate Gaussian (Gradient_free_Stein_thinning.ipynb's target, n rows) plus a twin of each row
    the NumPy path selects at `steps`, with x[:, 0] moved by `nudge` ulps (same score): at those steps
    the winner has a runner-up a few ulps of its running sum away and the selection rests on the pair
    values' last bits.  Returns (x, g, steps)."""
    from oracle import stein_numpy as o
    rng = np.random.default_rng(seed)
    cov = np.array([[1, .8], [.8, 1]])
    x = rng.multivariate_normal([0, 0], cov, size=n)
    g = -np.linalg.solve(cov, x.T).T
    pick = o.thin(x, g, max(steps) + 1)[list(steps)]
    xt = x[pick].copy()
    for _ in range(nudge):
        xt[:, 0] = np.nextafter(xt[:, 0], np.inf)
    return np.vstack([x, xt]), np.vstack([g, g[pick]]), np.array(steps)


def _scale(s, gs, j, l, tr):
    delta = s - s[j]
    S = np.sum(delta * delta, axis=1)
    qf = 1.0 + l * S
    sq = np.sqrt(qf)
    return (3.0 * l * l * S / (qf * qf * sq) + (tr + l * np.sum(np.abs((gs - gs[j]) * delta), axis=1)) / (qf * sq)
            + np.sum(np.abs(gs * gs[j]), axis=1) / sq)


def margins(s, gs, w, l, tr, m, arith):
    c = BAND_ULPS_PER_TERM[arith]
    diag = tr + np.sum(gs * gs, axis=1)
    if w is not None:
        diag = diag * w * w
    band = c * np.spacing(np.abs(diag))
    out = {'indices': [], 'margin_ulps': [], 'band_ulps': [], 'flagged': []}
    for t in range(m):
        _, A = oracle_c.greedy(s, gs, w, l, tr, t + 1, arith=arith)   # sums whose argmin is idx[t]
        if t > 0:
            j = out['indices'][t - 1]
            sc = _scale(s, gs, j, l, tr)
            if w is not None:
                sc = sc * w * w[j]
            band = band + 2.0 * c * np.spacing(np.abs(sc)) + np.spacing(np.abs(A))
        b = int(np.argmin(A))
        best = A[b]
        eq = A == best
        rest = np.where(eq, np.inf, A)
        r = int(np.argmin(rest))
        ub = np.spacing(abs(best))
        gap = rest[r] - best
        # rows tied with the winner that are not exact duplicates of it tie only by accident
        same = np.all(s[eq] == s[b], axis=1) & np.all(gs[eq] == gs[b], axis=1)
        if w is not None:
            same &= w[eq] == w[b]
        out['indices'].append(b)
        out['margin_ulps'].append(gap / ub)
        out['band_ulps'].append((band[b] + band[r]) / ub)
        out['flagged'].append(bool(gap <= band[b] + band[r]) or not bool(same.all()))
    return {k: np.array(v) for k, v in out.items()}
