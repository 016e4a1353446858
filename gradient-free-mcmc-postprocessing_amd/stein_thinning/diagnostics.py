"""Near-tie diagnostics for the greedy selection: per step, how far the
runner-up's running sum is from the winner's, against the error band of the kernels' arithmetic.

The reference's NumPy path is itself only reproducible to about an ulp per pair (its SIMD ``pow``
differs from a correctly rounded one on ~5 % of inputs), so two evaluations -- NumPy's, and either of
this engine's arithmetics -- can only be guaranteed to select the same row when the step's argmin
margin exceeds what their pair values may differ by.  ``greedy_margins`` runs the greedy loop on the
launch-per-step kernels (the same bits as the persistent kernel) and after every step reads the
running sums A on the device:

* ``margin_ulps[t]`` -- (second-smallest distinct A) - (smallest A), in ulps of the smallest, as
  ``tests/golden/make_config_golden.py`` measures the NumPy path's margins;
* ``band_ulps[t]`` -- the bound on how much the winner's and the runner-up's sums may differ from
  NumPy's: per pair term c ulps of the magnitudes the Stein kernel value is built from
  (``scale`` below; c = 8 for the compact arithmetic -- the per-pair bound
  ``tests/test_oracle_compact.py`` checks -- and 2 for the exact one, whose correctly rounded powers
  are within an ulp of NumPy's), plus an ulp of the sum per step for the propagated rounding;
* ``flagged[t]`` -- margin <= band, or rows tied with the winner that are not exact duplicates of it
  (duplicated rows of an MCMC chain tie exactly in every evaluation and resolve to the lowest index,
  like np.argmin): the selection at that step was decided inside the arithmetic's error band.

Per pair (x_i, g_i), (x_j, g_j) with delta = x_i - x_j, S = |delta|^2, qf = 1 + l S:
    scale = 3 l^2 S / qf^2.5 + (tr + l sum_k |(g_i - g_j)_k delta_k|) / qf^1.5 + sum_k |g_ik g_jk| / qf^0.5
(times w_i w_j for the gradient-free kernel); the diagonal's scale is tr + |g_i|^2 (times w_i^2).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _native as nat

BAND_ULPS_PER_TERM = {'compact': 8.0, 'exact': 2.0}


@dataclass
class GreedyMargins:
    indices: np.ndarray       # (m,) uint32 -- the selection (identical to DeviceProblem.greedy's)
    margin_ulps: np.ndarray   # (m,) float: runner-up minus winner, in ulps of the winner's sum (inf: no runner-up)
    band_ulps: np.ndarray     # (m,) float: error band of the winner's and the runner-up's sums, same units
    runner_up: np.ndarray     # (m,) int64: lowest row holding the second-smallest distinct sum (-1: none)
    ties: np.ndarray          # (m,) int64: rows sharing the smallest sum (duplicated rows included)
    flagged: np.ndarray       # (m,) bool: the step was decided inside the error band
    arithmetic: str

    def flagged_steps(self) -> np.ndarray:
        return np.flatnonzero(self.flagged)


def _ulp(torch, v):
    """spacing(|v|) elementwise (np.spacing for finite values)."""
    a = v.abs()
    return torch.nextafter(a, torch.full_like(a, float('inf'))) - a


def pair_scale(torch, xi, gi, xj, gj, l: float, tr: float):
    """``scale`` of the module docstring for rows (d, k) against one row (d, 1) (torch, fp64)."""
    delta = xi - xj
    S = (delta * delta).sum(0)
    qf = 1.0 + l * S
    sq = torch.sqrt(qf)
    return (3.0 * l * l * S / (qf * qf * sq) + (tr + l * ((gi - gj) * delta).abs().sum(0)) / (qf * sq)
            + (gi * gj).abs().sum(0) / sq)


def greedy_margins(prob, n_points: int) -> GreedyMargins:
    """Greedy run on ``prob`` (a DeviceProblem) with the margin bookkeeping above, one step launch
    at a time on the current stream (a diagnostic: a few small device reductions per step)."""
    import torch
    n, m = prob.n, int(n_points)
    arith = nat.arithmetic() if prob.d <= 8 else 'exact'
    c = BAND_ULPS_PER_TERM[arith]
    idx, a, ws = prob.greedy_buffers(m)
    L = nat.lib()
    x, g = prob.x[:, :n], prob.g[:, :n]
    w = prob.w[:n] if prob.w is not None else None
    A = a[:n]
    # running error band per row: c ulps of every term's scale, plus one ulp of the sum per step
    diag_scale = prob.tr + (g * g).sum(0)
    if w is not None:
        diag_scale = diag_scale * w * w
    band = c * _ulp(torch, diag_scale)
    inf = torch.full((1,), float('inf'), dtype=torch.float64, device=prob.device)
    margin = np.full(m, np.inf)
    bandu = np.zeros(m)
    runner = np.full(m, -1, dtype=np.int64)
    ties = np.zeros(m, dtype=np.int64)
    flagged = np.zeros(m, dtype=bool)
    chosen = np.zeros(m, dtype=np.int64)
    for t in range(m):
        nat.check(L.st_greedy_steps(
            nat.ptr(prob.x), nat.ptr(prob.g), nat.ptr(prob.w), n, prob.d, prob.ld, prob.l, prob.tr, t, t + 1, m,
            nat.ptr(idx), nat.ptr(a), nat.ptr(ws), ws.numel() * 8, nat.stream_handle()), 'st_greedy_steps')
        if t > 0:   # A now includes 2 k(., x_j) for j = the previous winner
            j = int(chosen[t - 1])
            sc = pair_scale(torch, x, g, x[:, j:j + 1], g[:, j:j + 1], prob.l, prob.tr)
            if w is not None:
                sc = sc * w * w[j]
            band = band + 2.0 * c * _ulp(torch, sc) + _ulp(torch, A)
        if torch.isnan(A).any():   # np.argmin picks the first NaN: no margin to speak of
            chosen[t] = int(torch.nonzero(torch.isnan(A))[0, 0])
            margin[t] = np.nan
            continue
        best = A.min()
        eq = A == best
        b = int(torch.nonzero(eq)[0, 0])
        chosen[t] = b
        ties[t] = int(eq.sum())
        rest = torch.where(eq, inf, A)
        second = rest.min()
        tie_hazard = False
        if ties[t] > 1:   # tied rows that are not duplicates of the winner tie only by accident
            rows = torch.nonzero(eq)[:, 0]
            same = (x[:, rows] == x[:, b:b + 1]).all(0) & (g[:, rows] == g[:, b:b + 1]).all(0)
            if w is not None:
                same &= w[rows] == w[b]
            tie_hazard = not bool(same.all())
        ub = float(_ulp(torch, best.reshape(1))[0])
        if torch.isfinite(second):
            r = int(torch.nonzero(rest == second)[0, 0])
            runner[t] = r
            gap = float(second - best)
            bb = float(band[b] + band[r])
            margin[t] = gap / ub if ub > 0 else np.inf
            bandu[t] = bb / ub if ub > 0 else np.inf
            flagged[t] = tie_hazard or gap <= bb
        else:
            flagged[t] = tie_hazard
    got = idx.cpu().numpy().view(np.uint32).copy()
    if not np.array_equal(got.astype(np.int64), chosen):
        raise nat.HipExtensionError('greedy_margins: device argmin disagrees with the step kernels')
    return GreedyMargins(got, margin, bandu, runner, ties, flagged, arith)


def thin_margins(sample, gradient, n_points: int, standardize: bool = True, preconditioner='id') -> GreedyMargins:
    """``thin``'s selection with the per-step margin diagnostics (same arguments as thin)."""
    from .thinning import _make_stein_integrand
    return greedy_margins(_make_stein_integrand(sample, gradient, standardize, preconditioner).device_problem(),
                          n_points)


def thin_gf_margins(sample, log_p, log_q, gradient_q, n_points: int, standardize: bool = True,
                    range_cap=None, preconditioner='id') -> GreedyMargins:
    """``thin_gf``'s selection with the per-step margin diagnostics (same arguments as thin_gf)."""
    from .thinning import _make_stein_gf_integrand
    integrand = _make_stein_gf_integrand(sample, log_p, log_q, gradient_q, standardize, range_cap, preconditioner)
    return greedy_margins(integrand.device_problem(), n_points)
