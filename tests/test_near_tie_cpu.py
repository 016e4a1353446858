"""Near-tie guard model on the CPU (oracle/stein_ref.c sr_greedy_mt_ties, the kernels' rule): it flags
exactly the constructed near-ties, never a step of the reference fixtures or of the BASELINE configs
(raw rows or run starts: ties between bitwise-equal rows do not count), and every departure of the compact arithmetic from the NumPy path lies at or after a
flagged step (so the drop-in's exact re-run of a flagged thin reproduces the NumPy selection)."""
import warnings

import numpy as np
import pytest

from oracle import models
from oracle import stein_numpy as o
from oracle import stein_ref_c as oc
from tests import margins_ref as mr
from stein_thinning import thinning as st


def _ties(integrand, m, arith='compact'):
    return oc.greedy_ties(integrand.sample, integrand.gradient, integrand.weights, integrand.linv_scale,
                          integrand.linv_trace, m, arith=arith)


@pytest.mark.parametrize('seed', range(10))
def test_model_flags_the_constructed_near_ties(seed):
    X, G, steps = mr.near_tie_twins(seed)
    integrand = st._make_stein_integrand(X, G)
    idx, _, gap, thr, flagged = _ties(integrand, 30)
    np.testing.assert_array_equal(np.flatnonzero(flagged), steps)
    want = o.thin(X, G, 30)
    bad = np.flatnonzero(idx != want)
    if bad.size:   # the compact arithmetic departs from NumPy only where the guard has flagged
        assert flagged[:bad[0] + 1].any()
    exact, *_ = _ties(integrand, 30, 'exact')
    np.testing.assert_array_equal(exact, want)
    assert np.all((gap / thr)[~flagged] > 1e6)   # everything else is far outside the band
    assert not _ties(integrand, 30, 'exact')[4].any()   # the exact arithmetic is never flagged


def _golden_problems():
    sample, gradient, log_p, _, _ = models.bivariate_reference_sample(1000)
    log_q, gq, _, _ = models.gaussian_proxy(sample, 2)
    gm, _, gm_logpdf, gm_score = models.gm_reference_sample(1000)
    gm_grad, gm_logp = gm_score(gm), gm_logpdf(gm)
    gm_logq, gm_gq, _, _ = models.gaussian_proxy(gm, 1)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        return {
            'F1a': (st._make_stein_integrand(sample, gradient), 20),
            'F1c': (st._make_stein_gf_integrand(sample, log_p, log_q, gq), 20),
            'F2a': (st._make_stein_integrand(gm, gm_grad, preconditioner='med'), 1000),
            'F2b': (st._make_stein_gf_integrand(gm, gm_logp, gm_logq, gm_gq, preconditioner='med'), 1000),
        }


def test_reference_fixtures_are_never_flagged():
    for name, (integrand, m) in _golden_problems().items():
        _, _, gap, thr, flagged = _ties(integrand, m)
        assert not flagged.any(), name
        assert np.min(gap / thr) > 100, (name, np.min(gap / thr))


def test_threshold_recurrence():
    integrand, m = _golden_problems()['F2a']
    idx, _, _, thr, _, wv = oc.greedy_ties(integrand.sample, integrand.gradient, None, integrand.linv_scale,
                                           integrand.linv_trace, m, winner_sums=True)
    g2, w2 = oc.tie_bounds(integrand.gradient, None)
    assert w2 == 1.0 and np.isclose(g2, np.max(np.sum(integrand.gradient ** 2, axis=1)), rtol=1e-15)
    np.testing.assert_array_equal(thr, model_thresholds(integrand.gradient, None, integrand.linv_scale,
                                                        integrand.linv_trace, idx, wv)[0][:m])
    assert thr[0] == 2.0 ** -50 * (8.0 * (integrand.linv_trace + g2))
    assert np.all(np.diff(thr) > 0)


def model_thresholds(g, w, l, tr, idx, wv):
    """thr(0 .. m) of the guard recurrence (stein_ref.c tie_init / tie_step) in Python floats -- the same
    IEEE operations in the same order (tests compare the kernels' final state with thr(m) bit for bit);
    also returns the final Q and E."""
    import math
    g2max, w2max = oc.tie_bounds(g, w)
    c1 = (((3.0 * l + tr) + math.sqrt(l) * math.sqrt(g2max)) + 0.5 * l) + 0.5 * g2max
    wmax = math.sqrt(w2max)
    dmax = (tr + g2max) * w2max
    Q = E = 0.0
    out = [2.0 ** -50 * (8.0 * dmax)]
    for t in range(1, len(idx) + 1):
        j = int(idx[t - 1])
        Q = Q + float(wv[t - 1])
        row = g[j]
        gj2 = float(row[0]) * float(row[0])
        for k in range(1, row.shape[0]):
            gj2 = gj2 + float(row[k]) * float(row[k])
        wj = 1.0 if w is None else float(w[j])
        scale = (c1 + gj2) * (wmax * wj)
        E = E + (16.0 * scale + (2.0 * dmax + max(Q, 0.0)))
        out.append(2.0 ** -50 * (8.0 * dmax + E))
    return np.array(out), Q, E


def _run_starts(s, g, w):
    same = np.all(s[1:] == s[:-1], axis=1) & np.all(g[1:] == g[:-1], axis=1)
    if w is not None:
        same &= w[1:] == w[:-1]
    return np.concatenate([[0], 1 + np.flatnonzero(~same)])


@pytest.mark.parametrize('name', ['c2', 'c3'])
def test_baseline_configs_unflagged(name):
    """Configs 2 and 3 (n = 2e5, m = 100): neither the run starts nor the raw rows -- ~77 % repeats, whose
    exact ties with the winner are ties between bitwise-equal rows and do not count -- carry a flag, with
    the same margins (round 5's rule flagged the raw rows at step 0)."""
    import bench
    integrand, _, _ = bench.make_integrand(dict(bench.CONFIGS[name]))
    s, g, w = integrand.sample, integrand.gradient, integrand.weights
    rows = _run_starts(s, g, w)
    assert rows.size < 0.3 * s.shape[0]
    m = bench.CONFIGS[name]['m']
    idx_r, _, gap_r, thr_r, flagged_r = oc.greedy_ties(s[rows], g[rows], None if w is None else w[rows],
                                                       integrand.linv_scale, integrand.linv_trace, m)
    assert not flagged_r.any() and np.min(gap_r / thr_r) > 1e3
    idx, _, gap, thr, flagged = _ties(integrand, m)
    assert not flagged.any()
    np.testing.assert_array_equal(idx, rows[idx_r])
    np.testing.assert_array_equal(gap, gap_r)   # the duplicates change nothing: same runner-ups


def test_non_adjacent_duplicates_do_not_flag():
    """Pooled identical chains and a permuted sample: every row has bitwise duplicates far from it (no
    adjacent repeat to drop), so the winner ties exactly at every step -- never flagged, the selection
    is the NumPy path's."""
    X, G = models.bivariate_reference_sample(500)[:2]
    for name, (Xp, Gp) in {'pooled': (np.vstack([X, X]), np.vstack([G, G])),
                           'permuted': (lambda p: (np.vstack([X, X])[p], np.vstack([G, G])[p]))(
                               np.random.default_rng(3).permutation(1000))}.items():
        integrand = st._make_stein_integrand(Xp, Gp)
        idx, _, gap, thr, flagged = _ties(integrand, 40)
        assert not flagged.any(), name
        assert np.min(gap / thr) > 1e6, name
        np.testing.assert_array_equal(idx, o.thin(Xp, Gp, 40))


def test_exact_tie_between_different_rows_flags():
    """An exact tie between rows that are NOT equal bit for bit still counts: rows r and -r of a standard
    Gaussian sample (score -x) have the same diagonal term, so with both nearest the origin step 0 ties
    exactly between different rows -- flagged."""
    rng = np.random.default_rng(8)
    X = rng.normal(size=(300, 2))
    X = X[np.sum(X * X, axis=1) > 0.5]
    X[3] = [0.125, -0.25]
    X[200] = -X[3]
    integrand = st._make_stein_integrand(X, -X, standardize=False)
    idx, _, gap, thr, flagged = _ties(integrand, 3)
    assert idx[0] == 3 and gap[0] == 0.0 and flagged[0]
