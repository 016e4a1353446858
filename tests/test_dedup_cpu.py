"""Run detection of the repeated-row path on the host (SteinIntegrand.run_starts_view: the row-sharded
thin's rule; the device kernels st_run_starts / st_run_compact are checked against it in
tests/test_gpu_dedup.py) against a plain loop: bitwise row comparison over x, g and w."""
import numpy as np
import pytest

from stein_thinning import thinning as st


def _loop(x, g, w):
    n = x.shape[0]
    keep = np.ones(n, dtype=bool)
    for i in range(1, n):
        same = (x[i].tobytes() == x[i - 1].tobytes()) and (g[i].tobytes() == g[i - 1].tobytes())
        if w is not None:
            same = same and w[i].tobytes() == w[i - 1].tobytes()
        keep[i] = not same
    return np.flatnonzero(keep)


@pytest.mark.parametrize('weights', [False, True])
def test_run_starts_view_matches_loop(weights):
    rng = np.random.default_rng(5)
    n, d = 3_001, 3
    x = rng.normal(size=(n, d))
    rep = rng.random(n) < 0.7
    for i in range(1, n):
        if rep[i]:
            x[i] = x[i - 1]
    g = -2.0 * x
    w = np.exp(x[:, 0]) if weights else None
    # edge rows: a signed zero, a gradient-only change, a weight-only change
    x[100] = x[99]
    g[100] = g[99]
    x[99, 1], x[100, 1] = 0.0, -0.0
    x[201], g[201] = x[200], g[200].copy()
    g[201, 0] = np.nextafter(g[201, 0], np.inf)
    if w is not None:
        x[301], g[301] = x[300], g[300]
        w[301] = np.nextafter(w[300], -np.inf)
    integ = st.SteinIntegrand(x, g, np.eye(d), w)
    compact, rows = integ.run_starts_view()
    want = _loop(x, g, w)
    np.testing.assert_array_equal(rows, want)
    assert 100 in rows and 201 in rows
    assert np.array_equal(compact.sample, x[want]) and np.array_equal(compact.gradient, g[want])
    if w is not None:
        assert 301 in rows and np.array_equal(compact.weights, w[want])


def test_run_starts_view_declines_without_repeats():
    x = np.random.default_rng(1).normal(size=(500, 2))
    assert st.SteinIntegrand(x, -x, np.eye(2)).run_starts_view() is None
