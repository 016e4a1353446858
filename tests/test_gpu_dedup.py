"""Repeated-row path on the GPU (DeviceProblem.dedup_view, the drop-in thin's default): thinning the
run starts of an MCMC sample selects the same rows as thinning every row, and the running sums
expanded back to all rows are bit-identical -- against the full device run and the C bit model.
"""
import numpy as np
import pytest

from oracle import stein_numpy as o
from tests import oracle_c

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

import stein_thinning  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402
from stein_thinning.device import DeviceProblem  # noqa: E402


def _chain(n, d, seed, accept=0.25):
    """Random-walk chain: each proposal accepted with probability ``accept``, else the previous row
    repeats (so ~1 - accept of the rows repeat their predecessor)."""
    rng = np.random.default_rng(seed)
    x = np.empty((n, d))
    x[0] = rng.normal(size=d)
    acc = rng.random(n) < accept
    for i in range(1, n):
        x[i] = x[i - 1] + 0.3 * rng.normal(size=d) if acc[i] else x[i - 1]
    g = -x * np.linspace(0.5, 2.0, d)
    return x, g


def _inputs(x, g, gf):
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    w = None
    if gf:
        w = np.exp(0.1 * np.tanh(s[:, 0]))   # weights that repeat with their rows
    return s, gs, w, float(linv[0, 0]), float(np.trace(linv))


@pytest.mark.parametrize('d', [1, 2, 4, 8, 16])
@pytest.mark.parametrize('gf', [False, True])
def test_dedup_bit_exact(d, gf):
    n, m = 40_001, 60
    x, g = _chain(n, d, seed=100 + d)
    s, gs, w, l, tr = _inputs(x, g, gf)
    prob = DeviceProblem(s, gs, w, l, tr)
    view = prob.dedup_view()
    assert view is not None and view.n_unique < 0.4 * n
    want, want_A = prob.greedy(m, return_sums=True)
    got, got_A = prob.greedy(m, return_sums=True, dedup='always')
    np.testing.assert_array_equal(got, want)
    assert np.array_equal(got_A, want_A), np.flatnonzero(got_A != want_A)[:10]
    cidx, cA = oracle_c.greedy(s, gs, w, l, tr, m)
    np.testing.assert_array_equal(got, cidx)
    assert np.array_equal(got_A, cA)
    # every selected row is a run start
    assert np.all(np.isin(got, view.rows_host))


def test_dedup_keeps_nonadjacent_copies_and_signed_zeros():
    """Only a row equal bit for bit to the row BEFORE it is dropped: copies elsewhere in the chain
    (a later chain revisiting a state, pooled chains) stay candidates and tie at the lower index, and
    rows differing only in the sign of a zero, or in their weight, are different rows."""
    n, m = 30_000, 80
    x, g = _chain(n, 4, seed=7)
    x[20_000:20_500] = x[1_000:1_500]
    g[20_000:20_500] = g[1_000:1_500]
    s, gs, w, l, tr = _inputs(x, g, True)
    s[5_001] = s[5_000]
    gs[5_001] = gs[5_000]
    s[5_000, 2], s[5_001, 2] = 0.0, -0.0
    w[5_003] = np.nextafter(w[5_002], np.inf)
    s[5_003], gs[5_003] = s[5_002], gs[5_002]
    prob = DeviceProblem(s, gs, w, l, tr)
    view = prob.dedup_view()
    assert view is not None
    keep = set(view.rows_host.tolist())
    assert {5_000, 5_001, 5_002, 5_003} <= keep
    got, got_A = prob.greedy(m, return_sums=True, dedup='always')
    want, want_A = prob.greedy(m, return_sums=True)
    np.testing.assert_array_equal(got, want)
    assert np.array_equal(got_A, want_A)


def test_dedup_skipped_without_repeats():
    """An iid sample has no repeats: no compact problem, the plain run."""
    rng = np.random.default_rng(3)
    x = rng.normal(size=(5_000, 4))
    s, gs, w, l, tr = _inputs(x, -x, False)
    prob = DeviceProblem(s, gs, w, l, tr)
    assert prob.dedup_view() is None
    np.testing.assert_array_equal(prob.greedy(30, dedup='always'), prob.greedy(30))
    assert not prob.dedup_used


def test_run_starts_kernel_matches_host(monkeypatch):
    """st_run_starts / st_run_compact against the host rule (SteinIntegrand.run_starts_view): the
    same run starts, the compact rows bit-identical to the source rows, padding zeroed."""
    x, g = _chain(100_003, 3, seed=9)   # odd n: a partial last tile
    s, gs, w, l, tr = _inputs(x, g, True)
    prob = DeviceProblem(s, gs, w, l, tr)
    view = prob.dedup_view()
    integ = st.SteinIntegrand(s, gs, np.eye(3) * l, w)
    hv = integ.run_starts_view()
    np.testing.assert_array_equal(view.rows_host, hv[1])
    sp = view.problem
    k = sp.n
    assert np.array_equal(sp.x[:, :k].cpu().numpy().T, s[hv[1]])
    assert np.array_equal(sp.g[:, :k].cpu().numpy().T, gs[hv[1]])
    assert np.array_equal(sp.w[:k].cpu().numpy(), w[hv[1]])
    assert not sp.x[:, k:].any() and not sp.g[:, k:].any() and not sp.w[k:].any()


def test_thin_default_and_switch(monkeypatch):
    """The drop-in thin / thin_gf use the repeated-row path when it pays (here the cost gate is
    lowered to take it at this size); set_dedup(False) (or ST_DEDUP=0) turns it off; the indices never
    change."""
    from stein_thinning import device
    monkeypatch.setattr(device, 'DEDUP_MIN_SAVING_S', 0.0)
    x, g = _chain(50_000, 4, seed=11)
    integ = st._make_stein_integrand(x, g, preconditioner='med')
    a = st._greedy_search(40, integ)
    assert integ.device_problem().dedup_used
    stein_thinning.set_dedup(False)
    try:
        b = st.thin(x, g, 40, preconditioner='med')
    finally:
        stein_thinning.set_dedup(None)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(a, o.thin(x, g, 40, preconditioner='med'))
    log_p = -0.5 * np.sum(x * x, axis=1)
    log_q = -0.6 * np.sum(x * x, axis=1)
    np.testing.assert_array_equal(st.thin_gf(x, log_p, log_q, -1.2 * x, 30, preconditioner='med'),
                                  o.thin_gf(x, log_p, log_q, -1.2 * x, 30, preconditioner='med'))


@pytest.mark.parametrize('gf', [False, True])
def test_dedup_bit_exact_outside_fast_range(gf):
    """Rows outside [2^-60, 2^60] (whole runs of them, and run starts whose repeats follow) take the
    general arithmetic's per-pair rule -- still a function of the two rows only, so the thin of the run
    starts matches the full thin and the C bit model bit for bit."""
    n, m = 120_001, 40
    x, g = _chain(n, 4, seed=31)
    s, gs, w, l, tr = _inputs(x, g, gf)
    starts = np.flatnonzero(np.r_[True, np.any(s[1:] != s[:-1], axis=1)])
    rng = np.random.default_rng(5)
    pick = rng.choice(starts[:-1], size=10, replace=False)
    for k, r in enumerate(pick):          # modify whole runs so they stay runs
        end = starts[np.searchsorted(starts, r) + 1]
        if k < 4:
            gs[r:end, 0] = 1e-25
        elif k < 7:
            gs[r:end, -1] = 2e19
        else:
            s[r:end, 1] = 1e-30
    prob = DeviceProblem(s, gs, w, l, tr)
    assert prob.dedup_view() is not None
    want, want_A = prob.greedy(m, return_sums=True)
    got, got_A = prob.greedy(m, return_sums=True, dedup='always')
    np.testing.assert_array_equal(got, want)
    assert np.array_equal(got_A, want_A)
    cidx, cA = oracle_c.greedy(s, gs, w, l, tr, m)
    np.testing.assert_array_equal(got, cidx)
    assert np.array_equal(got_A, cA)


@pytest.mark.parametrize('dedup', [True, False])
def test_thin_chains_equal_the_per_chain_loop(dedup, monkeypatch):
    """stein_thinning.thin_chains (device.greedy_concurrent: the chains' persistent launches side by
    side, each on a share of the CUs) returns the reference loop's indices for every chain."""
    from stein_thinning import device
    monkeypatch.setattr(device, 'DEDUP_MIN_SAVING_S', 0.0)   # take the repeated-row path at this size
    chains = [_chain(70_000 + 1_000 * k, 4, seed=50 + k) for k in range(6)]
    stein_thinning.set_dedup(dedup)
    try:
        got = stein_thinning.thin_chains([c[0] for c in chains], [c[1] for c in chains], 40,
                                         preconditioner='med')
        want = [st.thin(x, g, 40, preconditioner='med') for x, g in chains]
    finally:
        stein_thinning.set_dedup(None)
    assert len(got) == len(chains)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(want[0], o.thin(chains[0][0], chains[0][1], 40, preconditioner='med'))


def test_thin_gf_chains_equal_the_per_chain_loop():
    chains = [_chain(30_000 + 500 * k, 3, seed=70 + k) for k in range(5)]
    lps = [-0.5 * np.sum(x * x, axis=1) for x, _ in chains]
    lqs = [-0.55 * np.sum(x * x, axis=1) for x, _ in chains]
    got = stein_thinning.thin_gf_chains([c[0] for c in chains], lps, lqs, [c[1] for c in chains], 30,
                                        preconditioner='med')
    for (x, g), lp, lq, idx in zip(chains, lps, lqs, got):
        np.testing.assert_array_equal(idx, st.thin_gf(x, lp, lq, g, 30, preconditioner='med'))
    np.testing.assert_array_equal(got[0], o.thin_gf(chains[0][0], lps[0], lqs[0], chains[0][1], 30,
                                                    preconditioner='med'))
