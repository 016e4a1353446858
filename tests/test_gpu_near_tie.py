"""Near-tie guard on the GPU: the persistent kernel's flag equals the bit model's
(oracle/stein_ref.c sr_greedy_mt_ties) -- the first flagged step, the bounds and the final threshold
state bit for bit -- and the drop-in thin with default settings returns the NumPy path's indices on the
near-tie construction where the compact arithmetic alone departs from them (tests/test_gpu_margins.py)."""
import numpy as np
import pytest

from oracle import stein_numpy as o
from oracle import stein_ref_c as oc
from tests import margins_ref as mr
from tests.test_near_tie_cpu import model_thresholds

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

import stein_thinning  # noqa: E402
from stein_thinning import _native as nat  # noqa: E402
from stein_thinning import device as dv  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402

BOUNDS = 1088 // 8   # csrc/stein_internal.hpp kWsBoundsOff: max |g|^2, max w^2, then the final Q, E, thr


def _compact_run(prob, m):
    """One st_greedy (compact arithmetic, guard on) on the problem as it is: (indices, first flagged step,
    [g2max, w2max, Q, E, thr] the kernel left in the workspace)."""
    idx, a, ws = prob.greedy_buffers(m)
    prob.greedy_launch(m, idx, a, ws)
    out = idx.cpu().numpy().view(np.uint32).copy()
    step = nat.near_tie_step(ws)
    return out, step, ws[BOUNDS:BOUNDS + 5].cpu().numpy()


@pytest.mark.parametrize('seed', range(10))
def test_kernel_flag_and_state_equal_bit_model(seed):
    X, G, steps = mr.near_tie_twins(seed)
    integrand = st._make_stein_integrand(X, G)
    prob = integrand.device_problem()
    idx, step, state = _compact_run(prob, 30)
    midx, _, gap, thr, flagged, wv = oc.greedy_ties(integrand.sample, integrand.gradient, None,
                                                    integrand.linv_scale, integrand.linv_trace, 30,
                                                    winner_sums=True)
    np.testing.assert_array_equal(idx, midx)
    assert step == steps[0] == np.flatnonzero(flagged)[0]
    g2, w2 = oc.tie_bounds(integrand.gradient, None)
    thr_all, Q, E = model_thresholds(integrand.gradient, None, integrand.linv_scale, integrand.linv_trace, midx, wv)
    np.testing.assert_array_equal(state, [g2, w2, Q, E, thr_all[-1]])


def test_kernel_state_gradient_free_and_unflagged():
    from oracle import models
    sample, gradient, log_p, _, _ = models.bivariate_reference_sample(1000)
    log_q, gq, _, _ = models.gaussian_proxy(sample, 2)
    integrand = st._make_stein_gf_integrand(sample, log_p, log_q, gq, preconditioner='med')
    idx, step, state = _compact_run(integrand.device_problem(), 200)
    midx, _, _, _, flagged, wv = oc.greedy_ties(integrand.sample, integrand.gradient, integrand.weights,
                                                integrand.linv_scale, integrand.linv_trace, 200, winner_sums=True)
    np.testing.assert_array_equal(idx, midx)
    assert step == -1 and not flagged.any()
    thr_all, Q, E = model_thresholds(integrand.gradient, integrand.weights, integrand.linv_scale,
                                     integrand.linv_trace, midx, wv)
    np.testing.assert_array_equal(state, list(oc.tie_bounds(integrand.gradient, integrand.weights)) +
                                  [Q, E, thr_all[-1]])


@pytest.mark.parametrize('seed', range(10))
def test_dropin_thin_equals_numpy_on_near_ties(seed):
    X, G, steps = mr.near_tie_twins(seed)
    integrand = st._make_stein_integrand(X, G)
    got = st._greedy_search(30, integrand)
    np.testing.assert_array_equal(got, o.thin(X, G, 30))
    prob = integrand.device_problem()
    assert prob.near_tie == steps[0]   # flagged, re-run with the exact arithmetic
    np.testing.assert_array_equal(stein_thinning.thin(X, G, 30), o.thin(X, G, 30))


def test_guard_off_keeps_the_compact_selection():
    X, G, _ = mr.near_tie_twins(0)
    want = o.thin(X, G, 30)
    nat.set_near_tie_guard(False)
    try:
        integrand = st._make_stein_integrand(X, G)
        got = st._greedy_search(30, integrand)
        assert integrand.device_problem().near_tie is None
        idx, step, _ = _compact_run(integrand.device_problem(), 30)
        assert step == -2   # the kernel computed no flag
    finally:
        nat.set_near_tie_guard(None)
    assert not np.array_equal(got, want)   # seed 0: the compact arithmetic alone departs at step 8


def test_exact_arithmetic_needs_no_guard():
    X, G, _ = mr.near_tie_twins(1)
    with nat.arithmetic_override('exact'):
        integrand = st._make_stein_integrand(X, G)
        prob = integrand.device_problem()
        assert prob.guard_mode() is None
        np.testing.assert_array_equal(st._greedy_search(30, integrand), o.thin(X, G, 30))
        assert _compact_run(prob, 30)[1] == -2


@pytest.mark.parametrize('d', [1, 3, 5, 8])
def test_other_d_run_exact(d):
    """d outside {2, 4}: the launch-per-step kernels carry no flag, so the guarded drop-in runs them in the
    exact arithmetic: NumPy's indices, near-tie twins included."""
    rng = np.random.default_rng(d)
    X = rng.normal(size=(300, d))
    G = -X
    pick = o.thin(X, G, 12)[8:12]
    Xt = X[pick].copy()
    for _ in range(4):
        Xt[:, 0] = np.nextafter(Xt[:, 0], np.inf)
    X2, G2 = np.vstack([X, Xt]), np.vstack([G, G[pick]])
    integrand = st._make_stein_integrand(X2, G2)
    assert integrand.device_problem().guard_mode() == 'exact'
    np.testing.assert_array_equal(st._greedy_search(25, integrand), o.thin(X2, G2, 25))


def test_thin_chains_guarded():
    """thin_chains (one batch launch): each chain's tie word is read, flagged chains re-run exactly."""
    problems = [mr.near_tie_twins(s)[:2] for s in range(3)]
    rng = np.random.default_rng(5)
    Z = rng.normal(size=(405, 2))
    problems.append((Z, -Z))
    got = stein_thinning.thin_chains([p[0] for p in problems], [p[1] for p in problems], 30)
    for (X, G), idx in zip(problems, got):
        np.testing.assert_array_equal(idx, o.thin(X, G, 30))


@pytest.mark.parametrize('dedup', ['always', False])
def test_config2_unflagged_run_starts_and_raw_rows(dedup):
    """Config 2 through the guarded path, on its run starts and on all 2e5 raw rows (~77 % repeats, every
    winner tied exactly by its own repeats): no step is flagged -- ties between rows equal bit for bit do not
    count -- and the indices equal the plain full thin's."""
    import bench
    cfg = dict(bench.CONFIGS['c2'])
    integrand, _, _ = bench.make_integrand(cfg)
    prob = integrand.device_problem()
    got = prob.greedy(cfg["m"], dedup=dedup, guard=True)
    assert prob.dedup_used == bool(dedup) and prob.near_tie == -1
    full, _ = oc.greedy_mt(integrand.sample, integrand.gradient, None, integrand.linv_scale, integrand.linv_trace,
                           cfg['m'])
    np.testing.assert_array_equal(got, full)


def _pooled_permuted(n=50_000, seed=4):
    """A bivariate sample pooled with an identical copy and shuffled: every row has a bitwise duplicate far
    from it (two identical chains pooled, then permuted -- nothing adjacent for dedup_view to drop)."""
    from oracle import models
    X, G = models.bivariate_reference_sample(n)[:2]
    p = np.random.default_rng(seed).permutation(2 * n)
    return np.vstack([X, X])[p], np.vstack([G, G])[p]


def test_non_adjacent_duplicates_take_no_exact_rerun():
    """The default thin() on a sample whose duplicates are all non-adjacent: the guarded kernel sees the
    winner tied exactly by its duplicate at every step and flags nothing, so no exact re-run happens; the
    indices are the NumPy path's."""
    X, G = _pooled_permuted()
    want = o.thin(X, G, 30)
    integrand = st._make_stein_integrand(X, G)
    got = st._greedy_search(30, integrand)
    prob = integrand.device_problem()
    assert not prob.dedup_used and prob.near_tie == -1   # guarded, unflagged: no re-run
    np.testing.assert_array_equal(got, want)
    _, step, _ = _compact_run(prob, 30)
    assert step == -1


def test_duplicated_near_ties_flag_like_the_model():
    """Near-tie twins in a sample pooled with its own copy: the twins still flag (a twin is not a bitwise
    duplicate of the winner), the winners' exact copies do not; first flagged step, bounds and final
    threshold state equal the bit model's, and the default thin returns NumPy's indices."""
    X, G, steps = mr.near_tie_twins(2)
    X2, G2 = np.vstack([X, X]), np.vstack([G, G])
    integrand = st._make_stein_integrand(X2, G2)
    prob = integrand.device_problem()
    idx, step, state = _compact_run(prob, 30)
    midx, _, _, _, flagged, wv = oc.greedy_ties(integrand.sample, integrand.gradient, None, integrand.linv_scale,
                                                integrand.linv_trace, 30, winner_sums=True)
    np.testing.assert_array_equal(idx, midx)
    assert step == np.flatnonzero(flagged)[0] == steps[0]
    thr_all, Q, E = model_thresholds(integrand.gradient, None, integrand.linv_scale, integrand.linv_trace, midx, wv)
    np.testing.assert_array_equal(state, list(oc.tie_bounds(integrand.gradient, None)) + [Q, E, thr_all[-1]])
    np.testing.assert_array_equal(stein_thinning.thin(X2, G2, 30), o.thin(X2, G2, 30))


def test_exact_tie_between_different_rows_flags_on_the_gpu():
    """rows r and -r (score -x) tie exactly at step 0 without being duplicates: flagged at step 0, as the
    model (tests/test_near_tie_cpu.py) says."""
    rng = np.random.default_rng(8)
    X = rng.normal(size=(300, 2))
    X = X[np.sum(X * X, axis=1) > 0.5]
    X[3] = [0.125, -0.25]
    X[200] = -X[3]
    integrand = st._make_stein_integrand(X, -X, standardize=False)
    idx, step, _ = _compact_run(integrand.device_problem(), 3)
    assert idx[0] == 3 and step == 0


def test_thin_chains_one_near_tie_chain():
    """thin_chains with a single chain (greedy_concurrent's one-at-a-time branch, also what a
    GPU with one chain of a spread runs) keeps the guard: the twins' chain returns NumPy's indices."""
    X, G, _ = mr.near_tie_twins(0)
    got = stein_thinning.thin_chains([X], [G], 30)
    np.testing.assert_array_equal(got[0], o.thin(X, G, 30))


@pytest.mark.parametrize('n', [100_000, 300_000, 600_000])
def test_dropin_equals_numpy_on_near_ties_at_scale(n):
    """The near-tie twins planted in samples of 1e5 .. 6e5 rows: every persistent plan the drop-in takes
    at those sizes (the two-row small-shard kernel, 256-thread blocks with LDS rows, 512-thread blocks
    with dynamic chunks) flags the construction and the default thin returns NumPy's indices."""
    X, G, steps = mr.near_tie_twins(3, n=n)
    want = o.thin(X, G, 20)
    integrand = st._make_stein_integrand(X, G)
    np.testing.assert_array_equal(st._greedy_search(20, integrand), want)
    tie = integrand.device_problem().near_tie
    assert tie is not None and 0 <= tie <= steps[0]
    idx, step, _ = _compact_run(integrand.device_problem(), 20)
    _, _, _, _, flagged = oc.greedy_ties(integrand.sample, integrand.gradient, None, integrand.linv_scale,
                                         integrand.linv_trace, 20)
    assert step == np.flatnonzero(flagged)[0]


@pytest.mark.parametrize('shape', ['exp', 'log'])
def test_lv_call_all_rows_guarded_mid_size_plan(shape):
    """The LV call's 5e5 rows without dedup (1 954 rows per block): the guarded mid-size plan (the
    compact-only kernel of 4 register rows, persistent.hip mid_guard) -- indices, flag and final guard state
    equal the bit model over 300 steps."""
    from bench import lv_call_shape
    sample, grads = lv_call_shape(500_000, 12350, shape)
    integrand = st._make_stein_integrand(sample, grads, preconditioner='med')
    idx, step, state = _compact_run(integrand.device_problem(), 300)
    midx, _, _, _, flagged, wv = oc.greedy_ties(integrand.sample, integrand.gradient, None, integrand.linv_scale,
                                                integrand.linv_trace, 300, winner_sums=True)
    np.testing.assert_array_equal(idx, midx)
    assert step == (np.flatnonzero(flagged)[0] if flagged.any() else -1)
    thr_all, Q, E = model_thresholds(integrand.gradient, None, integrand.linv_scale, integrand.linv_trace, midx, wv)
    g2, w2 = oc.tie_bounds(integrand.gradient, None)
    np.testing.assert_array_equal(state, [g2, w2, Q, E, thr_all[-1]])


@pytest.mark.parametrize('n', [60, 300, 700, 5000])
def test_kernel_state_on_few_blocks_long_runs(n):
    """One to twenty blocks and up to 300 steps: the exchange is at its fastest, so the next pick lands
    soonest after the late check of the previous step -- the check must read only step-parity state (the
    winner's index and sum, the rescans) and the inputs.  Final (Q, E, thr) bit for bit against the model."""
    X, G, _ = mr.near_tie_twins(4, n=n)
    integrand = st._make_stein_integrand(X, G)
    m = min(300, X.shape[0])
    idx, step, state = _compact_run(integrand.device_problem(), m)
    midx, _, _, _, flagged, wv = oc.greedy_ties(integrand.sample, integrand.gradient, None, integrand.linv_scale,
                                                integrand.linv_trace, m, winner_sums=True)
    np.testing.assert_array_equal(idx, midx)
    assert step == (np.flatnonzero(flagged)[0] if flagged.any() else -1)
    thr_all, Q, E = model_thresholds(integrand.gradient, None, integrand.linv_scale, integrand.linv_trace, midx, wv)
    g2, w2 = oc.tie_bounds(integrand.gradient, None)
    np.testing.assert_array_equal(state, [g2, w2, Q, E, thr_all[-1]])


@pytest.mark.parametrize('seed', range(5))
def test_dropin_thin_gf_equals_numpy_on_near_ties(seed):
    """The gradient-free operator (weights w_i w_j in every pair and in the guard's bound): the twins of the
    rows NumPy selects, with their own log densities; the default thin_gf returns NumPy's indices."""
    X, G, steps = mr.near_tie_twins(seed)
    cov = np.array([[1, .8], [.8, 1]])
    log_p = -0.5 * np.sum(X * np.linalg.solve(cov, X.T).T, axis=1)
    log_q = 0.9 * log_p   # a proxy close enough that the weights' spread stays under the warning
    want = o.thin_gf(X, log_p, log_q, G, 30)
    np.testing.assert_array_equal(stein_thinning.thin_gf(X, log_p, log_q, G, 30), want)
    integrand = st._make_stein_gf_integrand(X, log_p, log_q, G)
    np.testing.assert_array_equal(st._greedy_search(30, integrand), want)
    assert integrand.device_problem().near_tie is not None and integrand.device_problem().near_tie >= -1
    _, step, _ = _compact_run(integrand.device_problem(), 30)
    _, _, _, _, flagged = oc.greedy_ties(integrand.sample, integrand.gradient, integrand.weights,
                                         integrand.linv_scale, integrand.linv_trace, 30)
    assert step == (np.flatnonzero(flagged)[0] if flagged.any() else -1)
