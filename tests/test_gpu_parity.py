"""HIP path vs the oracle (run on an MI355X: ``pytest -m gpu``).

Bar: selected indices identical to the NumPy oracle (itself pinned to the reference's golden
outputs); running sums / pair values bit-identical to the C bit model (oracle/stein_ref.c); KSD within
1e-10 relative of the NumPy oracle (north_star tolerance 1e-6).
"""
import contextlib
import warnings

import numpy as np
import pytest
from scipy.stats import multivariate_normal as mvn

from oracle import models
from oracle import stein_numpy as o
from tests import oracle_c

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import stein as ss  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402
from stein_thinning.device import DeviceProblem  # noqa: E402
from stein_thinning.distributed import HipShardBackend, shard_bounds  # noqa: E402


@contextlib.contextmanager
def arith(mode):
    """st_tune key 11 for the block: the greedy kernels' arithmetic ('compact' = the default)."""
    from stein_thinning import _native
    L = _native.lib()
    assert L.st_tune(11, {'exact': 0, 'compact': 1}[mode]) == 0
    try:
        yield
    finally:
        L.st_tune(11, -1)


def _native_loaded():
    from stein_thinning import _native
    assert _native._LIB is not None


# ------------------------------------------------------------------------------------------
# golden vectors (F1, F2, F3) through the shim
# ------------------------------------------------------------------------------------------
def test_f1_golden_indices(golden):
    sample, gradient, log_p, _, _ = models.bivariate_reference_sample(1000)
    idx = st.thin(sample, gradient, 20)
    assert idx.dtype == np.uint32
    np.testing.assert_array_equal(idx, golden['F1a_thin_bivariate_m20']['indices'])
    np.testing.assert_array_equal(st.thin_gf(sample, log_p, log_p, gradient, 20), idx)
    log_q, gq, _, _ = models.gaussian_proxy(sample, ddof=2)
    np.testing.assert_array_equal(st.thin_gf(sample, log_p, log_q, gq, 20),
                                  golden['F1c_thin_gf_simple_gaussian_ddof2']['indices'])
    _native_loaded()


@pytest.fixture(scope='module')
def gm_gpu(gm):
    sample, sample2, logpdf, score = gm
    gradient = score(sample)
    log_p = logpdf(sample)
    log_q, gq, _, _ = models.gaussian_proxy(sample, ddof=1)
    return dict(sample=sample, gradient=gradient, log_p=log_p, log_q=log_q, gq=gq,
                idx_st=st.thin(sample, gradient, 1000, preconditioner='med'),
                idx_gf=st.thin_gf(sample, log_p, log_q, gq, 1000, preconditioner='med'))


def test_f2_gaussian_mixture_1000_steps(gm_gpu, golden):
    f = golden['F2_gaussian_mixture']
    s = gm_gpu
    np.testing.assert_array_equal(s['idx_st'], o.thin(s['sample'], s['gradient'], 1000, preconditioner='med'))
    np.testing.assert_array_equal(
        s['idx_gf'], o.thin_gf(s['sample'], s['log_p'], s['log_q'], s['gq'], 1000, preconditioner='med'))
    assert len(np.unique(s['idx_st'])) == f['unique_counts']['stein']
    assert len(np.unique(s['idx_gf'])) == f['unique_counts']['gf_simple_gaussian']


def test_f2_laplace_collapse(gm, golden):
    sample, _, logpdf, _ = gm
    f = golden['F2_gaussian_mixture']
    lm, lc = np.array(f['laplace_mean']), np.array(f['laplace_cov'])
    log_p = logpdf(sample)
    log_q = mvn.logpdf(sample, mean=lm, cov=lc)
    gq = -np.einsum('ij,kj->ki', np.linalg.inv(lc), sample - lm)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        idx = st.thin_gf(sample, log_p, log_q, gq, 10_000, preconditioner='med')
    assert any('log_q differs from log_p by more than 10' in str(x.message) for x in w)
    assert idx.shape == (10_000,) and set(np.unique(idx).tolist()) == {f['laplace_all_selected']}


def test_f3_ksd_curves_on_gpu(gm_gpu, curves):
    """calculate_ksd (code/src/utils/ksd.py:19-27) through the shim: the reindexed closure runs on
    the tiled HIP KSD kernel; compare with the oracle and with the report's figure."""
    def reindex_integrand(integrand, indices):
        def res(ind1, ind2):
            return integrand(indices[ind1], indices[ind2])
        return res

    for name, idx in [('stein', gm_gpu['idx_st']), ('gf_simple_gaussian', gm_gpu['idx_gf'])]:
        integrand = st._make_stein_integrand(gm_gpu['sample'], gm_gpu['gradient'])
        ks = ss.ksd(reindex_integrand(integrand, idx), idx.shape[0])
        want = o.calculate_ksd(gm_gpu['sample'], gm_gpu['gradient'], idx)
        np.testing.assert_allclose(ks, want, rtol=1e-10)
        c = np.array(curves['ksd/' + name])
        np.testing.assert_allclose(ks[c[:, 0].astype(int) - 1], c[:, 1], rtol=1e-7)


def test_f4_kmat_on_gpu(gm, golden):
    sample, _, _, _ = gm
    f = golden['F2_gaussian_mixture']
    lm, lc = np.array(f['laplace_mean']), np.array(f['laplace_cov'])
    gq = -np.einsum('ij,kj->ki', np.linalg.inv(lc), sample - lm)
    km = ss.kmat(st._make_stein_integrand(sample, gq), sample.shape[0])
    want = o.kmat(o._make_stein_integrand(sample, gq), sample.shape[0])
    np.testing.assert_allclose(km, want, rtol=1e-13, atol=1e-13 * np.abs(want).max())
    assert np.array_equal(km, km.T)
    assert np.abs(km[np.triu_indices_from(km)]).max() == pytest.approx(f['kmat_laplace_abs_max'], rel=1e-7)


# ------------------------------------------------------------------------------------------
# bit-exactness against the C bit model
# ------------------------------------------------------------------------------------------
def _rw_chain(n, d, seed, dup_every=3):
    """Seeded synthetic chain with many duplicated rows (RW-MH style rejections)."""
    rng = np.random.default_rng(seed)
    x = np.cumsum(rng.normal(scale=0.3, size=(n, d)), axis=0) * 0.05 + rng.normal(size=(n, d))
    rep = rng.random(n) < (1 - 1 / dup_every)
    for i in range(1, n):
        if rep[i]:
            x[i] = x[i - 1]
    g = -x * np.linspace(0.5, 2.0, d)
    return x, g


@pytest.mark.parametrize('mode', ['compact', 'exact'])
@pytest.mark.parametrize('d', [1, 2, 3, 4, 5, 7, 8, 9, 16, 50])
@pytest.mark.parametrize('gf', [False, True])
def test_running_sums_bit_exact_vs_c_model(d, gf, mode):
    n, m = 4099, 25      # odd n: exercises the padded lane pair
    x, g = _rw_chain(n, d, seed=d)
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    w = None
    if gf:
        lw = -0.1 * np.sum(x * x, axis=1)
        w = np.exp(lw - lw.min())
    prob = DeviceProblem(s, gs, w, l, tr)
    with arith(mode):
        idx, A = prob.greedy(m, return_sums=True)
    cidx, cA = oracle_c.greedy(s, gs, w, l, tr, m, arith=mode)
    np.testing.assert_array_equal(idx, cidx)
    assert np.array_equal(A, cA), np.flatnonzero(A != cA)[:10]


@pytest.mark.parametrize('tune', [
    ('persistent: registers + LDS + streamed rows', 4, 1_000_003, 4),
    ('persistent: registers only', 4, 30_011, 4),
    ('persistent: d=2 gradient-free', -1, 200_003, 2),
    ('launch-per-step path', 0, 300_007, 4),
])
def test_persistent_and_fallback_bit_exact(tune):
    """st_greedy's two implementations (persistent on-chip kernel / one launch per step) against
    the C model: identical indices and bit-identical running sums."""
    from stein_thinning import _native
    _, rt, n, d = tune
    m = 30
    x, g = _rw_chain(n, d, seed=n % 97)
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    w = None
    if d == 2:
        lw = -0.2 * np.sum(x * x, axis=1)
        w = np.exp(lw - lw.min())
    _native.lib().st_tune(3, rt)
    try:
        idx, A = DeviceProblem(s, gs, w, l, tr).greedy(m, return_sums=True)
    finally:
        _native.lib().st_tune(3, -1)
    cidx, cA = oracle_c.greedy(s, gs, w, l, tr, m)
    np.testing.assert_array_equal(idx, cidx)
    assert np.array_equal(A, cA), np.flatnonzero(A != cA)[:10]


@pytest.mark.parametrize('knobs', [
    ('512-thread blocks, 8 register rows', {4: 512, 3: 8}),
    ('512-thread blocks, 4 register rows', {4: 512, 3: 4}),
    ('256-thread blocks (one wave per SIMD), LDS and streamed rows', {4: 256}),
    ('512-thread blocks, packed 16-B records', {4: 512, 9: 16}),
    ('one record array, 256-B pitch (no replicas)', {10: 1}),
    ('4 record replicas', {10: 4}),
    ('32 record replicas, 64-B pitch', {10: 32, 9: 64}),
])
@pytest.mark.parametrize('d,gf', [(4, False), (2, True)])
def test_persistent_two_wave_variants_bit_exact(knobs, d, gf):
    """The persistent plans forced through st_tune (keys 3, 4: threads per block and register rows) and the
    record layouts (keys 9, 10) against the C model: identical indices, bit-identical running sums."""
    from stein_thinning import _native
    n, m = 700_001, 20
    x, g = _rw_chain(n, d, seed=11 + d)
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    w = None
    if gf:
        lw = -0.2 * np.sum(x * x, axis=1)
        w = np.exp(lw - lw.min())
    L = _native.lib()
    for k, v in knobs[1].items():
        assert L.st_tune(k, v) == 0
    try:
        idx, A = DeviceProblem(s, gs, w, l, tr).greedy(m, return_sums=True)
    finally:
        for k in (3, 4, 8, 9, 10):
            L.st_tune(k, -1)
    cidx, cA = oracle_c.greedy(s, gs, w, l, tr, m)
    np.testing.assert_array_equal(idx, cidx)
    assert np.array_equal(A, cA), np.flatnonzero(A != cA)[:10]


@pytest.mark.parametrize('gf', [False, True])
@pytest.mark.parametrize('n', [60_001, 3_001])
def test_wide_persistent_d50_bit_exact(n, gf):
    """d = 50 shards of at most 256 rows per CU run the wide persistent kernel (x rows in
    registers, g rows in LDS): indices and running sums against the C model, and against the
    launch-per-step path (st_tune key 3 = 0)."""
    from stein_thinning import _native
    d, m = 50, 25
    x, g = _rw_chain(n, d, seed=50 + n % 7)
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    w = None
    if gf:
        lw = -0.02 * np.sum(x * x, axis=1)
        w = np.exp(lw - lw.min())
    prob = DeviceProblem(s, gs, w, l, tr)
    idx, A = prob.greedy(m, return_sums=True)
    cidx, cA = oracle_c.greedy(s, gs, w, l, tr, m)
    np.testing.assert_array_equal(idx, cidx)
    assert np.array_equal(A, cA), np.flatnonzero(A != cA)[:10]
    _native.lib().st_tune(3, 0)
    try:
        sidx, sA = prob.greedy(m, return_sums=True)
    finally:
        _native.lib().st_tune(3, -1)
    np.testing.assert_array_equal(sidx, idx)
    assert np.array_equal(sA, A)


@pytest.mark.parametrize('mode', ['compact', 'exact'])
@pytest.mark.parametrize('steps', [False, True])
@pytest.mark.parametrize('d,gf', [(4, False), (2, True)])
def test_persistent_exact_path_outside_fast_range(d, gf, steps, mode):
    """Rows with components outside [2^-60, 2^60] (tiny / huge scores, tiny coordinates) force the
    persistent kernel's general arithmetic for their blocks and for steps whose selected row is
    out of range (csrc/stein_math.hpp fast_range_ok) -- with the compact arithmetic, the per-pair
    rule (compact iff both rows in range: the mixed sweep); results stay bit-identical to the C
    model, on the persistent kernel and on the launch-per-step kernels (steps)."""
    n, m = 200_003, 40
    x, g = _rw_chain(n, d, seed=7 + d)
    s, gs = o._validate_and_standardize(x, g, True)
    rng = np.random.default_rng(d)
    rows = rng.choice(n, size=12, replace=False)
    gs = gs.copy()
    s = s.copy()
    gs[rows[:4], 0] = 1e-25          # tiny score component: small diagonal -> selected early
    gs[rows[4:6], :] = 3e-22
    gs[rows[6:8], -1] = 2e19         # huge component
    s[rows[8:10], 0] = 1e-30         # tiny coordinate
    gs[rows[10:], :] = 0.0           # exact zeros are inside the fast range
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    w = None
    if gf:
        lw = -0.2 * np.sum(x * x, axis=1)
        w = np.exp(lw - lw.min())
    from stein_thinning import _native
    if steps:
        _native.lib().st_tune(3, 0)
    try:
        with arith(mode):
            idx, A = DeviceProblem(s, gs, w, l, tr).greedy(m, return_sums=True)
    finally:
        _native.lib().st_tune(3, -1)
    cidx, cA = oracle_c.greedy(s, gs, w, l, tr, m, arith=mode)
    np.testing.assert_array_equal(idx, cidx)
    assert np.array_equal(A, cA), np.flatnonzero(A != cA)[:10]
    if not gf:   # Langevin: the tiny-score rows have the smallest diagonal and are selected
        assert np.intersect1d(idx, rows[:6]).size > 0


@pytest.mark.parametrize('case', ['in_range', 'tiny_rows_one_block', 'tiny_scores_selected', 'gf_inf_weights'])
def test_compact_only_kernel_and_handoff(case):
    """n = 1.1e6 rows (more than 8 register rows' worth per 512-thread block): the one-device
    compact-only persistent kernel (st_tune key 12) runs the thin; when a step needs the exact
    arithmetic -- rows out of [2^-60, 2^60] in one block, an out-of-range row selected, NaN sums
    from infinite gradient-free weights -- it hands the whole thin to the general kernel enqueued
    behind it.  Indices and running sums bit-identical to the C model and to the general kernel
    alone (key 12 = 0), whichever kernel finished the run."""
    from stein_thinning import _native
    n, m, d = 1_100_003, 30, 4
    x, g = _rw_chain(n, d, seed=31)
    s, gs = o._validate_and_standardize(x, g, True)
    s, gs = s.copy(), gs.copy()
    w = None
    if case == 'tiny_rows_one_block':
        s[500_000:500_010, 1] = 1e-30          # ten rows of one block, never near the minimum
    elif case == 'tiny_scores_selected':
        gs[[7, 800_001], :] = 3e-22            # smallest diagonals: selected at once
    elif case == 'gf_inf_weights':
        lw = -0.2 * np.sum(x * x, axis=1)
        lw[[123, 900_000]] = 900.0             # exp overflows: inf weights -> NaN running sums
        with np.errstate(over='ignore'):
            w = np.exp(lw - lw.min())
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    prob = DeviceProblem(s, gs, w, l, tr)
    idx, A = prob.greedy(m, return_sums=True)
    cidx, cA = oracle_c.greedy_mt(s, gs, w, l, tr, m)
    np.testing.assert_array_equal(idx, cidx)
    assert np.array_equal(A, cA, equal_nan=True), np.flatnonzero(~((A == cA) | (np.isnan(A) & np.isnan(cA))))[:10]
    L = _native.lib()
    assert L.st_tune(12, 0) == 0
    try:
        gidx, gA = prob.greedy(m, return_sums=True)
    finally:
        L.st_tune(12, -1)
    np.testing.assert_array_equal(gidx, idx)
    assert np.array_equal(gA, A, equal_nan=True)


@pytest.mark.parametrize('case', ['in_range', 'tiny_rows_one_block'])
def test_streamed_sums_in_lds_option(case):
    """st_tune key 15 = 1 keeps the streamed rows' running sums in LDS (measured slower, off by
    default): with the grid capped at 128 blocks, n = 1.1e6 leaves ~1 700 streamed rows per block;
    the compact-only kernel (and, after a handoff, the general one) give the C model's indices and
    running sums bit for bit either way."""
    from stein_thinning import _native
    n, m, d = 1_100_003, 30, 4
    x, g = _rw_chain(n, d, seed=37)
    s, gs = o._validate_and_standardize(x, g, True)
    s, gs = s.copy(), gs.copy()
    if case == 'tiny_rows_one_block':
        s[500_000:500_010, 1] = 1e-30
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    prob = DeviceProblem(s, gs, None, l, tr)
    cidx, cA = oracle_c.greedy_mt(s, gs, None, l, tr, m)
    L = _native.lib()
    assert L.st_tune(5, 128) == 0
    try:
        for sal in (0, 1):
            assert L.st_tune(15, sal) == 0
            idx, A = prob.greedy(m, return_sums=True)
            np.testing.assert_array_equal(idx, cidx)
            assert np.array_equal(A, cA), (sal, np.flatnonzero(A != cA)[:10])
    finally:
        L.st_tune(15, -1)
        L.st_tune(5, -1)


@pytest.mark.parametrize('case', ['in_range', 'tiny_rows_one_block'])
def test_streamed_sums_in_lds_guarded(case):
    """Under the near-tie guard the streamed rows' sums live in LDS by default (st_tune key 15 = -1: the
    rescans read them every step): the same streamed-row setup as above, guarded, with the key at -1 / 0 --
    no step flagged, the C model's indices and running sums bit for bit."""
    from stein_thinning import _native
    n, m, d = 1_100_003, 30, 4
    x, g = _rw_chain(n, d, seed=37)
    s, gs = o._validate_and_standardize(x, g, True)
    s, gs = s.copy(), gs.copy()
    if case == 'tiny_rows_one_block':
        s[500_000:500_010, 1] = 1e-30
    linv = o.make_precon(s, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    prob = DeviceProblem(s, gs, None, l, tr)
    cidx, cA = oracle_c.greedy_mt(s, gs, None, l, tr, m)
    L = _native.lib()
    assert L.st_tune(5, 128) == 0
    try:
        for sal in (-1, 0):
            assert L.st_tune(15, sal) == 0
            idx, A = prob.greedy(m, return_sums=True, guard=True)
            assert prob.near_tie == -1, (sal, prob.near_tie)
            np.testing.assert_array_equal(idx, cidx)
            assert np.array_equal(A, cA), (sal, np.flatnonzero(A != cA)[:10])
    finally:
        L.st_tune(15, -1)
        L.st_tune(5, -1)


@pytest.mark.parametrize('d', [2, 4, 9, 50])
def test_pair_values_bit_exact_vs_c_model(d):
    x, g = _rw_chain(700, d, seed=100 + d)
    s, gs = o._validate_and_standardize(x, g, True)
    rng = np.random.default_rng(d)
    lw = rng.normal(size=700)
    w = np.exp(lw - lw.min())          # min-anchored, as thin_gf builds its weights
    integ = st.SteinIntegrand(s, gs, o.make_precon(s, 'med'), w)
    i1 = rng.integers(0, 700, size=5000)
    i2 = rng.integers(0, 700, size=5000)
    got = integ(i1, i2)
    # the integrand protocol (vfk0_imq values) keeps the exact arithmetic
    want = oracle_c.pairs(s, gs, w, integ.linv_scale, integ.linv_trace, i1, i2, arith='exact')
    assert np.array_equal(got, want)
    # integrand protocol forms used by the reference: (slice, slice), (slice, [j])
    np.testing.assert_array_equal(integ(slice(None), [5]), oracle_c.pairs(
        s, gs, w, integ.linv_scale, integ.linv_trace, np.arange(700), np.full(700, 5), arith='exact'))
    # and against the NumPy oracle integrand (different pow rounding: <= 1e-15 relative)
    ref = o._make_stein_gf_integrand(x, np.zeros(700), lw, g, preconditioner='med')
    np.testing.assert_allclose(integ(slice(None), slice(None)), ref(slice(None), slice(None)), rtol=1e-14)


def test_vfk0_imq_on_gpu():
    from stein_thinning import kernel as sk
    x, g = _rw_chain(300, 4, seed=5)
    linv = o.make_precon(x, 'med')
    np.testing.assert_allclose(sk.vfk0_imq(x, x[[7]], g, g[[7]], linv), o.vfk0_imq(x, x[[7]], g, g[[7]], linv),
                               rtol=1e-14)
    np.testing.assert_allclose(sk.vfk0_imq(x, x, g, g, linv), o.vfk0_imq(x, x, g, g, linv), rtol=1e-15)


# ------------------------------------------------------------------------------------------
# edge cases the reference allows
# ------------------------------------------------------------------------------------------
def test_single_row_and_m_greater_than_n():
    x = np.array([[0.3, -1.2]])
    g = -x
    np.testing.assert_array_equal(st.thin(x, g, 5, standardize=False), np.zeros(5, dtype=np.uint32))
    x, g = _rw_chain(7, 2, seed=1, dup_every=1)
    np.testing.assert_array_equal(st.thin(x, g, 30), o.thin(x, g, 30))


def test_overflowing_weights_nan_semantics():
    """exp overflow -> inf/NaN running sums: np.argmin picks the first NaN; the kernel must too."""
    x, g = _rw_chain(600, 3, seed=9, dup_every=1)
    log_p = np.zeros(600)
    log_q = np.linspace(0, 900, 600)       # exp(900) = inf
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        want = o.thin_gf(x, log_p, log_q, g, 12)
        got = st.thin_gf(x, log_p, log_q, g, 12)
    np.testing.assert_array_equal(got, want)


def test_range_cap_matches_oracle():
    x, g = _rw_chain(2000, 4, seed=3)
    log_p = -0.5 * np.sum(x * x, axis=1) * 40
    log_q = -0.5 * np.sum(x * x, axis=1)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        np.testing.assert_array_equal(st.thin_gf(x, log_p, log_q, g, 50, range_cap=20, preconditioner='med'),
                                      o.thin_gf(x, log_p, log_q, g, 50, range_cap=20, preconditioner='med'))


# ------------------------------------------------------------------------------------------
# BASELINE configs (sizes the oracle finishes in seconds) and full-size properties
# ------------------------------------------------------------------------------------------
def _lv_surrogate(n, seed):
    from bench import lv_surrogate
    return lv_surrogate(n, seed)


def test_config2_langevin_n2e5_m100():
    x, g, _, _ = _lv_surrogate(200_000, 12347)
    np.testing.assert_array_equal(st.thin(x, g, 100, preconditioner='med'),
                                  o.thin(x, g, 100, preconditioner='med'))


def test_config3_gradient_free_n2e5_m100():
    x, g, log_p, log_q_gq = _lv_surrogate(200_000, 12348)
    log_q, gq = log_q_gq
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        np.testing.assert_array_equal(st.thin_gf(x, log_p, log_q, gq, 100, preconditioner='med'),
                                      o.thin_gf(x, log_p, log_q, gq, 100, preconditioner='med'))


def test_config5_d50_prefix():
    from bench import gaussian_d50
    x, log_p, log_q, gq = gaussian_d50(50_000, 12349)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        np.testing.assert_array_equal(st.thin_gf(x, log_p, log_q, gq, 40, preconditioner='med'),
                                      o.thin_gf(x, log_p, log_q, gq, 40, preconditioner='med'))


def _oracle_inputs(x, g, log_p=None, log_q=None):
    """The C bit model's inputs built by the NumPy oracle's own host steps (standardisation, 'med'
    preconditioner, min-anchored weights: oracle/stein_numpy.py)."""
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    w = None if log_p is None else np.exp(o._log_weights(log_p, log_q, None))
    return s, gs, w, float(linv[0, 0]), float(np.trace(linv))


def test_config4_full_length_bit_exact(config4):
    """The headline workload, every step: all 1000 indices identical to the C bit model and the
    final running sums bit-identical on all 2e6 rows; the bit model's first 20 indices identical to
    the NumPy restatement of JAX_Stein_Thinning.ipynb:281-295 on the same input; the drop-in
    thin() on host arrays returns the same indices."""
    c = config4
    np.testing.assert_array_equal(c['idx'][:20], o.thin(c['x'], c['g'], 20, preconditioner='med'))
    prob = DeviceProblem(c['s'], c['gs'], None, c['l'], c['tr'])
    idx, A = prob.greedy(c['m'], return_sums=True)
    np.testing.assert_array_equal(idx, c['idx'])
    assert np.array_equal(A, c['A']), np.flatnonzero(A != c['A'])[:10]
    # the repeated-row path (the drop-in thin's default): 24 % of the rows start a run
    didx, dA = prob.greedy(c['m'], return_sums=True, dedup=True)
    assert prob.dedup_used and prob.dedup_view().n_unique < 0.3 * prob.n
    np.testing.assert_array_equal(didx, c['idx'])
    assert np.array_equal(dA, c['A']), np.flatnonzero(dA != c['A'])[:10]
    np.testing.assert_array_equal(st.thin(c['x'], c['g'], c['m'], preconditioner='med'), c['idx'])


def test_config5_full_length_bit_exact():
    """BASELINE config 5 at full size (n = 5e5, d = 50, gradient-free, m = 500 -- the launch-per-step
    greedy_step_rt kernel on one GPU): all 500 indices identical to the C bit model, running sums
    bit-identical; the bit model's first 5 indices identical to the NumPy restatement."""
    from bench import gaussian_d50
    m = 500
    x, log_p, log_q, gq = gaussian_d50(500_000, 12349)
    s, gs, w, l, tr = _oracle_inputs(x, gq, log_p, log_q)
    cidx, cA = oracle_c.greedy_mt(s, gs, w, l, tr, m)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        np.testing.assert_array_equal(cidx[:5], o.thin_gf(x, log_p, log_q, gq, 5, preconditioner='med'))
        integ = st._make_stein_gf_integrand(x, log_p, log_q, gq, preconditioner='med')
    idx, A = integ.device_problem().greedy(m, return_sums=True)
    np.testing.assert_array_equal(idx, cidx)
    assert np.array_equal(A, cA), np.flatnonzero(A != cA)[:10]
    np.testing.assert_array_equal(st._greedy_search(m, integ), cidx)


def test_two_shards_on_one_gpu_equal_single():
    """HipShardBackend with nranks = 2 in one process (records exchanged by torch.cat in place of
    RCCL) reproduces the single-device indices, including ties across the shard boundary."""
    x, g = _rw_chain(30_001, 4, seed=21)
    x[20_000:20_500] = x[1_000:1_500]
    g[20_000:20_500] = g[1_000:1_500]
    m = 60
    integ = st._make_stein_integrand(x, g, preconditioner='med')
    want = integ.device_problem().greedy(m)
    bes = [HipShardBackend(integ, *shard_bounds(integ.n, r, 2), 2, m) for r in range(2)]
    for t in range(m):
        for be in bes:
            be.step(t)
        allrec = torch.cat([be.send for be in bes])
        for be in bes:
            be.recv.copy_(allrec)
    for be in bes:
        be.finalize(m - 1)
        np.testing.assert_array_equal(be.indices(), want)
    np.testing.assert_array_equal(want, o.thin(x, g, m, preconditioner='med'))


def test_ksd_kmat_wrappers_run_one_device_launch(gm_gpu, monkeypatch):
    """stein.ksd / kmat on wrappers of a SteinIntegrand under any name (closure, lambda, callable
    object, functools.partial, the reindex view): ONE tiled-KSD / kmat launch and no pair-kernel
    launch, values as calculate_ksd's (code/src/utils/ksd.py:19-27);
    a wrapper with arithmetic of its own runs the batched protocol (no per-row launches)."""
    import functools
    from stein_thinning.device import DeviceProblem
    calls = {'ksd': 0, 'kmat': 0, 'pairs': 0}
    for name in calls:
        orig = getattr(DeviceProblem, name)

        def counted(self, *a, _orig=orig, _name=name, **k):
            calls[_name] += 1
            return _orig(self, *a, **k)
        monkeypatch.setattr(DeviceProblem, name, counted)
    idx = gm_gpu['idx_st']
    integ = st._make_stein_integrand(gm_gpu['sample'], gm_gpu['gradient'])
    want = o.calculate_ksd(gm_gpu['sample'], gm_gpu['gradient'], idx)

    class Reindexed:
        def __init__(self, f, rows):
            self.f, self.rows = f, rows

        def __call__(self, i, j):
            return self.f(self.rows[i], self.rows[j])

    def take(rows, f, i, j):
        return f(rows[i], rows[j])
    m = idx.shape[0]
    for w in [lambda i, j: integ(idx[i], idx[j]), Reindexed(integ, idx), functools.partial(take, idx, integ),
              integ.reindex(idx)]:
        for k in calls:
            calls[k] = 0
        ks = ss.ksd(w, m)
        np.testing.assert_allclose(ks, want, rtol=1e-10)
        assert calls['ksd'] == 1 and calls['pairs'] == 0, calls
    for k in calls:
        calls[k] = 0
    km = ss.kmat(Reindexed(integ, idx[:300]), 300)
    assert calls['kmat'] == 1 and calls['pairs'] == 0, calls
    np.testing.assert_array_equal(km, ss.kmat(integ.reindex(idx[:300]), 300))
    # a wrapper doing its own arithmetic: the batched protocol, values as the reference loop's
    for k in calls:
        calls[k] = 0
    scaled = ss.ksd(lambda i, j: 0.5 * integ(idx[i], idx[j]), 200)
    # the elementwise check (ss._ELEMENTWISE_PREFIX separate calls + one batched) and ONE batch
    assert calls['ksd'] == 0 and calls['pairs'] == ss._ELEMENTWISE_PREFIX + 2, calls
    ref_int = o._make_stein_integrand(gm_gpu['sample'], gm_gpu['gradient'])
    np.testing.assert_allclose(scaled, o.ksd(lambda i, j: 0.5 * ref_int(idx[i], idx[j]), 200), rtol=1e-12)
    # an argument-swapping wrapper is not a re-indexing of the same rows: evaluated as written
    for k in calls:
        calls[k] = 0
    swapped = ss.ksd(lambda i, j: integ(idx[j], idx[i]), 200)
    assert calls['ksd'] == 0, calls
    np.testing.assert_allclose(swapped, o.ksd(lambda i, j: ref_int(idx[j], idx[i]), 200), rtol=1e-12)
