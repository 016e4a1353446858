"""Host-side logic of the stein_thinning shim (no GPU): validation, standardisation, preconditioner,
log-weights, the integrand protocol loops, and that the device path refuses to run without HIP."""
import subprocess
import sys
import warnings

import numpy as np
import pytest

from oracle import models
from oracle import stein_numpy as o
from stein_thinning import kernel as sk
from stein_thinning import stein as ss
from stein_thinning import thinning as st


@pytest.fixture(scope='module')
def biv():
    return models.bivariate_reference_sample(1000)


def test_standardize_bit_identical_to_oracle(biv):
    sample, gradient, _, _, _ = biv
    s1, g1 = st._validate_and_standardize(sample, gradient, True)
    s2, g2 = o._validate_and_standardize(sample, gradient, True)
    assert np.array_equal(s1, s2) and np.array_equal(g1, g2)
    s3, g3 = st._validate_and_standardize(sample, gradient, False)
    assert np.array_equal(s3, sample) and np.array_equal(g3, gradient)


@pytest.mark.parametrize('pre', ['id', 'med', 'sclmed', 2.5, '0.5'])
def test_precon_bit_identical_to_oracle(biv, pre):
    s, _ = o._validate_and_standardize(biv[0], biv[1], True)
    assert np.array_equal(sk.make_precon(s, pre), o.make_precon(s, pre))


def test_precon_med_subsamples_large_n():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(5000, 3))
    assert np.array_equal(sk.make_precon(x, 'med'), o.make_precon(x, 'med'))


def test_precon_errors():
    x = np.ones((10, 2))
    with pytest.raises(ValueError):
        sk.make_precon(x, 'med')
    with pytest.raises(ValueError):
        sk.make_precon(x, 'bogus')


@pytest.mark.parametrize('bad', [
    (np.zeros(5), np.zeros(5)),                       # not 2-D
    (np.zeros((0, 2)), np.zeros((0, 2))),             # empty
    (np.zeros((5, 2)), np.zeros((5, 3))),             # inconsistent
    (np.array([[np.nan, 1.], [2., 3.]]), np.ones((2, 2))),
    (np.array([[np.inf, 1.], [2., 3.]]), np.ones((2, 2))),
    (np.ones((4, 2)), np.ones((4, 2))),               # zero scale
])
def test_validation_errors(bad):
    with pytest.raises(ValueError):
        st._validate_and_standardize(bad[0], bad[1], True)


def test_log_weights_warning_and_anchor():
    log_p = np.array([0., -1., -30.])
    log_q = np.array([0., 0., 0.])
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        lw = st._log_weights(log_p, log_q, None)
    assert any('log_q differs from log_p by more than 10' in str(x.message) for x in w)
    assert np.array_equal(lw, o._log_weights(log_p, log_q, None))
    assert lw.min() == 0
    assert np.array_equal(st._log_weights(log_p, log_q, 5.0), np.minimum(lw, 5.0))
    with warnings.catch_warnings():
        warnings.simplefilter('error')
        st._log_weights(np.zeros(3), np.array([0., 1., 2.]), None)


def test_protocol_greedy_with_user_integrand_matches_oracle(biv):
    sample, gradient, _, _, _ = biv
    integrand = o._make_stein_integrand(sample, gradient)    # a plain NumPy callable (user plug-in)
    np.testing.assert_array_equal(st._greedy_search(20, integrand), o._greedy_search(20, integrand))


def test_greedy_argument_errors():
    with pytest.raises(IndexError):
        st._greedy_search(0, lambda a, b: np.zeros(3))
    with pytest.raises(ValueError):
        st._greedy_search(-1, lambda a, b: np.zeros(3))


def test_reference_test_ksd_through_shim(golden):
    """code/tests/test_ksd.py verbatim semantics, run against the shim's kmat."""
    f = golden['F5_test_ksd']
    mat = np.array(f['mat'])

    def integrand(ind1, ind2):
        return mat[ind1, ind2]

    def reindex_integrand(integrand, indices):   # code/src/utils/ksd.py:9-16
        def res(ind1, ind2):
            return integrand(indices[ind1], indices[ind2])
        return res
    res = ss.kmat(reindex_integrand(integrand, np.array(f['indices'])), mat.shape[0])
    np.testing.assert_array_equal(res, f['expected'])


def test_protocol_ksd_with_user_integrand_matches_oracle(biv):
    sample, gradient, _, _, _ = biv
    integrand = o._make_stein_integrand(sample[:200], gradient[:200])
    np.testing.assert_allclose(ss.ksd(integrand, 50), o.ksd(integrand, 50), rtol=1e-12)


def test_reindex_wrappers_are_traced_without_gpu():
    """Any wrapper that reaches one SteinIntegrand -- the reference's reindex closure
    (code/src/utils/ksd.py:9-16), a renamed closure, a lambda, functools.partial, a callable
    object, the SteinIntegrand.reindex view -- yields its row map from one recorded call, with no
    GPU work; wrappers that call the integrand twice or reach two integrands are not traced."""
    import functools
    s = np.random.default_rng(0).normal(size=(20, 2))
    integ = st.SteinIntegrand(s, -s, np.identity(2))
    other = st.SteinIntegrand(s, -s, np.identity(2))
    idx = np.array([3, 1, 2, 19, 0])

    def reindex_integrand(integrand, indices):   # code/src/utils/ksd.py:9-16
        def res(ind1, ind2):
            return integrand(indices[ind1], indices[ind2])
        return res

    def make_view(f, rows):
        def my_wrapper(i, j):
            return f(rows[i], rows[j])
        return my_wrapper

    class Reindexed:
        def __init__(self, f, rows):
            self.f, self.rows = f, rows

        def __call__(self, i, j):
            return self.f(self.rows[i], self.rows[j])

    def take(rows, f, i, j):
        return f(rows[i], rows[j])

    n = idx.shape[0]
    for w in [reindex_integrand(integ, idx), make_view(integ, idx), lambda i, j: integ(idx[i], idx[j]),
              Reindexed(integ, idx), functools.partial(take, idx, integ)]:
        assert ss._inner_integrand(w) is integ
        np.testing.assert_array_equal(ss._record_rows(w, integ, n), idx)
    view = integ.reindex(idx)
    assert view.n == n and view.base() is integ
    np.testing.assert_array_equal(view.base_rows(np.arange(n)), idx)
    np.testing.assert_array_equal(integ.reindex(idx).reindex([4, 0]).base_rows([0, 1]), [0, 3])
    assert ss._record_rows(lambda i, j: integ(idx[i], idx[j]) + integ(idx[i], idx[j]), integ, n) is None
    assert ss._inner_integrand(lambda i, j: integ(i, j) - other(i, j)) is None
    assert ss._inner_integrand(lambda a, b: a) is None
    # argument-swapping wrapper: passes the reversed-arange probe with rows = idx[::-1]
    # but not the random-permutation probe, so it is not traced (the batched path evaluates it)
    assert ss._record_rows(lambda a, b: integ(idx[b], idx[a]), integ, n) is None


def test_batching_requires_an_elementwise_wrapper():
    """stein.ksd / kmat batch the reference loop's calls only for wrappers that are elementwise over
    the index arrays: a wrapper that uses ind1[0] or len(ind2) keeps the per-row loop."""
    s = np.random.default_rng(1).normal(size=(30, 2))
    ref = o._make_stein_integrand(s, -s)
    elementwise = lambda i, j: 0.5 * ref(i, j)           # noqa: E731
    by_first = lambda i, j: 0.5 * ref(np.full(len(i), i[0]), j)   # noqa: E731
    by_len = lambda i, j: ref(i, j) / len(j)              # noqa: E731
    calls = [(np.full(k + 1, k), np.arange(k + 1)) for k in range(6)]
    assert ss._elementwise(elementwise, calls)
    assert not ss._elementwise(by_first, calls)
    assert not ss._elementwise(by_len, calls)


def test_device_path_refuses_without_gpu(biv):
    import torch
    if torch.cuda.is_available():
        pytest.skip('GPU present')
    from stein_thinning import _native
    with pytest.raises(_native.HipExtensionError):
        st.thin(biv[0], biv[1], 5)


def test_import_touches_no_gpu():
    code = ('import sys; sys.path.insert(0, "gradient-free-mcmc-postprocessing_amd"); '
            'import stein_thinning, stein_thinning.thinning, stein_thinning.stein, stein_thinning.kernel; '
            'assert "torch" not in sys.modules, "torch imported at package import"')
    import os
    subprocess.run([sys.executable, '-c', code], check=True,
                   cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _numpy_standardize(sample, gradient):
    """The reference's NumPy expressions (oracle restatement, JAX_Stein_Thinning.ipynb cells 15-18)."""
    loc = np.mean(sample, axis=0)
    scl = np.mean(np.abs(sample - loc), axis=0)
    return sample / scl, gradient * scl


@pytest.mark.parametrize('n,d', [(1, 3), (7, 1), (9, 1), (129, 1), (1000, 1), (250_003, 1), (1000, 2),
                                 (100_001, 4), (3000, 50), (20, 128)])
def test_native_standardize_bitwise_numpy(n, d):
    """st_standardize_host (native, three passes) == the NumPy expressions bit for bit, for the
    row-wise (d >= 2) and the pairwise (d == 1) reduction orders."""
    rng = np.random.default_rng(n + d)
    x = rng.normal(size=(n, d)) * rng.uniform(1e-3, 1e3, size=d) + rng.normal(size=d) * 10
    if n > 1:
        x[n // 2] = x[0]
    g = rng.normal(size=(n, d))
    if n == 1:
        with pytest.raises(ValueError, match='Too few unique samples'):
            st._validate_and_standardize(x, g)
        return
    xs, gs = st._validate_and_standardize(x, g)
    wx, wg = _numpy_standardize(x, g)
    assert xs.dtype == np.float64 and xs.shape == (n, d)
    np.testing.assert_array_equal(xs.view(np.uint64), wx.view(np.uint64))
    np.testing.assert_array_equal(gs.view(np.uint64), wg.view(np.uint64))
    # inputs untouched, standardize=False returns the validated inputs
    xs2, gs2 = st._validate_and_standardize(x, g, standardize=False)
    np.testing.assert_array_equal(xs2, x)
    np.testing.assert_array_equal(gs2, g)


def test_native_standardize_errors_and_inputs():
    x = np.arange(12.0).reshape(6, 2)
    g = np.ones((6, 2))
    for bad, msg in [((np.nan, 0), 'NaNs'), ((np.inf, 0), 'infs')]:
        xb = x.copy()
        xb[2, 1] = bad[0]
        with pytest.raises(ValueError, match=msg):
            st._validate_and_standardize(xb, g)
        with pytest.raises(ValueError, match=msg):
            st._validate_and_standardize(x, np.where(xb != xb, np.nan, np.where(np.isinf(xb), np.inf, g)))
    xc = x.copy()
    xc[:, 1] = 3.0
    with pytest.raises(ValueError, match='Too few unique samples'):
        st._validate_and_standardize(xc, g)
    # Fortran-ordered / float32 / list inputs are converted like np.asarray(dtype=float64)
    xs, gs = st._validate_and_standardize(np.asfortranarray(x), g.astype(np.float32))
    wx, wg = _numpy_standardize(x, g)
    np.testing.assert_array_equal(xs, wx)
    np.testing.assert_array_equal(gs, wg)
