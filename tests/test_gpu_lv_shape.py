"""The reference's own Lotka-Volterra thinning call at its own size (VERDICT r03 missing #1):
``thin(np.exp(rw_samples[i]), rw_grads[i], n_points_calculate, preconditioner='med')`` and the log-space
variant ``thin(rw_samples[i], np.exp(rw_samples[i]) * rw_grads[i], ...)``
(``code/notebooks/lotka_volterra/Stein_thinning.ipynb`` cells 12 and 14, json :204 / :264), with
``n_points_calculate = 10_000`` (cell 11, :188) on one RW-MH chain of 5e5 points (Sampling.ipynb cells
16-18).  The chains live in the reference's S3 bucket, so the input is the seeded LV surrogate chain of
bench.lv_call_shape (the same RW-MH generator as configs 2-4, one chain of 5e5).

Bar: all 10 000 indices of the drop-in ``thin`` equal the threaded C bit model (oracle/stein_ref.c, the
kernels' arithmetic), and the first 50 equal the NumPy restatement of the reference loop
(oracle/stein_numpy.py; the greedy selection is prefix-consistent, so a 50-step run is the first 50
steps of the 10 000-step one).  10 000 steps wrap the persistent kernel's 8-bit step tags 39 times.
"""
import numpy as np
import pytest

from oracle import stein_numpy as o
from tests import oracle_c

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import _native as nat  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402

N, M = 500_000, 10_000


@pytest.mark.parametrize('shape', ['exp', 'log'])
def test_lv_call_shape_10000_points(shape):
    from bench import lv_call_shape
    sample, grads = lv_call_shape(N, 12350, shape)
    assert M // 256 >= 39    # the step tags (8 bits) wrap this many times in one run
    idx = st.thin(sample, grads, M, preconditioner='med')
    assert idx.dtype == np.uint32 and idx.shape == (M,)
    integrand = st._make_stein_integrand(sample, grads, preconditioner='med')
    want, _ = oracle_c.greedy_mt(integrand.sample, integrand.gradient, None, integrand.linv_scale,
                                 integrand.linv_trace, M, arith=nat.arithmetic())
    bad = np.flatnonzero(idx != want)
    assert bad.size == 0, f'{bad.size} of {M} indices differ from the C bit model; first at step {bad[0]}'
    np.testing.assert_array_equal(idx[:50], o.thin(sample, grads, 50, preconditioner='med'))


def test_lv_gaussian_thin_call_shape_10000_points():
    """The gradient-free LV call (``Gradient_free.ipynb`` cell 37, json :875-881): per chain
    ``gaussian_thin(sample, log_p, np.mean(sample, 0), np.cov(sample, rowvar=False, ddof=d), 10_000)``
    -- code/src/thinning.py:14-17, i.e. thin_gf with the Gaussian proxy, range_cap=200 and 'med' -- on
    the 5e5-row log-space surrogate chain.  The GPU's proxy (log q, grad log q) feeds both sides: all
    10 000 indices equal the C bit model on the same weights, and the first 50 equal the scipy-fed
    NumPy oracle of the whole call (oracle/proxy_numpy.py)."""
    import warnings
    from bench import lv_surrogate
    from oracle import proxy_numpy as op
    from stein_thinning import proxy
    s, _, log_p, _ = lv_surrogate(N, 12350, chain_len=N)
    mean = np.mean(s, axis=0)
    cov = np.cov(s, rowvar=False, ddof=s.shape[1])
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        idx = proxy.gaussian_thin(s, log_p, mean, cov, M)
        log_q, gq = proxy.gaussian_proxy(s, mean, cov)
        integrand = st._make_stein_gf_integrand(s, log_p, log_q, gq, range_cap=200, preconditioner='med')
        head = op.gaussian_thin(s, log_p, mean, cov, 50)
    want, _ = oracle_c.greedy_mt(integrand.sample, integrand.gradient, integrand.weights, integrand.linv_scale,
                                 integrand.linv_trace, M, arith=nat.arithmetic())
    bad = np.flatnonzero(idx != want)
    assert bad.size == 0, f'{bad.size} of {M} indices differ from the C bit model; first at step {bad[0]}'
    np.testing.assert_array_equal(idx[:50], head)
