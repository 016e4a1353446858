"""Proxy producers on the GPU (csrc/proxy.hip via st_proxy_logpdf_grad) against the reference's
scipy computations (oracle/proxy_numpy.py): log q and grad log q to fp64 rounding (relative 1e-12;
the per-row dot products are summed in a different order than BLAS), and the downstream selections
of gaussian_thin / thin_gf_t identical to the reference's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from oracle import proxy_numpy as op  # noqa: E402
from oracle.models import gm_reference_sample  # noqa: E402
from stein_thinning import proxy  # noqa: E402

RTOL = 1e-12


def _close(got, want):
    scale = max(float(np.abs(want).max()), 1.0) if want.size else 1.0
    np.testing.assert_allclose(got, want, rtol=RTOL, atol=RTOL * scale)


def _case(n, d, seed):
    rng = np.random.default_rng(seed)
    a = rng.normal(size=(d, d))
    cov = a @ a.T / d + 0.3 * np.eye(d)
    mean = rng.normal(size=d)
    x = mean + rng.normal(size=(n, d)) @ np.linalg.cholesky(cov).T * 1.5
    return x, mean, cov


@pytest.mark.parametrize('d', [1, 2, 3, 4, 7, 8, 16, 17, 32, 33, 50, 64, 65, 128])
@pytest.mark.parametrize('n', [1, 63, 64, 65, 5000])
def test_gaussian_proxy_matches_scipy(n, d):
    x, mean, cov = _case(n, d, 10 * d + n)
    lq, gq = proxy.gaussian_proxy(x, mean, cov)
    wl, wg = op.gaussian_proxy(x, mean, cov)
    assert lq.shape == (n,) and gq.shape == (n, d)
    _close(lq, np.atleast_1d(wl))
    _close(gq, wg)


@pytest.mark.parametrize('d', [1, 2, 4, 9, 20, 50, 64, 128])
@pytest.mark.parametrize('df', [1.0, 3.0, 4.0, 30.5])
def test_student_t_proxy_matches_scipy_and_notebook_gradient(d, df):
    x, loc, shape = _case(777, d, d + int(df * 10))
    lq, gq = proxy.student_t_proxy(x, loc, shape * 3, df)
    wl, wg = op.student_t_proxy(x, loc, shape * 3, df)
    _close(lq, wl)
    _close(gq, wg)


def test_empty_sample():
    lq, gq = proxy.gaussian_proxy(np.zeros((0, 3)), np.zeros(3), np.eye(3))
    assert lq.shape == (0,) and gq.shape == (0, 3)


def test_gaussian_thin_selects_the_reference_points_gm():
    sample, _, logpdf, _ = gm_reference_sample()
    log_p = logpdf(sample)
    mean = np.mean(sample, axis=0)
    cov = np.cov(sample, rowvar=False, ddof=2)
    got = proxy.gaussian_thin(sample, log_p, mean, cov, 40)
    want = op.gaussian_thin(sample, log_p, mean, cov, 40)
    np.testing.assert_array_equal(got, want)


def test_thin_gf_t_selects_the_reference_points_gm():
    sample, _, logpdf, _ = gm_reference_sample()
    log_p = logpdf(sample)
    cov = np.cov(sample, rowvar=False, ddof=2)
    mode = sample[np.argmax(log_p)]
    got = proxy.thin_gf_t(sample, log_p, mode, cov * 3, 4, 100)
    want = op.thin_gf_t(sample, log_p, mode, cov * 3, 4, 100)
    np.testing.assert_array_equal(got, want)


def test_gaussian_thin_selects_the_reference_points_d50():
    rng = np.random.default_rng(12349)
    d, n = 50, 4000
    idx = np.arange(d)
    cov = 0.5 ** np.abs(idx[:, None] - idx[None, :])
    x = rng.normal(size=(n, d)) @ np.linalg.cholesky(cov).T
    log_p = -0.5 * np.einsum('ij,jk,ik->i', x, np.linalg.inv(cov), x)
    mean = x.mean(axis=0)
    qcov = 1.2 * np.cov(x, rowvar=False)
    got = proxy.gaussian_thin(x, log_p, mean, qcov, 60)
    want = op.gaussian_thin(x, log_p, mean, qcov, 60)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize('d', [17, 50, 64])
def test_valu_and_matrix_core_kernels_agree(d):
    """The VALU kernel (st_tune key 7 = 1) on the d range the MFMA kernel serves by default."""
    from stein_thinning import _native as nat
    x, mean, cov = _case(3000, d, 99 + d)
    wl, wg = op.gaussian_proxy(x, mean, cov)
    lm, gm = proxy.gaussian_proxy(x, mean, cov)
    assert nat.lib().st_tune(7, 1) == 0
    try:
        lv_, gv = proxy.gaussian_proxy(x, mean, cov)
    finally:
        nat.lib().st_tune(7, 0)
    for lq, gq in ((lm, gm), (lv_, gv)):
        _close(lq, wl)
        _close(gq, wg)


@pytest.mark.parametrize('mode', [2, 3, 4])
@pytest.mark.parametrize('d', [17, 18, 24, 25, 31, 40, 47, 49, 50, 57, 63, 64])
def test_matrix_core_variants_match_scipy(mode, d):
    """Every matrix-core variant (st_tune key 7: 2 LDS-tiled, 3 guarded streaming form -- the odd-d
    default --, 4 buffer-instruction form -- the even-d default; odd d falls back to 3) over each
    (T, S) instantiation; n not a multiple of 16; both proxies."""
    from stein_thinning import _native as nat
    x, mean, cov = _case(1237, d, 7 * d + mode)
    wl, wg = op.gaussian_proxy(x, mean, cov)
    tl, tg = op.student_t_proxy(x, mean, cov * 2, 3.5)
    assert nat.lib().st_tune(7, mode) == 0
    try:
        lq, gq = proxy.gaussian_proxy(x, mean, cov)
        ltq, gtq = proxy.student_t_proxy(x, mean, cov * 2, 3.5)
    finally:
        nat.lib().st_tune(7, 0)
    _close(lq, wl)
    _close(gq, wg)
    _close(ltq, tl)
    _close(gtq, tg)


@pytest.mark.parametrize('d', [1, 2, 3, 4, 8, 9, 12])
@pytest.mark.parametrize('weighted', [False, True])
def test_kde_proxy_matches_restatement(d, weighted):
    """KDE proxy (csrc/kde.hip) against oracle.proxy_numpy.kde_proxy (jax gaussian_kde restated):
    log q and grad log q to fp64 rounding, at the sample itself and at other points; the
    compile-time-d (d <= 8) and runtime-d kernels; uniform and weighted KDEs (cell 51)."""
    x, mean, cov = _case(1501, d, 31 * d + weighted)
    w = np.exp(-0.3 * np.sum((x - mean) ** 2, axis=1)) if weighted else None
    lq, gq = proxy.kde_proxy(x, bw_method='silverman', weights=w)
    wl, wg = op.kde_proxy(x, bw_method='silverman', weights=w)
    _close(lq, wl)
    _close(gq, wg)
    y = x[:257] * 1.1 + 0.05
    lq, gq = proxy.kde_proxy(x, y, bw_method='scott')
    wl, wg = op.kde_proxy(x, y, bw_method='scott')
    _close(lq, wl)
    _close(gq, wg)


def test_kde_gradient_free_curves_on_gpu(gm, curves):
    """Gaussian_mixture.ipynb cells 42-48 end to end on the GPU: the KDE proxy, thin_gf (1 000
    points, 'med'), calculate_ksd and the energy-distance curve -- against the report's gf_kde
    curves (report/figures/gaussian-mixture-comparison.pdf) at the PDF's precision."""
    from stein_thinning import energy as se
    from stein_thinning import stein as ss
    from stein_thinning import thinning as st
    sample, sample2, logpdf, score = gm
    log_q, gq = proxy.kde_proxy(sample, bw_method='silverman')
    idx = st.thin_gf(sample, logpdf(sample), log_q, gq, 1000, preconditioner='med')
    integrand = st._make_stein_integrand(sample, score(sample))
    ks = ss.ksd(integrand.reindex(idx), idx.shape[0])
    c = np.array(curves['ksd/gf_kde'])
    np.testing.assert_allclose(ks[c[:, 0].astype(int) - 1], c[:, 1], rtol=1e-7)
    c = np.array(curves['ed/gf_kde'])
    got = se.energy_distance_curve(sample2, sample, idx, c[:, 0].astype(int))
    np.testing.assert_allclose(got, c[:, 1], rtol=1.5e-8)
