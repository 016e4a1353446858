"""Proxy producers on the CPU: the scipy-based oracle against closed forms, and the product's
host-side argument handling (no device needed)."""
import numpy as np
import pytest

from oracle import proxy_numpy as op


def _spd(d, rng):
    a = rng.normal(size=(d, d))
    return a @ a.T / d + 0.5 * np.eye(d)


def test_oracle_gaussian_matches_closed_form():
    rng = np.random.default_rng(0)
    d = 5
    cov = _spd(d, rng)
    mean = rng.normal(size=d)
    x = rng.normal(size=(200, d))
    lq, gq = op.gaussian_proxy(x, mean, cov)
    prec = np.linalg.inv(cov)
    dev = x - mean
    want = -0.5 * (d * np.log(2 * np.pi) + np.linalg.slogdet(cov)[1] + np.einsum('ij,jk,ik->i', dev, prec, dev))
    np.testing.assert_allclose(lq, want, rtol=1e-12)
    np.testing.assert_allclose(gq, -dev @ prec, rtol=1e-12, atol=1e-13)


def test_oracle_student_t_gradient_is_the_logpdf_gradient():
    rng = np.random.default_rng(1)
    d = 3
    shape = _spd(d, rng)
    loc = rng.normal(size=d)
    x = rng.normal(size=(5, d))
    _, gq = op.student_t_proxy(x, loc, shape, 4.5)
    h = 1e-6
    for k in range(d):
        e = np.zeros(d)
        e[k] = h
        fd = (op.student_t_proxy(x + e, loc, shape, 4.5)[0] - op.student_t_proxy(x - e, loc, shape, 4.5)[0]) / (2 * h)
        np.testing.assert_allclose(gq[:, k], fd, rtol=1e-6, atol=1e-8)


def test_oracle_student_t_tends_to_gaussian():
    rng = np.random.default_rng(2)
    d = 4
    cov = _spd(d, rng)
    x = rng.normal(size=(50, d))
    lt, gt = op.student_t_proxy(x, np.zeros(d), cov, 1e9)
    lg, gg = op.gaussian_proxy(x, np.zeros(d), cov)
    np.testing.assert_allclose(lt, lg, rtol=1e-6)
    np.testing.assert_allclose(gt, gg, rtol=1e-6, atol=1e-9)


def test_product_validates_arguments_before_any_device_work():
    from stein_thinning import proxy
    x = np.zeros((10, 3))
    with pytest.raises(ValueError, match='2-d'):
        proxy.gaussian_proxy(np.zeros(10), np.zeros(1), np.eye(1))
    with pytest.raises(ValueError, match='length 3'):
        proxy.gaussian_proxy(x, np.zeros(2), np.eye(3))
    with pytest.raises(ValueError, match=r'\(3, 3\)'):
        proxy.gaussian_proxy(x, np.zeros(3), np.eye(2))
    with pytest.raises(np.linalg.LinAlgError):
        proxy.gaussian_proxy(x, np.zeros(3), np.diag([1.0, 1.0, 0.0]))     # scipy: singular
    with pytest.raises(ValueError, match='df'):
        proxy.student_t_proxy(x, np.zeros(3), np.eye(3), 0.0)
    with pytest.raises(ValueError, match='df'):
        proxy.student_t_proxy(x, np.zeros(3), np.eye(3), np.inf)


@pytest.mark.parametrize('d', [1, 2, 5, 50])
def test_psd_factor_is_scipys(d):
    """stein_thinning.proxy.PsdFactor returns scipy's _PSD factor bit for bit (the kernel's U)."""
    from scipy.stats._multivariate import _PSD
    from stein_thinning.proxy import PsdFactor
    rng = np.random.default_rng(d)
    m = _spd(d, rng)
    for allow in (True, False):
        a, b = PsdFactor(m, allow), _PSD(m, allow_singular=allow)
        assert np.array_equal(a.U, b.U) and a.rank == b.rank and a.log_pdet == b.log_pdet
    sing = np.diag([1.0] * (d - 1) + [0.0]) if d > 1 else np.zeros((1, 1))
    with pytest.raises(np.linalg.LinAlgError):
        PsdFactor(sing, allow_singular=False)
    if d > 1:
        a, b = PsdFactor(sing, True), _PSD(sing, allow_singular=True)
        assert np.array_equal(a.U, b.U) and a.rank == b.rank
