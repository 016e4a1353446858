"""Proxy producers of the reference, restated with scipy -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` (and bench.py's cpu_baseline leg) import this module, as the checker of
``stein_thinning.proxy`` (csrc/proxy.hip).  scipy is the reference's own dependency for these
functions, so this is the reference computation itself, not a restatement of an absent package:

* ``gaussian_proxy`` / ``gaussian_thin`` -- ``code/src/thinning.py:14-17``
* ``t_grad_log_pdf``                     -- ``code/notebooks/lotka_volterra/Gradient_free_Student_t.ipynb``
                                            cell 31
* ``student_t_proxy`` / ``thin_gf_t``    -- same notebook, cells 29 and 40
* ``kde_proxy``                          -- ``code/notebooks/gaussian_mixture/Gaussian_mixture.ipynb``
                                            cells 42-48 (51: weighted): jax.scipy.stats.gaussian_kde
                                            (jax is absent here; its published algorithm is restated:
                                            scipy's gaussian_kde constructor, whitening by the
                                            Cholesky factor of the precision, a logsumexp over the
                                            data, and the analytic gradient of that logsumexp, which
                                            is what jax.grad returns).  Pinned by the report's
                                            gradient-free-KDE curves (tests/test_oracle_golden.py)
"""
from __future__ import annotations

import numpy as np
from scipy import stats
from scipy.stats import multivariate_normal as mvn

from . import stein_numpy as sn


def gaussian_proxy(sample, mean, cov):
    log_q = mvn.logpdf(sample, mean=mean, cov=cov)
    gradient_q = -np.einsum('ij,kj->ki', np.linalg.inv(cov), sample - mean)
    return log_q, gradient_q


def t_grad_log_pdf(x, mu, sigma, df):
    d = x.shape[1]
    sigma_inv = np.linalg.inv(sigma)
    x_mu = x - mu
    direction_scaled = np.einsum('jk,ik->ij', sigma_inv, x_mu)
    mahalanobis_d = np.einsum('ij,jk,ik->i', x_mu, sigma_inv, x_mu)
    return -(df + d) / df / (1 + mahalanobis_d / df).reshape(-1, 1) * direction_scaled


def student_t_proxy(sample, loc, shape, df):
    log_q = stats.multivariate_t.logpdf(sample, loc=loc, shape=shape, df=df)
    return log_q, t_grad_log_pdf(sample, loc, shape, df)


def gaussian_thin(sample, log_p, mean, cov, thinned_size, range_cap=200):
    log_q, gradient_q = gaussian_proxy(sample, mean, cov)
    return sn.thin_gf(sample, log_p, log_q, gradient_q, thinned_size, range_cap=range_cap, preconditioner='med')


def thin_gf_t(sample, log_p, t_mu, t_scale, t_df, thinned_size, range_cap=200):
    log_q, gradient_q = student_t_proxy(sample, t_mu, t_scale, t_df)
    return sn.thin_gf(sample, log_p, log_q, gradient_q, thinned_size, range_cap=range_cap)


def kde_proxy(sample, points=None, bw_method='silverman', weights=None):
    from scipy.special import logsumexp
    x = np.asarray(sample, dtype=np.float64)
    y = x if points is None else np.asarray(points, dtype=np.float64)
    n, d = x.shape
    w = np.full(n, 1.0 / n) if weights is None else np.asarray(weights, dtype=np.float64) / np.sum(weights)
    neff = 1.0 / np.sum(w ** 2)
    if bw_method == 'scott':
        factor = np.power(neff, -1.0 / (d + 4))
    elif bw_method == 'silverman':
        factor = np.power(neff * (d + 2) / 4.0, -1.0 / (d + 4))
    else:
        factor = float(bw_method)
    cov = np.atleast_2d(np.cov(x.T, rowvar=1, bias=False, aweights=w))
    L = np.linalg.cholesky(np.linalg.inv(cov) / factor ** 2)
    pts, qs = x @ L, y @ L
    log_norm = np.sum(np.log(np.diag(L))) - 0.5 * d * np.log(2 * np.pi)
    diff = pts[None, :, :] - qs[:, None, :]                      # (m, n, d)
    arg = np.log(w)[None, :] + (log_norm - 0.5 * np.sum(diff * diff, axis=2))
    log_q = logsumexp(arg, axis=1)
    s = np.exp(arg - log_q[:, None])
    return log_q, np.einsum('mi,mid->md', s, diff) @ L.T
