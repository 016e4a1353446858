"""Proxy producers of the reference, restated with scipy -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` (and bench.py's cpu_baseline leg) import this module, as the checker of
``stein_thinning.proxy`` (csrc/proxy.hip).  scipy is the reference's own dependency for these
functions, so this is the reference computation itself, not a restatement of an absent package:

* ``gaussian_proxy`` / ``gaussian_thin`` -- ``code/src/thinning.py:14-17``
* ``t_grad_log_pdf``                     -- ``code/notebooks/lotka_volterra/Gradient_free_Student_t.ipynb``
                                            cell 31
* ``student_t_proxy`` / ``thin_gf_t``    -- same notebook, cells 29 and 40
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
