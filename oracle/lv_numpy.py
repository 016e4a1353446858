"""Lotka-Volterra gradient / log density with scipy -- TEST INFRASTRUCTURE ONLY (checker of
stein_thinning.lotka_volterra / csrc/lv.hip).  Restates code/src/lotka_volterra.py (model,
sensitivity system, log_target_density) and Sensitivity_analysis.ipynb cells 16, 40, 46
(grad_log_likelihood, grad_log_posterior) on top of scipy's solve_ivp, the reference's solver."""
from __future__ import annotations

import numpy as np
import scipy.stats as stats
from numpy.linalg import inv
from scipy.integrate import solve_ivp


def lotka_volterra(t, u, theta):
    theta1, theta2, theta3, theta4 = theta
    u1, u2 = u
    return [theta1 * u1 - theta2 * u1 * u2, theta4 * u1 * u2 - theta3 * u2]


def lotka_volterra_sensitivity(t, uw, theta):
    theta1, theta2, theta3, theta4 = theta
    u1, u2, w1, w2, w3, w4, w5, w6, w7, w8 = uw
    return [
        theta1 * u1 - theta2 * u1 * u2,
        theta4 * u1 * u2 - theta3 * u2,
        u1 + (theta1 - theta2 * u2) * w1 - theta2 * u1 * w5,
        -u1 * u2 + (theta1 - theta2 * u2) * w2 - theta2 * u1 * w6,
        (theta1 - theta2 * u2) * w3 - theta2 * u1 * w7,
        (theta1 - theta2 * u2) * w4 - theta2 * u1 * w8,
        theta4 * u2 * w1 + (theta4 * u1 - theta3) * w5,
        theta4 * u2 * w2 + (theta4 * u1 - theta3) * w6,
        -u2 + theta4 * u2 * w3 + (theta4 * u1 - theta3) * w7,
        u1 * u2 + theta4 * u2 * w4 + (theta4 * u1 - theta3) * w8,
    ]


def grad_log_posterior(theta, t, y, C, t_span=(0, 25), u_init=(1., 1.)):
    q, d = 2, 4
    uw_init = np.concatenate([np.array(u_init), np.zeros(d * q)])
    sol = solve_ivp(lotka_volterra_sensitivity, t_span, uw_init, args=(theta,), dense_output=True)
    sensitivity_forward = sol.sol(t).T
    J = sensitivity_forward[:, q:].reshape(len(t), -1, q, order='F')
    grad_log_phi = (inv(C) @ (y - sensitivity_forward[:, :q]).T).T[:, :, np.newaxis]
    grad_log_lik = np.sum(np.squeeze(J @ grad_log_phi), axis=0)
    return grad_log_lik - np.log(theta) / theta


def log_target_density(log_theta, t, y, C, t_span=(0, 25), u_init=(1., 1.)):
    sol = solve_ivp(lotka_volterra, t_span, list(u_init), args=(np.exp(log_theta),), dense_output=True)
    u = sol.sol(t).T
    log_likelihood = np.sum(stats.multivariate_normal.logpdf(y - u, mean=[0, 0], cov=C))
    log_prior = np.sum(stats.norm.logpdf(log_theta))
    return log_likelihood + log_prior


def n_steps(theta, t_span=(0, 25), u_init=(1., 1.), sensitivity=True):
    """Accepted RK45 steps scipy takes (for reporting)."""
    if sensitivity:
        sol = solve_ivp(lotka_volterra_sensitivity, t_span, np.concatenate([np.array(u_init), np.zeros(8)]),
                        args=(theta,), dense_output=True)
    else:
        sol = solve_ivp(lotka_volterra, t_span, list(u_init), args=(theta,), dense_output=True)
    return len(sol.t) - 1
