"""Seeded input generators for the golden fixtures and the bench -- TEST INFRASTRUCTURE ONLY.

* ``make_mvn_mixture`` restates the reference's Gaussian-mixture target
  (``code/src/utils/mvn.py:7-50``; rvs / logpdf / score, without the JAX variant) so the
  Gaussian-mixture fixtures of ``Gaussian_mixture.ipynb`` (cells 5-16) can be regenerated.
* ``gm_reference_sample`` reproduces the notebook's sample (weights/means/covs at cell 5,
  ``default_rng(12345)``, n=1000; ``Gaussian_mixture.ipynb:83-97,145``).
* ``bivariate_reference_sample`` reproduces ``Gradient_free_Stein_thinning.ipynb`` cells 2-6.
"""
from __future__ import annotations

import numpy as np
from scipy.stats import multivariate_normal as mvn


def make_mvn_mixture(weights, means, covs):
    covs_inv = np.linalg.inv(covs)
    k, d = means.shape

    def rvs(size, random_state):
        component_samples = [
            mvn.rvs(mean=means[i], cov=covs[i], size=size, random_state=random_state)
            for i in range(len(weights))
        ]
        indices = random_state.choice(len(weights), size=size, p=weights)
        return np.take_along_axis(
            np.stack(component_samples, axis=1), indices.reshape(size, 1, 1), axis=1).squeeze()

    def logpdf(x):
        f = np.stack([mvn.pdf(x, mean=means[i], cov=covs[i]) for i in range(len(weights))]).reshape(len(weights), -1)
        return np.log(np.einsum('i,il->l', weights, f))

    def score(x):
        xc = x[np.newaxis, :, :] - means[:, np.newaxis, :]
        f = np.stack([mvn.pdf(x, mean=means[i], cov=covs[i]) for i in range(len(weights))]).reshape(len(weights), -1)
        num = np.einsum('i,il,ijk,ilk->lj', weights, f, covs_inv, xc)
        den = np.einsum('i,il->l', weights, f)
        return -num / den[:, np.newaxis]

    return rvs, logpdf, score


GM_WEIGHTS = np.array([0.3, 0.7])
GM_MEANS = np.array([[-1., -1.], [1., 1.]])
GM_COVS = np.array([
    [[0.5, 0.25], [0.25, 1.]],
    [[2.0, -np.sqrt(3.) * 0.8], [-np.sqrt(3.) * 0.8, 1.5]],
])


def gm_reference_sample(n: int = 1000):
    """Returns (sample, sample2, logpdf, score) exactly as Gaussian_mixture.ipynb cells 8-10, 77."""
    rvs, logpdf, score = make_mvn_mixture(GM_WEIGHTS, GM_MEANS, GM_COVS)
    rng = np.random.default_rng(12345)
    sample = rvs(n, random_state=rng)
    sample2 = rvs(n, random_state=rng)
    return sample, sample2, logpdf, score


def bivariate_reference_sample(n: int = 1000):
    """Gradient_free_Stein_thinning.ipynb cells 2-6: N(0, [[1,.8],[.8,1]]), default_rng(12345)."""
    rng = np.random.default_rng(12345)
    means = np.array([0., 0.])
    covs = np.array([[1., 0.8], [0.8, 1.]])
    sample = mvn.rvs(mean=means, cov=covs, size=n, random_state=rng)
    gradient = np.einsum('kj,ij->ik', np.linalg.inv(covs), means - sample)
    log_p = mvn.logpdf(sample, mean=means, cov=covs)
    return sample, gradient, log_p, means, covs


def gaussian_proxy(sample: np.ndarray, ddof: int):
    """Simple Gaussian proxy q = N(sample mean, sample cov) -> (log_q, grad log_q, mean, cov)."""
    mean = np.mean(sample, axis=0)
    cov = np.cov(sample, rowvar=False, ddof=ddof)
    log_q = mvn.logpdf(sample, mean=mean, cov=cov)
    gradient_q = -np.einsum('ij,kj->ki', np.linalg.inv(cov), sample - mean)
    return log_q, gradient_q, mean, cov
