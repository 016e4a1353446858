"""NumPy restatement of the reference's Stein-thinning hot path -- TEST INFRASTRUCTURE ONLY.

This module is the CPU oracle.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker / the timed CPU
baseline.  The product (``stein_thinning`` shim + HIP library) never calls into it.

What it restates
----------------
The hot path lives in the third-party package ``stein_thinning`` (imported by the reference at
``code/src/thinning.py:5``, ``code/src/utils/ksd.py:5-6``, ``code/tests/test_ksd.py:3``; unpinned in
``pyproject.toml:31``, environment hint ``stein-thinning~=1.1.0`` at
``code/notebooks/examples/Dask_AWS.ipynb:656``).  That package is not present in
``/root/reference`` nor installable offline, so this file restates its published algorithm from
the reference's own restatements and maths:

* ``vfk0_imq``      -- ``JAX_Stein_Thinning.ipynb`` cell 27 (json line ~354-361),
                       ``Kernel_Stein_discrepancy.ipynb`` cell 7 (~126-141), ``report/report.tex:853-868``
* ``make_precon``   -- ``report.tex:432`` (median heuristic); called at ``JAX_Stein_Thinning.ipynb`` cell 28
* ``_greedy_search`` -- ``JAX_Stein_Thinning.ipynb`` cell 22 (~281-295) and ``report.tex:413-426``
* ``_validate_and_standardize`` -- called at ``JAX_Stein_Thinning.ipynb`` cell 16; per-dimension
                       mean-absolute-deviation scaling pinned by the golden index vectors of
                       ``Gradient_free_Stein_thinning.ipynb`` cell 8 (see tests/golden)
* gradient-free kernel ``w_i w_j k_Q`` -- ``report.tex:359-400``; warning text quoted at
                       ``Gaussian_mixture.ipynb:751-752`` (``thinning.py:127`` of the package)
* ``ksd`` / ``kmat`` -- integrand protocol used at ``code/src/utils/ksd.py:19-27`` and
                       ``code/tests/test_ksd.py:8-27``; cumulative KSD definition ``report.tex:311-313``

Parity pinning: every function is checked against the reference's printed outputs and the vector
curves of ``report/figures/gaussian-mixture-comparison.pdf`` by ``tests/test_oracle_golden.py``
(fixtures in ``tests/golden/``).  ``range_cap`` and the n>1000 ``'med'`` sub-sampling rule have no
fixture in the reference: "parity unpinned" for those two.

The arithmetic deliberately follows NumPy's evaluation order of the reference code (transposed
``(d, n)`` temporaries, ``np.dot`` with the preconditioner, axis-0 sums, ``**`` powers), because the
HIP kernel is specified to reproduce exactly those roundings.
"""
from __future__ import annotations

import warnings
from typing import Callable, Optional

import numpy as np
from numpy.linalg import inv
from scipy.spatial.distance import pdist

WEIGHT_SCALE_THRESHOLD = 10
MED_SUBSAMPLE = 1000


# --------------------------------------------------------------------------------------------
# kernel module (stein_thinning.kernel)
# --------------------------------------------------------------------------------------------
def vfk0_imq(a: np.ndarray, b: np.ndarray, sa: np.ndarray, sb: np.ndarray, linv: np.ndarray) -> np.ndarray:
    """IMQ Langevin Stein kernel, c=1, beta=-1/2.

    Restates ``JAX_Stein_Thinning.ipynb`` cell 27 with beta=-1/2 substituted
    (-4b(b-1) = -3, -2b = 1, qf**0.5 == sqrt) -- same NumPy op order as the package.
    """
    amb = a.T - b.T
    qf = 1 + np.sum(np.dot(linv, amb) * amb, axis=0)
    t1 = -3 * np.sum(np.dot(np.dot(linv, linv), amb) * amb, axis=0) / (qf ** 2.5)
    t2 = (np.trace(linv) + np.sum(np.dot(linv, sa.T - sb.T) * amb, axis=0)) / (qf ** 1.5)
    t3 = np.sum(sa.T * sb.T, axis=0) / (qf ** 0.5)
    return t1 + t2 + t3


def make_precon(sample: np.ndarray, preconditioner: str = 'id') -> np.ndarray:
    """Preconditioner Gamma^-1 (``JAX_Stein_Thinning.ipynb`` cell 28: ``make_precon(s, 'id')``).

    'id' -> I; 'med' -> inv(med^2 I) with med the median pairwise distance of (a sub-sample of)
    the standardised sample (report.tex:432); 'sclmed' and a float scale are the package's other
    isotropic options (unused by the reference notebooks -> unpinned).
    """
    n, d = sample.shape

    def med2():
        if n > MED_SUBSAMPLE:
            sub = sample[np.linspace(0, n - 1, MED_SUBSAMPLE, dtype=int)]
        else:
            sub = sample
        return np.median(pdist(sub)) ** 2

    if isinstance(preconditioner, str) and preconditioner == 'id':
        return np.identity(d)
    if isinstance(preconditioner, str) and preconditioner == 'med':
        m2 = med2()
        if m2 == 0:
            raise ValueError('Too few unique samples in smp.')
        return inv(m2 * np.identity(d))
    if isinstance(preconditioner, str) and preconditioner == 'sclmed':
        m2 = med2()
        if m2 == 0:
            raise ValueError('Too few unique samples in smp.')
        return inv(m2 / np.log(np.minimum(MED_SUBSAMPLE, n)) * np.identity(d))
    try:
        scale = float(preconditioner)
    except (TypeError, ValueError):
        raise ValueError('Incorrect preconditioner type.') from None
    return inv(scale * np.identity(d))


def make_imq(sample: np.ndarray, preconditioner: str = 'id') -> Callable:
    linv = make_precon(sample, preconditioner)

    def vfk0(a, b, sa, sb):
        return vfk0_imq(a, b, sa, sb, linv)
    return vfk0


# --------------------------------------------------------------------------------------------
# thinning module (stein_thinning.thinning)
# --------------------------------------------------------------------------------------------
def _validate_sample_and_gradient(sample: np.ndarray, gradient: np.ndarray) -> None:
    if sample.ndim != 2 or gradient.ndim != 2:
        raise ValueError('sample or gradient is not two-dimensional.')
    n, d = sample.shape
    if n == 0 or d == 0:
        raise ValueError('sample is empty.')
    if gradient.shape != (n, d):
        raise ValueError('Dimensions of sample and gradient are inconsistent.')
    if np.isnan(sample).any() or np.isnan(gradient).any():
        raise ValueError('sample or gradient contains NaNs.')
    if np.isinf(sample).any() or np.isinf(gradient).any():
        raise ValueError('sample or gradient contains infs.')


def _validate_and_standardize(sample: np.ndarray, gradient: np.ndarray, standardize: bool):
    """Per-dimension mean-absolute-deviation standardisation (pinned by F1, tests/golden)."""
    _validate_sample_and_gradient(sample, gradient)
    if standardize:
        loc = np.mean(sample, axis=0)
        scl = np.mean(np.abs(sample - loc), axis=0)
        if np.min(scl) == 0:
            raise ValueError('Too few unique samples in smp.')
        sample = sample / scl
        gradient = gradient * scl
    return sample, gradient


def _make_stein_integrand(sample, gradient, standardize: bool = True, preconditioner: str = 'id'):
    sample, gradient = _validate_and_standardize(sample, gradient, standardize)
    vfk0 = make_imq(sample, preconditioner)

    def stein_integrand(ind1, ind2):
        return vfk0(sample[ind1], sample[ind2], gradient[ind1], gradient[ind2])
    return stein_integrand


def _log_weights(log_p: np.ndarray, log_q: np.ndarray, range_cap: Optional[float]) -> np.ndarray:
    """log(q/p) anchored at its minimum; optional cap of its range (cap: parity unpinned)."""
    log_ratio = log_q - log_p
    if np.ptp(log_ratio) > WEIGHT_SCALE_THRESHOLD:
        warnings.warn(f'log_q differs from log_p by more than {WEIGHT_SCALE_THRESHOLD} '
                      f'- consider using q that matches target better')
    log_ratio = log_ratio - np.min(log_ratio)
    if range_cap is not None:
        log_ratio = np.minimum(log_ratio, range_cap)
    return log_ratio


def _make_stein_gf_integrand(sample, log_p, log_q, gradient_q, standardize: bool = True,
                             range_cap: Optional[float] = None, preconditioner: str = 'id'):
    sample, gradient_q = _validate_and_standardize(sample, gradient_q, standardize)
    log_p = np.asarray(log_p, dtype=np.float64).reshape(-1)
    log_q = np.asarray(log_q, dtype=np.float64).reshape(-1)
    if log_p.shape[0] != sample.shape[0] or log_q.shape[0] != sample.shape[0]:
        raise ValueError('Dimensions of sample and log densities are inconsistent.')
    weights = np.exp(_log_weights(log_p, log_q, range_cap))
    vfk0 = make_imq(sample, preconditioner)

    def stein_integrand(ind1, ind2):
        return vfk0(sample[ind1], sample[ind2], gradient_q[ind1], gradient_q[ind2]) * weights[ind1] * weights[ind2]
    return stein_integrand


def _greedy_search(n_points: int, integrand: Callable) -> np.ndarray:
    """Running-sum greedy selection (JAX_Stein_Thinning.ipynb cell 22; report.tex:413-426)."""
    idx = np.empty(n_points, dtype=np.uint32)
    k0 = integrand(slice(None), slice(None))
    idx[0] = np.argmin(k0)
    for i in range(1, n_points):
        k0 += 2 * integrand(slice(None), [idx[i - 1]])
        idx[i] = np.argmin(k0)
    return idx


def thin(sample, gradient, n_points, standardize=True, preconditioner='id'):
    integrand = _make_stein_integrand(sample, gradient, standardize, preconditioner)
    return _greedy_search(n_points, integrand)


def thin_gf(sample, log_p, log_q, gradient_q, n_points, standardize=True, range_cap=None, preconditioner='id'):
    integrand = _make_stein_gf_integrand(sample, log_p, log_q, gradient_q, standardize, range_cap, preconditioner)
    return _greedy_search(n_points, integrand)


# --------------------------------------------------------------------------------------------
# stein module (stein_thinning.stein)
# --------------------------------------------------------------------------------------------
def kmat(integrand: Callable, n: int) -> np.ndarray:
    """Full symmetric matrix K[i, j] = integrand(i, j), filled from the upper triangle."""
    res = None
    for i in range(n):
        row = np.asarray(integrand(np.full(n - i, i), np.arange(i, n)))
        if res is None:
            res = np.zeros((n, n), dtype=row.dtype)
        res[i, i:] = row
        res[i:, i] = row
    return res if res is not None else np.zeros((0, 0))


def ksd(integrand: Callable, n: int) -> np.ndarray:
    """Cumulative KSD: ks[i] = sqrt(sum_{a,b<=i} k(a,b)) / (i+1)."""
    ks = np.empty(n)
    ps = 0.
    for i in range(n):
        k0 = integrand(np.full(i + 1, i), np.arange(i + 1))
        ps += 2 * np.sum(k0[:i]) + k0[i]
        ks[i] = np.sqrt(ps) / (i + 1)
    return ks


# --------------------------------------------------------------------------------------------
# reference-harness callers (code/src/utils/ksd.py, code/src/thinning.py)
# --------------------------------------------------------------------------------------------
def reindex_integrand(integrand, indices):
    def res(ind1, ind2):
        return integrand(indices[ind1], indices[ind2])
    return res


def calculate_ksd(sample, gradient, idx):
    integrand = _make_stein_integrand(sample, gradient)
    return ksd(reindex_integrand(integrand, idx), idx.shape[0])


def energy_distance(x: np.ndarray, y: np.ndarray) -> float:
    """V-statistic energy distance 2E|X-Y| - E|X-X'| - E|Y-Y'| (dcor.energy_distance default)."""
    from scipy.spatial.distance import cdist
    return 2 * np.mean(cdist(x, y)) - np.mean(cdist(x, x)) - np.mean(cdist(y, y))
