"""Proxy producers for gradient-free Stein thinning: log q and grad log q on the GPU.

The reference builds the proxy q of ``thin_gf`` on the host before every gradient-free thin:

* ``gaussian_thin(sample, log_p, mean, cov, thinned_size, range_cap=200)``
  (``code/src/thinning.py:14-17``): ``log_q = scipy.stats.multivariate_normal.logpdf(sample, mean,
  cov)``, ``gradient_q = -np.einsum('ij,kj->ki', np.linalg.inv(cov), sample - mean)``;
* ``thin_gf_t(sample, log_p, t_mu, t_scale, t_df, thinned_size)``
  (``code/notebooks/lotka_volterra/Gradient_free_Student_t.ipynb`` cells 29, 31, 40):
  ``log_q = scipy.stats.multivariate_t.logpdf(sample, loc, shape, df)``, ``gradient_q =
  t_grad_log_pdf(sample, loc, shape, df)``; both with ``range_cap=200``.

* the KDE proxy of ``Gaussian_mixture.ipynb`` cells 42-48 (and the weighted KDE of cell 51):
  ``kde = jax.scipy.stats.gaussian_kde(sample.T, bw_method='silverman'[, weights=w])``,
  ``log_q = kde.logpdf(sample.T)``, ``gradient_q`` = jax.grad of it at every row
  (``kde_proxy``; O(n^2 d): csrc/kde.hip, ``st_kde_logpdf_grad``).

The parametric proxies are O(n d^2) per proxy (C5: n = 5e5, d = 50).  Here the d x d factors are computed on the host
exactly as scipy does (``_PSD``: eigh, pseudo-inverse square root; ``np.linalg.inv``; the scalar
constants in scipy's operation order) and the per-row work runs in one HIP kernel
(``st_proxy_logpdf_grad``, csrc/proxy.hip).  The per-row dot products are summed in a different
order than NumPy/BLAS: log q and grad log q agree with scipy to fp64 rounding (tests: relative
1e-12), not bit for bit.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np

from . import _native as nat

_LOG_2PI = float(np.log(2 * np.pi))   # scipy.stats._multivariate._LOG_2PI


class PsdFactor:
    """The factorisation scipy's multivariate_normal / multivariate_t logpdf use
    (scipy.stats._multivariate._PSD, restated on its public pieces so the same doubles come out):
    eigh of the lower triangle, eigenvalues below 1e6 * eps * max|eigenvalue| treated as zero,
    U = eigenvectors * sqrt(pseudo-inverse eigenvalues) (so U U^T = pinv(M)), log pseudo-determinant
    and rank."""

    def __init__(self, m: np.ndarray, allow_singular: bool = True):
        import scipy.linalg
        m = np.asarray(m)
        s, u = scipy.linalg.eigh(m, lower=True, check_finite=True)
        eps = 1e6 * np.finfo(s.dtype.char.lower()).eps * np.max(abs(s))
        if np.min(s) < -eps:
            raise ValueError('The input matrix must be symmetric positive semidefinite.')
        d = s[s > eps]
        if len(d) < len(s) and not allow_singular:
            raise np.linalg.LinAlgError('When `allow_singular is False`, the input matrix must be '
                                        'symmetric positive definite.')
        s_pinv = np.array([0 if abs(x) <= eps else 1 / x for x in s], dtype=float)
        self.U = np.multiply(u, np.sqrt(s_pinv))
        self.rank = len(d)
        self.log_pdet = np.sum(np.log(d))


def _psd(m: np.ndarray, allow_singular: bool) -> PsdFactor:
    return PsdFactor(m, allow_singular=allow_singular)


def _params(sample, loc, cov):
    x = np.ascontiguousarray(sample, dtype=np.float64)
    if x.ndim != 2:
        raise ValueError(f'sample must be 2-d (n, d), got shape {x.shape}')
    d = x.shape[1]
    loc = np.zeros(d) if loc is None else np.asarray(loc, dtype=np.float64).reshape(-1)
    if loc.shape != (d,):
        raise ValueError(f"location must be a vector of length {d}, got shape {loc.shape}")
    cov = np.asarray(cov, dtype=np.float64)
    if cov.ndim == 0:
        cov = cov * np.eye(d)
    elif cov.ndim == 1:
        cov = np.diag(cov)
    if cov.shape != (d, d):
        raise ValueError(f'covariance / shape matrix must be ({d}, {d}), got {cov.shape}')
    return x, loc, cov


def _device_eval(x, loc, whiten, precision, df: float, c_log: float):
    import torch
    dev = nat.require_device()
    n, d = x.shape
    log_q = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    grad = torch.empty((max(n, 1), d), dtype=torch.float64, device=dev)
    if n:
        xd = torch.from_numpy(x).to(dev)
        ld = torch.from_numpy(np.ascontiguousarray(loc)).to(dev)
        ud = torch.from_numpy(np.ascontiguousarray(whiten, dtype=np.float64)).to(dev)
        pd = torch.from_numpy(np.ascontiguousarray(precision, dtype=np.float64)).to(dev)
        nat.check(nat.lib().st_proxy_logpdf_grad(nat.ptr(xd), n, d, nat.ptr(ld), nat.ptr(ud), nat.ptr(pd),
                                                 float(df), float(c_log), nat.ptr(log_q), nat.ptr(grad),
                                                 nat.stream_handle()), 'st_proxy_logpdf_grad')
    return log_q[:n].cpu().numpy(), grad[:n].cpu().numpy()


def gaussian_proxy(sample, mean, cov) -> Tuple[np.ndarray, np.ndarray]:
    """(log_q, gradient_q) of the Gaussian proxy N(mean, cov) at every row of ``sample``:
    ``multivariate_normal.logpdf(sample, mean, cov)`` and ``-inv(cov) @ (x - mean)`` per row
    (code/src/thinning.py:15-16).  Raises like scipy / NumPy on a singular covariance."""
    x, mean, cov = _params(sample, mean, cov)
    psd = _psd(cov, allow_singular=False)
    precision = np.linalg.inv(cov)
    return _device_eval(x, mean, psd.U, precision, 0.0, psd.rank * _LOG_2PI + psd.log_pdet)


def student_t_proxy(sample, loc, shape, df: float) -> Tuple[np.ndarray, np.ndarray]:
    """(log_q, gradient_q) of the multivariate t proxy: ``multivariate_t.logpdf(sample, loc, shape,
    df)`` and the notebook's ``t_grad_log_pdf(sample, loc, shape, df)``
    (Gradient_free_Student_t.ipynb cells 29, 31)."""
    from scipy.special import gammaln
    x, loc, shape = _params(sample, loc, shape)
    df = float(df)
    if not df > 0 or not math.isfinite(df):
        raise ValueError("'df' must be a finite number greater than zero")
    d = x.shape[1]
    psd = _psd(shape, allow_singular=True)        # scipy.stats.multivariate_t's default
    precision = np.linalg.inv(shape)               # t_grad_log_pdf: np.linalg.inv(sigma)
    if psd.rank < d:
        raise ValueError('singular shape matrix')
    # scipy multivariate_t._logpdf: A - B - C - D + E, constants in its order
    t = 0.5 * (df + d)
    c_log = gammaln(t) - gammaln(0.5 * df) - d / 2. * np.log(df * np.pi) - 0.5 * psd.log_pdet
    return _device_eval(x, loc, psd.U, precision, df, float(c_log))


def kde_factors(dataset, bw_method='silverman', weights=None):
    """The constructor arithmetic of jax.scipy.stats.gaussian_kde (= scipy.stats.gaussian_kde) on an
    (n, d) dataset: normalised weights, n_eff, the bandwidth factor ('scott', 'silverman' or a
    scalar), the weighted data covariance, the precision inv(cov) / factor^2 and its lower
    Cholesky factor L (the kernel evaluation whitens with it: points @ L), log_norm =
    sum(log diag L) - d/2 log(2 pi).  Returns (weights, L, log_norm)."""
    x = np.asarray(dataset, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    n, d = x.shape
    if n < 2:
        raise ValueError('a KDE needs at least two data points')
    w = np.full(n, 1.0 / n) if weights is None else np.asarray(weights, dtype=np.float64).reshape(-1)
    if w.shape != (n,):
        raise ValueError(f'weights must have length {n}')
    w = w / np.sum(w)
    neff = 1.0 / np.sum(w ** 2)
    if bw_method is None or bw_method == 'scott':
        factor = np.power(neff, -1.0 / (d + 4))
    elif bw_method == 'silverman':
        factor = np.power(neff * (d + 2) / 4.0, -1.0 / (d + 4))
    elif np.isscalar(bw_method) and not isinstance(bw_method, str):
        factor = float(bw_method)
    else:
        raise ValueError("bw_method must be 'scott', 'silverman' or a scalar")
    cov = np.atleast_2d(np.cov(x.T, rowvar=1, bias=False, aweights=w))
    inv_cov = np.linalg.inv(cov) / factor ** 2
    L = np.linalg.cholesky(inv_cov)
    log_norm = float(np.sum(np.log(np.diag(L))) - 0.5 * d * np.log(2 * np.pi))
    return w, L, log_norm


def kde_proxy(sample, points=None, bw_method='silverman', weights=None) -> Tuple[np.ndarray, np.ndarray]:
    """(log_q, gradient_q) of the Gaussian KDE of ``sample`` at ``points`` (default: the sample
    itself) -- ``gaussian_kde(sample.T, bw_method, weights).logpdf(points.T)`` and its gradient, as
    Gaussian_mixture.ipynb cells 46-48 / 51 compute them for thin_gf.  The O(n m d) pair sums run
    on the GPU (st_kde_logpdf_grad); agrees with the restatement to fp64 rounding (the
    logsumexp and the softmax-weighted sums are sequential here, pairwise in NumPy)."""
    import torch
    from .device import padded_ld
    data = np.asarray(sample, dtype=np.float64)
    data = data[:, None] if data.ndim == 1 else data
    pts = data if points is None else np.asarray(points, dtype=np.float64)
    pts = pts[:, None] if pts.ndim == 1 else pts
    n, d = data.shape
    if pts.ndim != 2 or pts.shape[1] != d:
        raise ValueError(f'points must be (m, {d})')
    m = pts.shape[0]
    w, L, log_norm = kde_factors(data, bw_method, weights)
    dev = nat.require_device()
    log_q = torch.empty(max(m, 1), dtype=torch.float64, device=dev)
    grad = torch.empty((max(m, 1), d), dtype=torch.float64, device=dev)
    if m:
        def soa(a):
            ld = padded_ld(a.shape[0])
            t = torch.zeros((d, ld), dtype=torch.float64, device=dev)
            t[:, :a.shape[0]] = torch.from_numpy(np.ascontiguousarray((a @ L).T)).to(dev)   # whitened: a @ L
            return t, ld
        p_t, ldp = soa(data)
        q_t, ldq = soa(pts)
        uniform = weights is None
        logw = None if uniform else torch.from_numpy(np.log(w)).to(dev)
        lt = torch.from_numpy(np.ascontiguousarray(L)).to(dev)
        wsb = int(nat.lib().st_kde_workspace_bytes(m, d))
        ws = torch.empty(max(wsb // 8, 2), dtype=torch.float64, device=dev)
        nat.check(nat.lib().st_kde_logpdf_grad(nat.ptr(p_t), ldp, n, nat.ptr(logw), float(np.log(1.0 / n)),
                                               nat.ptr(q_t), ldq, m, d, log_norm, nat.ptr(lt), nat.ptr(log_q),
                                               nat.ptr(grad), nat.ptr(ws), ws.numel() * 8, nat.stream_handle()),
                  'st_kde_logpdf_grad')
    return log_q[:m].cpu().numpy(), grad[:m].cpu().numpy()


def gaussian_thin(sample, log_p, mean, cov, thinned_size: int, range_cap: Optional[float] = 200) -> np.ndarray:
    """code/src/thinning.py:14-17 with the proxy evaluated on the GPU."""
    from .thinning import thin_gf
    log_q, gradient_q = gaussian_proxy(sample, mean, cov)
    return thin_gf(sample, log_p, log_q, gradient_q, thinned_size, range_cap=range_cap, preconditioner='med')


def thin_gf_t(sample, log_p, t_mu, t_scale, t_df, thinned_size: int, range_cap: Optional[float] = 200) -> np.ndarray:
    """Gradient_free_Student_t.ipynb cell 40 with the proxy evaluated on the GPU (that cell keeps
    thin_gf's default preconditioner 'id')."""
    from .thinning import thin_gf
    log_q, gradient_q = student_t_proxy(sample, t_mu, t_scale, t_df)
    return thin_gf(sample, log_p, log_q, gradient_q, thinned_size, range_cap=range_cap)
