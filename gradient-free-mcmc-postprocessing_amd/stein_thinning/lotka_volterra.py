"""Lotka-Volterra posterior inputs on the GPU, batched over parameter points.

The reference's LV experiments feed Stein thinning with, for every MCMC sample theta,
* the gradient of the log posterior from the forward sensitivity equations
  (``Sensitivity_analysis.ipynb`` cells 16, 40, 46: ``solve_ivp(lotka_volterra_sensitivity, ...,
  dense_output=True)``, the likelihood gradient sum_k J_k^T C^-1 (y_k - u_k), minus log(theta)/theta),
  evaluated for the unique samples of each chain (``parallelise_for_unique``,
  ``code/src/utils/parallel.py``; 18 minutes for 113 143 points on the reference's machine,
  ``Dask_AWS.ipynb``), and
* the log target density ``lotka_volterra.log_target_density(log_theta)``
  (``code/src/lotka_volterra.py``) for the gradient-free operator's log p.

Each parameter point is one thread of ``csrc/lv.hip`` running scipy's RK45 algorithm step for step
(same tableau, initial step, step-size control and dense output), so the values agree with scipy to
rounding.  The observation data ``y`` and times ``t`` are inputs (the reference reads them from its
S3 bucket; ``reference_data()`` rebuilds them with the module's own recipe).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Optional, Sequence

import numpy as np

from . import _native as nat

T_SPAN = (0.0, 25.0)                  # code/src/lotka_volterra.py: t_span
T_N = 2400                            # t_n
THETA = np.array([0.67, 1.33, 1., 1.])  # theta (data-generating parameters)
U_INIT = (1.0, 1.0)                   # u_init
MEANS = np.array([0., 0.])
C = np.diag([0.2 ** 2, 0.2 ** 2])     # observation noise covariance
RTOL, ATOL = 1e-3, 1e-6               # scipy.integrate.solve_ivp defaults (the reference passes none)
MAX_STEPS = 1_000_000


@dataclass
class LvData:
    t: np.ndarray                     # (t_n,) ascending observation times
    y: np.ndarray                     # (t_n, 2) observations
    cov: np.ndarray = field(default_factory=lambda: C.copy())
    t_span: Sequence[float] = T_SPAN
    u_init: Sequence[float] = U_INIT


def reference_data() -> LvData:
    """The observations ``code/src/lotka_volterra.py`` builds at import: the RK45 solution at the
    true theta on np.linspace(0, 25, 2400) plus N(0, C) noise from default_rng(12345)."""
    from scipy import stats
    from scipy.integrate import solve_ivp

    def rhs(t, u, theta):
        theta1, theta2, theta3, theta4 = theta
        u1, u2 = u
        return [theta1 * u1 - theta2 * u1 * u2, theta4 * u1 * u2 - theta3 * u2]
    sol = solve_ivp(rhs, T_SPAN, list(U_INIT), args=(list(THETA),), dense_output=True)
    t = np.linspace(T_SPAN[0], T_SPAN[1], T_N)
    u = sol.sol(t).T
    eps = stats.multivariate_normal.rvs(mean=MEANS, cov=C, size=len(u), random_state=np.random.default_rng(12345))
    return LvData(t=t, y=u + eps)


def _points(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    if a.ndim == 1:
        a = a[None, :]
    if a.ndim != 2 or a.shape[1] != 4:
        raise ValueError(f'parameter points must be (n, 4) (or (4,)), got {a.shape}')
    return a


def _settings(data: LvData, rtol: float, atol: float):
    t = np.ascontiguousarray(data.t, dtype=np.float64)
    y = np.ascontiguousarray(data.y, dtype=np.float64)
    if t.ndim != 1 or y.shape != (t.size, 2):
        raise ValueError(f'need t (t_n,) and y (t_n, 2), got {t.shape} and {y.shape}')
    if t.size and np.any(np.diff(t) < 0):
        raise ValueError('observation times must be ascending')
    s = np.array([data.t_span[0], data.t_span[1], data.u_init[0], data.u_init[1], rtol, atol], dtype=np.float64)
    return t, y, s


def _status_check(status: np.ndarray, what: str):
    bad = np.flatnonzero(status)
    if bad.size:
        import warnings
        warnings.warn(f'{what}: the RK45 integration failed for {bad.size} parameter point(s) '
                      f'(first: {bad[0]}, status {status[bad[0]]}); their values are NaN', RuntimeWarning)


def grad_log_posterior(theta, data: Optional[LvData] = None, rtol: float = RTOL, atol: float = ATOL,
                       max_steps: int = MAX_STEPS, chunk: int = 1 << 16) -> np.ndarray:
    """``grad_log_posterior`` of Sensitivity_analysis.ipynb cell 46 for every row of ``theta``
    ((n, 4) or (4,)): returns (n, 4).  Two-phase kernels (``st_lv_grad_log_posterior_ws``), at most
    ``chunk`` points per launch (the step table is ~29 KB per point; fewer when device memory is
    short).  A point whose integration takes more than 64 accepted steps is recomputed by the
    single-phase kernel, whose sum over the observation times runs in time order instead of in
    pieces: the two forms agree to rounding (1e-11 relative, tests/test_gpu_lv.py), both within the
    1e-8 tolerance against scipy."""
    import torch
    data = reference_data() if data is None else data
    th = _points(theta)
    t, y, s = _settings(data, rtol, atol)
    cinv = np.ascontiguousarray(np.linalg.inv(np.asarray(data.cov, dtype=np.float64)))
    dev = nat.require_device()
    n = th.shape[0]
    out = torch.empty((max(n, 1), 4), dtype=torch.float64, device=dev)
    status = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    if n:
        L = nat.lib()
        thd, td, yd = (torch.from_numpy(a).to(dev) for a in (th, t, y))
        # the step table is ~29 KB per point: cap a launch's points at a quarter of the free device
        # memory (torch's caching allocator keeps the block for the next call)
        per_point = int(L.st_lv_grad_workspace_bytes(1, t.size))
        free, _ = torch.cuda.mem_get_info(dev)
        chunk = min(int(chunk), max(1024, free // 4 // per_point))
        m = min(n, chunk)
        wb = int(L.st_lv_grad_workspace_bytes(m, t.size))
        work = torch.empty((wb + 7) // 8, dtype=torch.float64, device=dev)
        for c0 in range(0, n, chunk):
            c1 = min(n, c0 + chunk)
            nat.check(L.st_lv_grad_log_posterior_ws(
                nat.ptr(thd[c0:c1]), c1 - c0, nat.ptr(td), t.size, nat.ptr(yd), s.ctypes.data, cinv.ctypes.data,
                int(max_steps), nat.ptr(out[c0:c1]), nat.ptr(status[c0:c1]), nat.ptr(work), wb,
                nat.stream_handle()), 'st_lv_grad_log_posterior_ws')
    res, st = out[:n].cpu().numpy(), status[:n].cpu().numpy()
    _status_check(st, 'grad_log_posterior')
    return res


def log_target_density(log_theta, data: Optional[LvData] = None, rtol: float = RTOL, atol: float = ATOL,
                       max_steps: int = MAX_STEPS, chunk: int = 1 << 16) -> np.ndarray:
    """``lotka_volterra.log_target_density`` for every row of ``log_theta`` ((n, 4) or (4,)):
    returns (n,)."""
    import torch
    from .proxy import PsdFactor
    data = reference_data() if data is None else data
    lth = _points(log_theta)
    th = np.exp(lth)                                   # as the reference: np.exp(log_theta)
    t, y, s = _settings(data, rtol, atol)
    psd = PsdFactor(np.asarray(data.cov, dtype=np.float64), allow_singular=False)
    c_log = psd.rank * float(np.log(2 * np.pi)) + psd.log_pdet
    U = np.ascontiguousarray(psd.U, dtype=np.float64)
    norm_logc = float(np.log(np.sqrt(2 * np.pi)))      # scipy.stats._continuous_distns._norm_pdf_logC
    dev = nat.require_device()
    L = nat.lib()
    n = th.shape[0]
    res = np.empty(n)
    st = np.zeros(n, dtype=np.int32)
    td, yd = (torch.from_numpy(a).to(dev) for a in (t, y))
    for c0 in range(0, n, chunk):
        c1 = min(n, c0 + chunk)
        m = c1 - c0
        ltd = torch.from_numpy(lth[c0:c1]).to(dev)
        thd = torch.from_numpy(th[c0:c1]).to(dev)
        out = torch.empty(m, dtype=torch.float64, device=dev)
        status = torch.zeros(m, dtype=torch.int32, device=dev)
        wb = int(L.st_lv_log_density_workspace_bytes(m, t.size))
        work = torch.empty((wb + 7) // 8, dtype=torch.float64, device=dev)
        nat.check(L.st_lv_log_target_density(
            nat.ptr(ltd), nat.ptr(thd), m, nat.ptr(td), t.size, nat.ptr(yd), s.ctypes.data, U.ctypes.data,
            c_log, norm_logc, int(max_steps), nat.ptr(out), nat.ptr(status), nat.ptr(work), wb,
            nat.stream_handle()), 'st_lv_log_target_density')
        res[c0:c1] = out.cpu().numpy()
        st[c0:c1] = status.cpu().numpy()
    _status_check(st, 'log_target_density')
    return res


def for_unique(func: Callable[[np.ndarray], np.ndarray], sample: np.ndarray) -> np.ndarray:
    """``parallelise_for_unique`` (code/src/utils/parallel.py) with a batched ``func``: evaluate the
    unique rows once, in one batch, and scatter back."""
    unique_samples, inverse_index = np.unique(sample, axis=0, return_inverse=True)
    return func(unique_samples)[inverse_index.reshape(-1)]
