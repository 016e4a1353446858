"""``stein_thinning.thinning`` -- Stein thinning front-end over the MI355X engine.

Mirrors the reference dependency's module as used by the reference repository:
``thin`` (``Stein_thinning.ipynb``; ``Gaussian_mixture.ipynb`` cell 28), ``thin_gf``
(``code/src/thinning.py:14-17``; ``Gradient_free_Stein_thinning.ipynb`` cells 13, 21),
``_greedy_search`` / ``_validate_and_standardize`` (``JAX_Stein_Thinning.ipynb`` cells 15-18),
``_make_stein_integrand`` (``code/src/utils/ksd.py:25``) and ``_make_stein_gf_integrand``
(``Gaussian_mixture.ipynb`` cell 93).  Same names, argument meaning and error behaviour
(ValueError on malformed input; UserWarning ``log_q differs from log_p by more than 10`` as quoted
at ``Gaussian_mixture.ipynb:751-752``).

Host work (validation, per-dimension standardisation, 'med' preconditioner, log-weights) is the
reference's O(n d) NumPy preprocessing, kept bit-identical; the greedy loop, the kernel columns
and the argmins run in HIP kernels on the GPU (``_native`` C-ABI).  Integrands built here are
``SteinIntegrand`` objects: calling them follows the reference's integrand protocol
``integrand(ind1, ind2)`` (evaluated on the GPU), and ``_greedy_search`` / ``stein.ksd`` /
``stein.kmat`` recognise them and run the whole computation on the device.
"""
from __future__ import annotations

import contextlib
import logging
import warnings
from typing import Callable, Optional

import numpy as np

from .kernel import make_precon

logger = logging.getLogger(__name__)

WEIGHT_SCALE_THRESHOLD = 10


def _as_numpy(a) -> np.ndarray:
    if hasattr(a, 'detach') and hasattr(a, 'cpu'):   # torch tensor (CPU or ROCm)
        a = a.detach().cpu().numpy()
    return np.asarray(a, dtype=np.float64)


def _host_buffer(shape) -> np.ndarray:
    """float64 host array for standardised data that is about to be uploaded: page-locked memory
    from torch's caching host allocator when a HIP device is present (the upload then runs at
    PCIe DMA speed instead of registering fresh pageable pages: 1 ms vs ~6 ms per 64 MB on the
    MI355X box), plain NumPy memory otherwise."""
    try:
        import torch
        if torch.cuda.is_available():
            return torch.empty(shape, dtype=torch.float64, pin_memory=True).numpy()
    except Exception:   # noqa: BLE001 -- pinned memory is an optimisation only
        pass
    return np.empty(shape, dtype=np.float64)


def _validate_shapes(sample: np.ndarray, gradient: np.ndarray) -> None:
    if sample.ndim != 2 or gradient.ndim != 2:
        raise ValueError('sample or gradient is not two-dimensional.')
    n, d = sample.shape
    if n == 0 or d == 0:
        raise ValueError('sample is empty.')
    if gradient.shape != (n, d):
        raise ValueError('Dimensions of sample and gradient are inconsistent.')


def _validate_and_standardize(sample, gradient, standardize: bool = True):
    """Validate, then (optionally) scale each dimension by its mean absolute deviation.

    loc = mean(x, 0); scl = mean(|x - loc|, 0); x / scl, g * scl  (per-dimension scaling pinned
    by the golden indices of ``Gradient_free_Stein_thinning.ipynb`` cell 8).  Evaluated by the
    host routine ``st_standardize_host`` of the native library in three passes (the NumPy
    expressions' reduction orders reproduced bit for bit; tests/test_shim_host.py), errors as the
    NumPy checks raise them.
    """
    import ctypes
    from . import _native as nat
    sample = np.ascontiguousarray(_as_numpy(sample))
    gradient = np.ascontiguousarray(_as_numpy(gradient))
    _validate_shapes(sample, gradient)
    n, d = sample.shape
    if d == 1 and np.getbufsize() != 8192:     # the native column sum models the default bufsize
        return _validate_and_standardize_numpy(sample, gradient, standardize)
    out_s = _host_buffer(sample.shape) if standardize else sample
    out_g = _host_buffer(gradient.shape) if standardize else gradient
    status = ctypes.c_int32(0)
    nat.check_host(nat.lib().st_standardize_host(
        sample.ctypes.data, gradient.ctypes.data, n, d, 1 if standardize else 0, out_s.ctypes.data,
        out_g.ctypes.data, None, None, ctypes.byref(status)), 'st_standardize_host')
    if status.value == 1:
        raise ValueError('sample or gradient contains NaNs.')
    if status.value == 2:
        raise ValueError('sample or gradient contains infs.')
    if status.value == 3:
        raise ValueError('Too few unique samples in smp.')
    return out_s, out_g


def _log_weights(log_p: np.ndarray, log_q: np.ndarray, range_cap: Optional[float]) -> np.ndarray:
    """log(q/p) anchored at its minimum (argmin-invariant global scale); optional range cap.

    The warning threshold tests np.ptp(log_q - log_p) (the quantity the reference inspects at
    ``Gradient_free.ipynb`` cell 47).  ``range_cap`` semantics are parity-unpinned (no fixture in
    the reference): the log-ratio range is capped from above after min-anchoring.
    """
    log_ratio = log_q - log_p
    if np.ptp(log_ratio) > WEIGHT_SCALE_THRESHOLD:
        warnings.warn(f'log_q differs from log_p by more than {WEIGHT_SCALE_THRESHOLD} '
                      f'- consider using q that matches target better')
    log_ratio = log_ratio - np.min(log_ratio)
    if range_cap is not None:
        log_ratio = np.minimum(log_ratio, range_cap)
    return log_ratio


def _validate_and_standardize_numpy(sample, gradient, standardize):
    """The NumPy expressions themselves (host preprocessing; used only when NumPy's ufunc buffer
    size was changed from its default, which the native routine models)."""
    if np.isnan(sample).any() or np.isnan(gradient).any():
        raise ValueError('sample or gradient contains NaNs.')
    if np.isinf(sample).any() or np.isinf(gradient).any():
        raise ValueError('sample or gradient contains infs.')
    if standardize:
        loc = np.mean(sample, axis=0)
        scl = np.mean(np.abs(sample - loc), axis=0)
        if np.min(scl) == 0:
            raise ValueError('Too few unique samples in smp.')
        sample = sample / scl
        gradient = gradient * scl
    return sample, gradient


class SteinIntegrand:
    """Stein-kernel integrand over a standardised sample, resident on the GPU on first use.

    ``integrand(ind1, ind2)`` returns k(x[ind1], x[ind2]) (times w[ind1] w[ind2] for the
    gradient-free kernel), broadcasting ind1 against ind2 like the reference's NumPy integrand.
    ``reindex(rows)`` is the view ``(a, b) -> integrand(rows[a], rows[b])`` -- what the reference
    harness's ``reindex_integrand`` closure computes (``code/src/utils/ksd.py:9-16``) -- sharing
    this integrand's device arrays; ``thin`` / ``stein.ksd`` / ``stein.kmat`` accept it directly.
    """

    def __init__(self, sample: np.ndarray, gradient: np.ndarray, linv: np.ndarray,
                 weights: Optional[np.ndarray] = None):
        from .device import isotropic_scale
        self._sample = sample
        self._gradient = gradient
        self._materialize = None   # deferred host arrays (_deferred): computed on first access
        self._n = sample.shape[0]
        self.linv = linv
        self.weights = weights
        iso = isotropic_scale(linv)
        if iso is None:
            raise NotImplementedError('only isotropic preconditioners run on the HIP engine')
        self.linv_scale, self.linv_trace = iso
        self._problem = None
        self._base: Optional['SteinIntegrand'] = None   # views: the integrand whose rows these index
        self._rows: Optional[np.ndarray] = None
        self._rec = None

    @classmethod
    def _deferred(cls, n: int, materialize: Callable, linv: np.ndarray,
                  weights: Optional[np.ndarray] = None) -> 'SteinIntegrand':
        """Integrand whose standardised host arrays are computed only if something reads them
        (``materialize() -> (sample, gradient)``): the drop-in thin's device-side standardisation
        (_upload_standardized) needs them on the host only for the sharded path and host-side
        helpers."""
        self = cls(np.empty((n, 0)), np.empty((n, 0)), linv, weights)
        self._sample = self._gradient = None
        self._materialize = materialize
        return self

    def _host_arrays(self) -> None:
        if self._sample is None:
            self._sample, self._gradient = self._materialize()
            self._materialize = None

    @property
    def sample(self) -> np.ndarray:
        self._host_arrays()
        return self._sample

    @property
    def gradient(self) -> np.ndarray:
        self._host_arrays()
        return self._gradient

    @property
    def n(self) -> int:
        return self._n if self._rows is None else self._rows.shape[0]

    def reindex(self, indices) -> 'SteinIntegrand':
        """View over rows ``indices`` of this integrand (no copy of the device arrays)."""
        view = SteinIntegrand.__new__(SteinIntegrand)
        view.__dict__.update(self.__dict__)
        view._problem = None
        view._rec = None
        view._base = self.base()
        view._rows = self.base_rows(np.asarray(indices, dtype=np.int64).reshape(-1))
        return view

    def base(self) -> 'SteinIntegrand':
        return self if self._base is None else self._base

    def base_rows(self, rows) -> np.ndarray:
        """Rows of the base integrand that this integrand's indices ``rows`` denote."""
        local = np.arange(self.n)[rows]   # reference indexing semantics (negative wrap, IndexError)
        return local if self._rows is None else self._rows[local]

    def base_problem(self):
        return self.base().device_problem()

    def run_starts_view(self):
        """(compact integrand of the run starts, their rows) on the host arrays, or None when the
        repeated-row path does not pay (device.DeviceProblem.dedup_view's rule and reasoning; used by
        the row-sharded thin, which builds every rank's shard from the host arrays)."""
        from .device import DEDUP_MAX_FRAC
        if self._base is not None or self.n < 2:
            return None
        cols = [self.sample, self.gradient] + ([self.weights.reshape(-1, 1)] if self.weights is not None else [])
        diff = np.zeros(self.n - 1, dtype=bool)
        for c in cols:
            u = np.ascontiguousarray(c).view(np.uint64)
            diff |= (u[1:] != u[:-1]).any(axis=1)
        rows = np.concatenate([[0], 1 + np.flatnonzero(diff)])
        if rows.size > DEDUP_MAX_FRAC * self.n:
            return None
        w = self.weights[rows] if self.weights is not None else None
        return SteinIntegrand(self.sample[rows], self.gradient[rows], self.linv, w), rows

    def device_problem(self):
        if self._problem is None:
            if self._base is not None:
                self._problem = self._base.device_problem().subset(self._rows)
            else:
                from .device import DeviceProblem
                self._problem = DeviceProblem(self.sample, self.gradient, self.weights,
                                              self.linv_scale, self.linv_trace)
                # a page-locked source is copied asynchronously, and torch records no event for a
                # buffer it did not allocate: wait here, so the copy has landed whatever happens to the
                # host arrays or the stream the problem is used on next
                self._problem.wait_upload()
        return self._problem

    @contextlib.contextmanager
    def recording(self):
        """Trace mode for stein.ksd / kmat dispatch: calls record their (broadcast) index arrays
        and return signed pair-specific sentinel values instead of evaluating (no GPU work)."""
        self._rec = []
        try:
            yield self._rec
        finally:
            self._rec = None

    def __call__(self, ind1, ind2) -> np.ndarray:
        i1 = np.atleast_1d(np.arange(self.n)[ind1])
        i2 = np.atleast_1d(np.arange(self.n)[ind2])
        b1, b2 = np.broadcast_arrays(i1, i2)
        if self._rec is not None:
            u1, u2 = b1.astype(np.int64), b2.astype(np.int64)
            sent = (((u1 * 2654435761 + u2 * 40503) % 1000003) + 0.375) * np.where((u1 + u2) % 2 == 0, 1.0, -1.0)
            self._rec.append((np.array(b1), np.array(b2), sent))
            return sent.copy()
        r1 = self.base_rows(b1.reshape(-1))
        r2 = self.base_rows(b2.reshape(-1))
        out = self.base_problem().pairs(r1, r2)
        return out.reshape(b1.shape)


def _early_upload(sample: np.ndarray, gradient: np.ndarray, weights: Optional[np.ndarray]):
    """Start the device copy of standardised, page-locked host arrays before the preconditioner is
    known (its 'med' heuristic is host work: the H2D DMA and the SoA layout run meanwhile); None when
    the arrays are not page-locked (no HIP device) -- the integrand then uploads on first use."""
    try:
        import torch
        if not (torch.cuda.is_available() and torch.from_numpy(sample).is_pinned()):
            return None
    except Exception:   # noqa: BLE001 -- an optimisation only
        return None
    from .device import DeviceProblem
    return DeviceProblem(sample, gradient, weights, 0.0, 0.0)   # l, tr filled in with the preconditioner


def _on_device(a) -> bool:
    """A ROCm tensor (torch reports HIP devices as 'cuda')."""
    return bool(getattr(a, 'is_cuda', False))


def _download_standardized(sample, gradient):
    """The drop-in thin's input path for ROCm tensors (float64, one device, standardize=True):
    the inputs stay where they are.  Only x travels, device to host, into a page-locked buffer
    (st_standardize_download: NumPy's sequential axis-0 sums of mean / mean |x - loc| as the chunks land,
    bit-identical), because its statistics and the 'med' subsample are host work; g's NaN / inf check is a
    device reduction and g is scaled on the device with x (st_layout_soa_scaled) -- never copied to the
    host.  Errors as _validate_and_standardize raises them (NaNs before infs, either array).  Returns
    _upload_standardized's tuple (stage_g None: the host g is fetched only if something reads
    integrand.gradient) or None (other dtypes, two devices, or d = 1 under a changed NumPy bufsize: the
    host route)."""
    import ctypes
    import torch
    from . import _native as nat
    _validate_shapes(sample, gradient)
    n, d = sample.shape
    if sample.dtype != torch.float64 or gradient.dtype != torch.float64 or sample.device != gradient.device \
            or (d == 1 and np.getbufsize() != 8192):   # the native d = 1 column sum models the default bufsize
        return None
    with torch.cuda.device(sample.device):
        x = sample.detach().contiguous()
        g = gradient.detach().contiguous()
        flags = torch.stack([torch.isnan(g).any(), torch.isinf(g).any()])   # queued before the download
        stage_x = _host_buffer((n, d))
        loc, scl = np.empty(d), np.empty(d)
        status = ctypes.c_int32(0)
        nat.check(nat.lib().st_standardize_download(nat.ptr(x), n, d, stage_x.ctypes.data, loc.ctypes.data,
                                                    scl.ctypes.data, ctypes.byref(status), nat.stream_handle()),
                  'st_standardize_download')
        g_nan, g_inf = (bool(v) for v in flags.tolist())
    if status.value == 1 or g_nan:
        raise ValueError('sample or gradient contains NaNs.')
    if status.value == 2 or g_inf:
        raise ValueError('sample or gradient contains infs.')
    if status.value == 3:
        raise ValueError('Too few unique samples in smp.')
    return n, d, scl, stage_x, None, x, g


def _upload_standardized(sample, gradient, standardize: bool):
    """The drop-in thin's input path when a HIP device is present, d = 2 .. 8 and n >= 65536:
    st_standardize_upload computes loc / scl on the host while the raw arrays are staged into
    page-locked buffers and copied to the device underneath, then the device lays them out with the
    scaling applied (st_layout_soa_scaled: x / scl, g * scl, the host's bits).  Returns
    (n, d, scl, stage_x, stage_g, x_raw, g_raw) or None (the st_standardize_host route applies).
    Raises the reference's ValueErrors like _validate_and_standardize.  ROCm tensor inputs take
    _download_standardized (no host copy of g)."""
    import ctypes
    if not standardize:
        return None
    try:
        import torch
        if not torch.cuda.is_available():
            return None
    except Exception:   # noqa: BLE001 -- an optimisation only
        return None
    from . import _native as nat
    if _on_device(sample) and _on_device(gradient):
        up = _download_standardized(sample, gradient)
        if up is not None:
            return up
    sample = np.ascontiguousarray(_as_numpy(sample))
    gradient = np.ascontiguousarray(_as_numpy(gradient))
    _validate_shapes(sample, gradient)
    n, d = sample.shape
    if not (2 <= d <= 8 and n >= 65536):
        return None
    dev = nat.require_device()
    stage_x, stage_g = _host_buffer(sample.shape), _host_buffer(gradient.shape)
    if not torch.from_numpy(stage_x).is_pinned():
        return None
    x_raw = torch.empty((n, d), dtype=torch.float64, device=dev)
    g_raw = torch.empty((n, d), dtype=torch.float64, device=dev)
    loc, scl = np.empty(d), np.empty(d)
    status = ctypes.c_int32(0)
    nat.check(nat.lib().st_standardize_upload(
        sample.ctypes.data, gradient.ctypes.data, n, d, stage_x.ctypes.data, stage_g.ctypes.data,
        nat.ptr(x_raw), nat.ptr(g_raw), loc.ctypes.data, scl.ctypes.data, ctypes.byref(status),
        nat.stream_handle()), 'st_standardize_upload')
    if status.value == 1:
        raise ValueError('sample or gradient contains NaNs.')
    if status.value == 2:
        raise ValueError('sample or gradient contains infs.')
    if status.value == 3:
        raise ValueError('Too few unique samples in smp.')
    return n, d, scl, stage_x, stage_g, x_raw, g_raw


def _device_integrand(up, preconditioner, weights: Optional[np.ndarray]) -> SteinIntegrand:
    """SteinIntegrand over _upload_standardized's device arrays; the host arrays are deferred."""
    from .device import DeviceProblem
    from .kernel import make_precon_rows
    n, d, scl, stage_x, stage_g, x_raw, g_raw = up
    prob = DeviceProblem.from_raw_device(x_raw, g_raw, weights, scl, 0.0, 0.0)

    def materialize():   # device-tensor inputs (stage_g None): g comes to the host only here
        return _validate_and_standardize(stage_x, stage_g if stage_g is not None else g_raw, True)
    try:
        # the preconditioner's subsample rows, standardised on the host (x / scl: the same IEEE divisions)
        linv = make_precon_rows(n, d, lambda rows: stage_x[rows] / scl, preconditioner, on_device=True)
        integrand = SteinIntegrand._deferred(n, materialize, linv, weights)
    except Exception:
        prob.wait_upload()   # the queued copies read the staging buffers about to be dropped
        raise
    return _attach(integrand, prob)


def _attach(integrand: SteinIntegrand, prob) -> SteinIntegrand:
    if prob is not None:
        prob.l, prob.tr = float(integrand.linv_scale), float(integrand.linv_trace)
        # the preconditioner took longer than the DMA: this normally returns at once, and it keeps
        # the integrand safe to use from any stream afterwards
        prob.wait_upload()
        integrand._problem = prob
    return integrand


def _make_stein_integrand(sample, gradient, standardize: bool = True, preconditioner='id') -> SteinIntegrand:
    with _on_home(sample):   # ROCm tensors: the problem lives on their device
        return _make_stein_integrand_here(sample, gradient, standardize, preconditioner)


def _make_stein_integrand_here(sample, gradient, standardize, preconditioner) -> SteinIntegrand:
    up = _upload_standardized(sample, gradient, standardize)
    if up is not None:
        return _device_integrand(up, preconditioner, None)
    sample, gradient = _validate_and_standardize(sample, gradient, standardize)
    prob = _early_upload(sample, gradient, None) if preconditioner == 'med' else None
    linv = make_precon(sample, preconditioner, on_device=prob is not None)
    return _attach(SteinIntegrand(sample, gradient, linv), prob)


def _make_stein_gf_integrand(sample, log_p, log_q, gradient_q, standardize: bool = True,
                             range_cap: Optional[float] = None, preconditioner='id') -> SteinIntegrand:
    with _on_home(sample):   # ROCm tensors: the problem lives on their device
        return _make_stein_gf_integrand_here(sample, log_p, log_q, gradient_q, standardize, range_cap,
                                             preconditioner)


def _make_stein_gf_integrand_here(sample, log_p, log_q, gradient_q, standardize, range_cap,
                                  preconditioner) -> SteinIntegrand:
    up = _upload_standardized(sample, gradient_q, standardize)
    if up is None:
        sample, gradient_q = _validate_and_standardize(sample, gradient_q, standardize)
        n = sample.shape[0]
    else:
        n = up[0]
    log_p = _as_numpy(log_p).reshape(-1)
    log_q = _as_numpy(log_q).reshape(-1)
    if log_p.shape[0] != n or log_q.shape[0] != n:
        raise ValueError('Dimensions of sample and log densities are inconsistent.')
    if np.isnan(log_p).any() or np.isnan(log_q).any():
        raise ValueError('log_p or log_q contains NaNs.')
    weights = np.exp(_log_weights(log_p, log_q, range_cap))
    if up is not None:
        return _device_integrand(up, preconditioner, weights)
    prob = _early_upload(sample, gradient_q, weights) if preconditioner == 'med' else None
    linv = make_precon(sample, preconditioner, on_device=prob is not None)
    return _attach(SteinIntegrand(sample, gradient_q, linv, weights), prob)


def _greedy_search_protocol(n_points: int, integrand: Callable) -> np.ndarray:
    """The reference's running-sum loop for arbitrary user integrands (plug-in protocol, e.g. the
    JAX integrand of ``JAX_Stein_Thinning.ipynb`` cell 30): the user's callable does the arithmetic."""
    idx = np.empty(n_points, dtype=np.uint32)
    k0 = np.array(integrand(slice(None), slice(None)), dtype=np.float64)
    idx[0] = np.argmin(k0)
    logger.debug('THIN: %d of %d', 1, n_points)
    for i in range(1, n_points):
        k0 += 2 * np.asarray(integrand(slice(None), [idx[i - 1]]))
        idx[i] = np.argmin(k0)
        logger.debug('THIN: %d of %d', i + 1, n_points)
    return idx


_SHARD_THIN: Optional[bool] = None   # set_rank_sharding(); None: the ST_SHARD_THIN environment variable


def set_rank_sharding(enabled: Optional[bool]) -> None:
    """Opt in (True) or out (False) of row sharding for the drop-in ``thin`` / ``thin_gf`` under a
    multi-rank launch; None returns to the ST_SHARD_THIN environment variable ('1' = on; off by
    default).  Sharding makes ``thin`` a collective: every rank must call it with the same problem."""
    global _SHARD_THIN
    _SHARD_THIN = None if enabled is None else bool(enabled)


def _rank_sharding() -> bool:
    """True when thin / thin_gf should shard their candidate rows across the ranks: the caller opted
    in (set_rank_sharding(True) or ST_SHARD_THIN=1) and torch.distributed is initialised with more
    than one rank (e.g. torchrun, one process per GPU).  Off by default: a sharded thin is a
    collective, and scripts that thin on one rank only, or a different chain on every rank (the
    reference's per-chain fan-out, ``code/src/utils/parallel.py:48-52``), must keep every call local."""
    import os
    enabled = _SHARD_THIN if _SHARD_THIN is not None else os.environ.get('ST_SHARD_THIN', '0') == '1'
    if not enabled:
        return False
    try:
        import torch.distributed as dist
    except ImportError:
        return False
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _greedy_search(n_points: int, integrand: Callable) -> np.ndarray:
    """Greedy KSD minimisation (Algorithm 3, report.tex:413-426); returns uint32 indices.

    SteinIntegrand -> the whole m-step loop runs on the GPU (one persistent launch, or one fused
    kernel per step; no host round trip); under a multi-rank launch that opted in
    (set_rank_sharding / ST_SHARD_THIN=1) its rows are sharded across the ranks
    (stein_thinning.distributed.thin_across_ranks, same indices).  Any other callable ->
    the reference protocol loop.
    """
    n_points = int(n_points)
    if n_points < 0:
        raise ValueError('negative dimensions are not allowed')
    if n_points == 0:
        raise IndexError('index 0 is out of bounds for axis 0 with size 0')
    if isinstance(integrand, SteinIntegrand):
        if integrand._base is None and _rank_sharding():
            from .distributed import thin_across_ranks
            return thin_across_ranks(integrand, n_points)
        from . import _native as nat
        return integrand.device_problem().greedy(n_points, dedup=_dedup(), guard=nat.near_tie_guard())
    return _greedy_search_protocol(n_points, integrand)


_DEDUP = None


def set_dedup(enabled: Optional[bool]) -> None:
    """Thin only the first row of each run of repeated rows (DeviceProblem.dedup_view: the same
    indices bit for bit, a fraction of the pair work on MCMC output full of rejected proposals):
    True / False, or None to return to the ST_DEDUP environment variable ('0' = off; on by default)."""
    global _DEDUP
    _DEDUP = None if enabled is None else bool(enabled)


def _dedup() -> bool:
    import os
    return _DEDUP if _DEDUP is not None else os.environ.get('ST_DEDUP', '1') != '0'


def _guard() -> bool:
    from . import _native as nat
    return nat.near_tie_guard()


def _home(a):
    """The device index of a ROCm tensor input, else None."""
    return a.device.index if _on_device(a) else None


def _on_home(a):
    """Run on the device a ROCm tensor input lives on (its arrays are used in place), else as is."""
    if _home(a) is None:
        return contextlib.nullcontext()
    import torch
    return torch.cuda.device(a.device)


def thin(sample, gradient, n_points: int, standardize: bool = True, preconditioner='id') -> np.ndarray:
    """Stein thinning: indices of ``n_points`` rows of ``sample`` greedily minimising the KSD.  ``sample`` /
    ``gradient`` may be NumPy arrays or ROCm tensors (used in place on their device: _download_standardized)."""
    with _on_home(sample):
        integrand = _make_stein_integrand(sample, gradient, standardize, preconditioner)
        return _greedy_search(n_points, integrand)


def _thin_chains(count: int, build: Callable, n_points, homes=None) -> list:
    """The per-chain loop ``[thin(...) for each chain]`` with the thins side by side: chain i's integrand is
    ``build(i)`` (validation errors in the loop's order: chain 0's input, then n_points, then the other
    chains'), the chains are dealt round-robin to the GPUs this process may use (all visible ones, or
    the one the device policy pins: _native.select_device_index), and each GPU runs its chains with
    device.greedy_concurrent (one batch launch: each latency-bound thin on a share of the CUs), the GPUs
    at the same time; a chain given as ROCm tensors runs on their device (homes[i]).  The same indices as
    the loop."""
    import torch
    from . import _native as nat
    from .device import greedy_concurrent
    n_points = int(n_points)
    nat.require_device()
    devs = ([torch.cuda.current_device()] if nat.policy_pinned() or count < 2
            else list(range(torch.cuda.device_count())))
    owner = [devs[i % len(devs)] if homes is None or homes[i] is None else homes[i] for i in range(count)]
    integrands = []
    for i in range(count):
        with torch.cuda.device(owner[i]):
            integrands.append(build(i))
        if i == 0:   # the loop's first thin() checks n_points after its input
            if n_points < 0:
                raise ValueError('negative dimensions are not allowed')
            if n_points == 0:
                raise IndexError('index 0 is out of bounds for axis 0 with size 0')
    if count == 0:
        return []
    groups = {}
    for i, dv in enumerate(owner):
        groups.setdefault(dv, []).append(i)

    def run(dv, ids):
        with torch.cuda.device(dv):
            return greedy_concurrent([integrands[i].device_problem() for i in ids], n_points, dedup=_dedup(),
                                     guard=_guard())
    out = [None] * count
    if len(groups) == 1:
        (dv, ids), = groups.items()
        for i, r in zip(ids, run(dv, ids)):
            out[i] = r
        return out
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=len(groups)) as ex:   # one host thread per GPU (HIP calls drop the GIL)
        futs = {dv: ex.submit(run, dv, ids) for dv, ids in groups.items()}
        for dv, ids in groups.items():
            for i, r in zip(ids, futs[dv].result()):
                out[i] = r
    return out


def _same_length(*lists) -> int:
    n = len(lists[0])
    if any(len(x) != n for x in lists[1:]):
        raise ValueError('samples and gradients (and log densities) must have one entry per chain')
    return n


def thin_chains(samples, gradients, n_points: int, standardize: bool = True, preconditioner='id') -> list:
    """``[thin(s, g, n_points, standardize, preconditioner) for s, g in zip(samples, gradients)]`` -- the
    reference's per-chain loop (Stein_thinning.ipynb cells 12-14, fanned out over processes by
    code/src/utils/parallel.py:48-52) -- with the thins side by side: on each GPU in one batch launch, and
    over the visible GPUs (_thin_chains); the same indices as the loop."""
    samples, gradients = list(samples), list(gradients)
    count = _same_length(samples, gradients)
    return _thin_chains(count, lambda i: _make_stein_integrand(samples[i], gradients[i], standardize,
                                                               preconditioner), n_points,
                        [_home(x) for x in samples])


def thin_gf_chains(samples, log_ps, log_qs, gradients_q, n_points: int, standardize: bool = True,
                   range_cap: Optional[float] = None, preconditioner='id') -> list:
    """``[thin_gf(s, lp, lq, gq, n_points, ...) for ...]`` with the thins side by side (see thin_chains);
    the same indices as the loop."""
    samples, log_ps, log_qs, gradients_q = list(samples), list(log_ps), list(log_qs), list(gradients_q)
    count = _same_length(samples, log_ps, log_qs, gradients_q)
    return _thin_chains(count, lambda i: _make_stein_gf_integrand(samples[i], log_ps[i], log_qs[i], gradients_q[i],
                                                                  standardize, range_cap, preconditioner),
                        n_points, [_home(x) for x in samples])


def thin_gf(sample, log_p, log_q, gradient_q, n_points: int, standardize: bool = True,
            range_cap: Optional[float] = None, preconditioner='id') -> np.ndarray:
    """Gradient-free Stein thinning with auxiliary density q (report.tex:390-426)."""
    with _on_home(sample):
        integrand = _make_stein_gf_integrand(sample, log_p, log_q, gradient_q, standardize, range_cap,
                                             preconditioner)
        return _greedy_search(n_points, integrand)
