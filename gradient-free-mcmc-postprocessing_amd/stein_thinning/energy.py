"""Energy distance on the GPU -- the reference's thinning-quality metric.

The reference scores every thinned subsample with ``dcor.energy_distance`` (V-statistic,
exponent 1): ``fit_quality(subsample) = sqrt(dcor.energy_distance(validation[::10], subsample))``
(``code/notebooks/lotka_volterra/Comparison.ipynb`` cell 19, ``Gradient_free_Student_t.ipynb``),
and ``Gaussian_mixture.ipynb`` cells 63-71 evaluate it for prefixes of the selected indices.
``dcor`` is not installed here; the restatement it is checked against is
``oracle.stein_numpy.energy_distance`` (pinned to the notebooks' printed values, tests/golden).

    ED(x, y) = 2 E|X - Y| - E|X - X'| - E|Y - Y'|      (all means over all ordered pairs)

Device work: K7 (``st_distance_colsum``): per point of A, the sum of Euclidean distances to a range
of B (or to the earlier points of A itself).  ``energy_distance_curve`` evaluates all prefixes of
one selection in one pass: the validation set's self term once, the cross sums once per selected
point, the selection's self sums once -- instead of one dcor call (and one n_v^2 self term) per
prefix.  Sums of the per-point totals are formed on the host in float64.
"""
from __future__ import annotations

import numpy as np

from . import _native as nat
from .device import padded_ld


def _soa(points: np.ndarray, device):
    import torch
    pts = np.ascontiguousarray(points, dtype=np.float64)
    if pts.ndim == 1:
        pts = pts[:, None]
    n, d = pts.shape
    ld = padded_ld(n)
    soa = torch.zeros((d, ld), dtype=torch.float64, device=device)
    if n:
        soa[:, :n] = torch.from_numpy(np.ascontiguousarray(pts.T)).to(device)
    return soa, n, d, ld


def _colsum(a, na, lda, b, nb, ldb, d, b0, b1, tri, device):
    import torch
    out = torch.zeros(max(na, 1), dtype=torch.float64, device=device)
    nat.check(nat.lib().st_distance_colsum(nat.ptr(a), lda, na, nat.ptr(b), ldb, nb, d, b0, b1,
                                           1 if tri else 0, nat.ptr(out), nat.stream_handle()),
              'st_distance_colsum')
    return out[:na].cpu().numpy()


def _points(a) -> np.ndarray:
    """(n, d) float64; a 1-d array is n points in one dimension (dcor's convention)."""
    a = np.asarray(a, dtype=np.float64)
    return a[:, None] if a.ndim == 1 else a


def _check(x, y):
    if x.ndim != 2 or y.ndim != 2 or x.shape[1] != y.shape[1]:
        raise ValueError(f'x and y must be 2-d with the same number of columns ({x.shape}, {y.shape})')
    if x.shape[0] == 0 or y.shape[0] == 0:
        raise ValueError('energy distance of an empty sample')


def energy_distance(x, y) -> float:
    """dcor.energy_distance(x, y) (V-statistic, exponent 1), evaluated on the GPU."""
    x, y = _points(x), _points(y)
    _check(x, y)
    dev = nat.require_device()
    xs, nx, d, ldx = _soa(x, dev)
    ys, ny, _, ldy = _soa(y, dev)
    cross = _colsum(xs, nx, ldx, ys, ny, ldy, d, 0, ny, False, dev).sum()
    xx = _colsum(xs, nx, ldx, xs, nx, ldx, d, 0, nx, True, dev).sum()
    yy = _colsum(ys, ny, ldy, ys, ny, ldy, d, 0, ny, True, dev).sum()
    return float(2.0 * cross / (nx * ny) - 2.0 * xx / (nx * nx) - 2.0 * yy / (ny * ny))


def energy_distance_curve(reference_points, sample, idx, sizes) -> np.ndarray:
    """sqrt(energy_distance(reference_points, sample[idx[:k]])) for every k in ``sizes`` -- the
    reference's fit_quality curve (Comparison.ipynb cells 19-23) in one pass."""
    x = _points(reference_points)
    s = _points(sample)
    sizes = np.asarray(sizes, dtype=np.int64).reshape(-1)
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    kmax = int(sizes.max()) if sizes.size else 0
    if kmax > idx.shape[0] or (sizes.size and sizes.min() < 1):
        raise ValueError('sizes must lie in [1, len(idx)]')
    y = s[idx[:kmax]]
    _check(x, y)
    dev = nat.require_device()
    xs, nx, d, ldx = _soa(x, dev)
    ys, ny, _, ldy = _soa(y, dev)
    xx = _colsum(xs, nx, ldx, xs, nx, ldx, d, 0, nx, True, dev).sum()
    cross = np.cumsum(_colsum(ys, ny, ldy, xs, nx, ldx, d, 0, nx, False, dev))   # per selected point
    yy = np.cumsum(_colsum(ys, ny, ldy, ys, ny, ldy, d, 0, ny, True, dev))       # sum_{a<j} |y_a - y_j|
    k = sizes.astype(np.float64)
    ed = 2.0 * cross[sizes - 1] / (nx * k) - 2.0 * xx / (nx * nx) - 2.0 * yy[sizes - 1] / (k * k)
    return np.sqrt(ed)
