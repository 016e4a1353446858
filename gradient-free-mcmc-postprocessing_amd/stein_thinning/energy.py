"""Energy distance on the GPU -- the reference's thinning-quality metric.

The reference scores every thinned subsample with ``dcor.energy_distance`` (V-statistic,
exponent 1): ``fit_quality(subsample) = sqrt(dcor.energy_distance(validation[::10], subsample))``
(``code/notebooks/lotka_volterra/Comparison.ipynb`` cell 19, ``Gradient_free_Student_t.ipynb``),
and ``Gaussian_mixture.ipynb`` cells 63-71 evaluate it for prefixes of the selected indices.
``dcor`` is not installed here; the restatement it is checked against is
``oracle.stein_numpy.energy_distance`` (pinned to the notebooks' printed values, tests/golden).

    ED(x, y) = 2 E|X - Y| - E|X - X'| - E|Y - Y'|      (all means over all ordered pairs)

Device work: K7 (``st_distance_colsum_ws``): per point of A, the sum of Euclidean distances to a
range of B (or to the earlier points of A itself), the B range split over blockIdx.y chunks so that
a short A (the selected points) against a long B (the validation sample) still fills the chip.  ``energy_distance_curve`` evaluates all prefixes of
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


def _colsum(a, na, lda, b, nb, ldb, d, b0, b1, tri, device, host=True):
    """Per point of A: sum of distances to B[b0:b1] (strictly earlier points when tri), with the B
    range split over enough blocks to fill the GPU (st_distance_colsum_ws)."""
    import torch
    L = nat.lib()
    out = torch.zeros(max(na, 1), dtype=torch.float64, device=device)
    wsb = int(L.st_distance_workspace_bytes(na, b0, b1))
    ws = torch.empty(max(wsb // 8, 2), dtype=torch.float64, device=device)
    nat.check(L.st_distance_colsum_ws(nat.ptr(a), lda, na, nat.ptr(b), ldb, nb, d, b0, b1, 1 if tri else 0,
                                      nat.ptr(out), nat.ptr(ws), ws.numel() * 8, nat.stream_handle()),
              'st_distance_colsum_ws')
    return out[:na].cpu().numpy() if host else out[:na]


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


class EnergyCurve:
    """The reference's fit_quality curve, sqrt(ED(reference_points, sample[idx[:k]])) for every k in
    ``sizes`` (Comparison.ipynb cells 19-23), with both point sets resident on the GPU: the
    reference set's self term once, the cross sums once per selected point, the selection's self
    sums once (instead of one full dcor evaluation per prefix)."""

    def __init__(self, reference_points, selection):
        x, y = _points(reference_points), _points(selection)
        _check(x, y)
        self.device = nat.require_device()
        self.xs, self.nx, self.d, self.ldx = _soa(x, self.device)
        self.ys, self.ny, _, self.ldy = _soa(y, self.device)

    def pair_count(self) -> int:
        """Distance evaluations per run: the reference set's triangle, the cross block, the
        selection's triangle."""
        return self.nx * (self.nx - 1) // 2 + self.nx * self.ny + self.ny * (self.ny - 1) // 2

    def launch(self, sizes):
        """Enqueue one curve evaluation (device tensors; no host sync)."""
        import torch
        dev, d = self.device, self.d
        xx = _colsum(self.xs, self.nx, self.ldx, self.xs, self.nx, self.ldx, d, 0, self.nx, True, dev, host=False).sum()
        cross = torch.cumsum(_colsum(self.ys, self.ny, self.ldy, self.xs, self.nx, self.ldx, d, 0, self.nx, False,
                                     dev, host=False), 0)                       # per selected point
        yy = torch.cumsum(_colsum(self.ys, self.ny, self.ldy, self.ys, self.ny, self.ldy, d, 0, self.ny, True,
                                  dev, host=False), 0)                          # sum_{a<j} |y_a - y_j|
        si = torch.as_tensor(np.asarray(sizes, dtype=np.int64) - 1, device=dev)
        k = (si + 1).to(torch.float64)
        nx = float(self.nx)
        ed = 2.0 * cross[si] / (nx * k) - 2.0 * xx / (nx * nx) - 2.0 * yy[si] / (k * k)
        return torch.sqrt(ed)

    def run(self, sizes) -> np.ndarray:
        return self.launch(sizes).cpu().numpy()


def energy_distance_curve(reference_points, sample, idx, sizes) -> np.ndarray:
    """sqrt(energy_distance(reference_points, sample[idx[:k]])) for every k in ``sizes`` -- the
    reference's fit_quality curve (Comparison.ipynb cells 19-23) in one pass."""
    s = _points(sample)
    sizes = np.asarray(sizes, dtype=np.int64).reshape(-1)
    idx = np.asarray(idx, dtype=np.int64).reshape(-1)
    kmax = int(sizes.max()) if sizes.size else 0
    if kmax > idx.shape[0] or (sizes.size and sizes.min() < 1):
        raise ValueError('sizes must lie in [1, len(idx)]')
    return EnergyCurve(reference_points, s[idx[:kmax]]).run(sizes)
