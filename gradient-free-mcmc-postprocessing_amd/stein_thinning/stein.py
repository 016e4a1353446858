"""``stein_thinning.stein`` -- kernel Stein discrepancy of an ordered point set, and the Gram matrix.

Mirrors the reference dependency's ``ksd(integrand, n)`` (called through ``calculate_ksd``,
``code/src/utils/ksd.py:19-27``) and ``kmat(integrand, n)`` (``code/tests/test_ksd.py:20``,
``Gaussian_mixture.ipynb`` cells 94, 102, 106).

Device fast paths: a ``SteinIntegrand`` -- or the reference harness's re-indexed closure around
one (``reindex_integrand``, ``code/src/utils/ksd.py:9-16``: ``res(ind1, ind2) =
integrand(indices[ind1], indices[ind2])``) -- runs the LDS-tiled HIP kernels (``st_ksd_cumulative``
/ ``st_kmat``).  Any other callable (e.g. the matrix-lookup integrand of ``test_ksd.py``) follows
the reference's protocol loop, calling the user's integrand.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np

from .thinning import SteinIntegrand


def _resolve(integrand: Callable) -> Optional[Tuple[SteinIntegrand, Optional[np.ndarray]]]:
    """(SteinIntegrand, row indices or None) if the integrand can run on the device."""
    if isinstance(integrand, SteinIntegrand):
        return integrand, None
    cells = getattr(integrand, '__closure__', None)
    code = getattr(integrand, '__code__', None)
    if cells and code is not None and len(cells) == 2 and code.co_argcount == 2:
        vals = {name: c.cell_contents for name, c in zip(code.co_freevars, cells)}
        inner, indices = vals.get('integrand'), vals.get('indices')
        # the closure of code/src/utils/ksd.py:reindex_integrand, exactly
        if isinstance(inner, SteinIntegrand) and isinstance(indices, np.ndarray) \
                and indices.ndim == 1 and np.issubdtype(indices.dtype, np.integer) \
                and code.co_names == () and set(code.co_freevars) == {'integrand', 'indices'}:
            return inner, np.asarray(indices, dtype=np.int64)
    return None


def _device_rows(integrand, n: int):
    res = _resolve(integrand)
    if res is None:
        return None
    inner, indices = res
    prob = inner.device_problem()
    if indices is None:
        rows = np.arange(n, dtype=np.int64)
    else:
        rows = indices[:n]
        if rows.shape[0] < n:
            raise IndexError(f'index {rows.shape[0]} is out of bounds for axis 0 with size {rows.shape[0]}')
    if rows.size and (rows.min() < 0 or rows.max() >= prob.n):
        rows = np.arange(prob.n)[rows]   # reference semantics: negative wrap / IndexError
    return prob, rows


def ksd(integrand: Callable, n: int) -> np.ndarray:
    """Cumulative KSD: ks[i] = sqrt(sum_{a,b <= i} k(a, b)) / (i + 1), i < n."""
    n = int(n)
    dev = _device_rows(integrand, n)
    if dev is not None:
        prob, rows = dev
        if n == 0:
            return np.empty(0)
        sub = prob if (rows.shape[0] <= prob.n and np.array_equal(rows, np.arange(rows.shape[0]))) \
            else prob.subset(rows)
        return sub.ksd(n)
    ks = np.empty(n)
    ps = 0.
    for i in range(n):
        k0 = np.asarray(integrand(np.full(i + 1, i), np.arange(i + 1)))
        ps += 2 * np.sum(k0[:i]) + k0[i]
        ks[i] = np.sqrt(ps) / (i + 1)
    return ks


def kmat(integrand: Callable, n: int) -> np.ndarray:
    """Symmetric (n, n) matrix K[i, j] = integrand(i, j), filled from the upper triangle."""
    n = int(n)
    dev = _device_rows(integrand, n)
    if dev is not None:
        prob, rows = dev
        sub = prob if np.array_equal(rows, np.arange(rows.shape[0])) else prob.subset(rows)
        return sub.kmat(n)
    res = None
    for i in range(n):
        row = np.asarray(integrand(np.full(n - i, i), np.arange(i, n)))
        if res is None:
            res = np.zeros((n, n), dtype=row.dtype)
        res[i, i:] = row
        res[i:, i] = row
    return res if res is not None else np.zeros((0, 0))
