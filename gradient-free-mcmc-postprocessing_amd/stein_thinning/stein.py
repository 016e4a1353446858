"""``stein_thinning.stein`` -- kernel Stein discrepancy of an ordered point set, and the Gram matrix.

Mirrors the reference dependency's ``ksd(integrand, n)`` (called through ``calculate_ksd``,
``code/src/utils/ksd.py:19-27``) and ``kmat(integrand, n)`` (``code/tests/test_ksd.py:20``,
``Gaussian_mixture.ipynb`` cells 94, 102, 106).

Dispatch, for an integrand passed in:

* a ``SteinIntegrand`` (or its ``reindex(rows)`` view): the LDS-tiled HIP kernels
  (``st_ksd_cumulative`` / ``st_kmat``) over its rows, one launch;
* any other callable that reaches exactly ONE ``SteinIntegrand`` (through closure cells,
  ``functools.partial``, bound methods or instance attributes -- e.g. the reference harness's
  ``reindex_integrand`` closure, ``code/src/utils/ksd.py:9-16``, under any name): the wrapper is
  traced once with the inner integrand recording instead of computing (it returns pair-specific
  sentinel values, so a wrapper that transforms the values is detected), which yields the row map
  ``rows`` with ``wrapper(a, b) == inner(rows[a], rows[b])``; the device kernels then run over
  ``rows`` (one launch).  A wrapper that does its own arithmetic is evaluated in row blocks: all pairs of a
  block of the reference loop's rows in ONE wrapper call (its inner integrand is elementwise over
  index arrays), summed in the reference's order;
* any other callable (e.g. the matrix-lookup integrand of ``test_ksd.py``): the reference's protocol
  loop, one call per row, exactly as the reference issues them.
"""
from __future__ import annotations

import functools
import types
from typing import Callable, List, Optional, Tuple

import numpy as np

from .thinning import SteinIntegrand

_PAIR_BLOCK = 1 << 22   # pairs per batched wrapper call (32 MB of results)


def _children(obj):
    """Objects a callable holds on to: partial func/args, closure cells, bound self, attributes."""
    if isinstance(obj, functools.partial):
        yield obj.func
        yield from obj.args
        yield from obj.keywords.values()
    for c in getattr(obj, '__closure__', None) or ():
        try:
            yield c.cell_contents
        except ValueError:   # empty cell
            pass
    owner = getattr(obj, '__self__', None)
    if owner is not None and not isinstance(owner, types.ModuleType):
        yield owner
    attrs = None if isinstance(obj, (type, types.ModuleType)) else getattr(obj, '__dict__', None)
    if isinstance(attrs, dict):
        yield from attrs.values()


def _reachable_integrands(obj, depth: int = 0, seen=None) -> List[SteinIntegrand]:
    """Distinct SteinIntegrand objects reachable from a callable (depth <= 4, cycles skipped)."""
    seen = set() if seen is None else seen
    if id(obj) in seen or depth > 4:
        return []
    seen.add(id(obj))
    if isinstance(obj, SteinIntegrand):
        return [obj]
    found: List[SteinIntegrand] = []
    for k in _children(obj):
        if isinstance(k, SteinIntegrand) or callable(k):
            for f in _reachable_integrands(k, depth + 1, seen):
                if all(f is not g for g in found):
                    found.append(f)
    return found


def _inner_integrand(integrand: Callable) -> Optional[SteinIntegrand]:
    found = _reachable_integrands(integrand)
    return found[0] if len(found) == 1 else None


def _record_rows(integrand: Callable, inner: SteinIntegrand, n: int) -> Optional[np.ndarray]:
    """rows with integrand(a, b) == inner(rows[a], rows[b]) for index arrays a, b < n, or None.

    One call of the wrapper on the probes (arange(n), reversed arange(n)) with ``inner`` in
    recording mode (no GPU work): inner records the indices it receives and returns signed,
    pair-specific sentinel values.  Accepted only if the wrapper made exactly one inner call,
    mapped both probes through the same row vector, and returned the sentinels unchanged (a
    wrapper that scales, shifts or otherwise transforms the values is not a pure re-indexing)."""
    if n == 0:
        return np.empty(0, dtype=np.int64)
    a = np.arange(n, dtype=np.int64)
    b = a[::-1].copy()
    try:
        with inner.recording() as rec:
            out = np.asarray(integrand(a, b))
    except Exception:   # noqa: BLE001 -- an integrand we cannot trace runs the protocol loop
        return None
    if len(rec) != 1 or out.shape != (n,):
        return None
    r1, r2, sent = rec[0]
    if r1.shape != (n,) or r2.shape != (n,) or not np.array_equal(r2, r1[::-1]):
        return None
    if out.dtype != np.float64 or not np.array_equal(out, sent.reshape(-1)):
        return None
    rows = r1.astype(np.int64)
    # second, independent probe (two random permutations): the map must hold for it too -- a
    # wrapper that swaps its arguments (inner(perm[b], perm[a])) passes the reversed-arange probe
    # with rows = perm[::-1] but fails here
    rng = np.random.default_rng(0x5eed)
    a2, b2 = rng.permutation(n), rng.permutation(n)
    try:
        with inner.recording() as rec:
            out2 = np.asarray(integrand(a2, b2))
    except Exception:   # noqa: BLE001
        return None
    if len(rec) != 1 or out2.shape != (n,):
        return None
    q1, q2, sent2 = rec[0]
    if not (np.array_equal(q1, rows[a2]) and np.array_equal(q2, rows[b2])
            and out2.dtype == np.float64 and np.array_equal(out2, sent2.reshape(-1))):
        return None
    return rows


def _device_rows(integrand: Callable, n: int) -> Optional[Tuple[SteinIntegrand, np.ndarray]]:
    if isinstance(integrand, SteinIntegrand):
        inner, rows = integrand, np.arange(n, dtype=np.int64)
        if n > inner.n:
            raise IndexError(f'index {inner.n} is out of bounds for axis 0 with size {inner.n}')
        return inner, rows
    inner = _inner_integrand(integrand)
    if inner is None:
        return None
    rows = _record_rows(integrand, inner, n)
    if rows is None:
        return None
    return inner, rows


def _problem(inner: SteinIntegrand, rows: np.ndarray):
    prob = inner.base_problem()
    rows = inner.base_rows(rows)
    if rows.size and (rows.min() < 0 or rows.max() >= prob.n):
        rows = np.arange(prob.n)[rows]   # reference semantics: negative wrap / IndexError
    if rows.shape[0] <= prob.n and np.array_equal(rows, np.arange(rows.shape[0])):
        return prob
    return prob.subset(rows)


def _row_blocks(n: int, start_pairs):
    """Consecutive row blocks [i0, i1) whose pair counts (start_pairs(i0, i1)) stay near _PAIR_BLOCK."""
    i0 = 0
    while i0 < n:
        i1 = i0 + 1
        while i1 < n and start_pairs(i0, i1 + 1) <= _PAIR_BLOCK:
            i1 += 1
        yield i0, i1
        i0 = i1


_ELEMENTWISE_PREFIX = 8   # reference-loop rows compared against one batched call


def _elementwise(integrand: Callable, calls) -> bool:
    """True iff ONE call on the concatenated index arrays of ``calls`` (a few of the reference
    loop's (ind1, ind2) calls) returns exactly what the separate calls return: only then may the
    loop's calls be batched (a wrapper that uses ind1[0], len(ind2), or mixes elements is not
    elementwise and keeps the per-row protocol)."""
    try:
        sep = [np.asarray(integrand(i1, i2), dtype=np.float64).reshape(-1) for i1, i2 in calls]
        one = np.asarray(integrand(np.concatenate([c[0] for c in calls]), np.concatenate([c[1] for c in calls])),
                         dtype=np.float64).reshape(-1)
    except Exception:   # noqa: BLE001 -- not batchable: the reference loop raises or runs as it would
        return False
    return np.array_equal(one, np.concatenate(sep), equal_nan=True)


def ksd(integrand: Callable, n: int) -> np.ndarray:
    """Cumulative KSD: ks[i] = sqrt(sum_{a,b <= i} k(a, b)) / (i + 1), i < n."""
    n = int(n)
    dev = _device_rows(integrand, n)
    if dev is not None:
        if n == 0:
            return np.empty(0)
        return _problem(*dev).ksd(n)
    ks = np.empty(n)
    ps = 0.
    if _inner_integrand(integrand) is not None and _elementwise(
            integrand, [(np.full(i + 1, i), np.arange(i + 1)) for i in range(min(n, _ELEMENTWISE_PREFIX))]):
        # batched: the reference loop's calls for rows [i0, i1) as ONE call, summed per row in its order
        for i0, i1 in _row_blocks(n, lambda a, b: (b * (b + 1) - a * (a + 1)) // 2):
            lens = np.arange(i0, i1) + 1
            ind1 = np.repeat(np.arange(i0, i1), lens)
            ind2 = np.concatenate([np.arange(i + 1) for i in range(i0, i1)])
            vals = np.asarray(integrand(ind1, ind2))
            off = 0
            for i in range(i0, i1):
                k0 = vals[off:off + i + 1]
                off += i + 1
                ps += 2 * np.sum(k0[:i]) + k0[i]
                ks[i] = np.sqrt(ps) / (i + 1)
        return ks
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
        return _problem(*dev).kmat(n)
    res = None
    if _inner_integrand(integrand) is not None and n > 0 and _elementwise(
            integrand, [(np.full(n - i, i), np.arange(i, n)) for i in range(min(n, 2))]):
        for i0, i1 in _row_blocks(n, lambda a, b: (b - a) * n - (b * (b - 1) - a * (a - 1)) // 2):
            ind1 = np.repeat(np.arange(i0, i1), n - np.arange(i0, i1))
            ind2 = np.concatenate([np.arange(i, n) for i in range(i0, i1)])
            vals = np.asarray(integrand(ind1, ind2))
            off = 0
            for i in range(i0, i1):
                row = vals[off:off + n - i]
                off += n - i
                if res is None:
                    res = np.zeros((n, n), dtype=row.dtype)
                res[i, i:] = row
                res[i:, i] = row
        return res
    for i in range(n):
        row = np.asarray(integrand(np.full(n - i, i), np.arange(i, n)))
        if res is None:
            res = np.zeros((n, n), dtype=row.dtype)
        res[i, i:] = row
        res[i:, i] = row
    return res if res is not None else np.zeros((0, 0))

