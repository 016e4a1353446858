"""ctypes loader for the C bit-model oracle (oracle/stein_ref.c) -- TEST INFRASTRUCTURE ONLY.

Loaded by tests/ (as the checker), __graft_entry__.smoke() and bench.py's cpu_baseline leg (the
threaded port timed on the host cores); never by the product package."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'oracle', '_build', 'libstein_ref.so')   # built by __graft_entry__.build()
SRC = os.path.join(ROOT, 'oracle', 'stein_ref.c')
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
            os.makedirs(os.path.dirname(LIB), exist_ok=True)
            subprocess.run(['gcc', '-O2', '-fPIC', '-shared', '-ffp-contract=off', '-pthread', '-o', LIB, SRC, '-lm'],
                           check=True)
        L = ctypes.CDLL(LIB)
        dp, i64 = ctypes.c_void_p, ctypes.c_int64
        L.sr_greedy.restype = ctypes.c_int
        L.sr_greedy.argtypes = [dp, dp, dp, i64, ctypes.c_int, ctypes.c_double, ctypes.c_double, i64, dp, dp,
                                ctypes.c_int]
        L.sr_greedy_mt.restype = ctypes.c_int
        L.sr_greedy_mt.argtypes = [dp, dp, dp, i64, ctypes.c_int, ctypes.c_double, ctypes.c_double, i64, dp, dp,
                                   ctypes.c_int, ctypes.c_int]
        L.sr_greedy_mt_ties.restype = ctypes.c_int
        L.sr_greedy_mt_ties.argtypes = [dp, dp, dp, i64, ctypes.c_int, ctypes.c_double, ctypes.c_double, i64, dp,
                                        dp, ctypes.c_int, ctypes.c_int, dp, dp, dp]
        L.sr_tie_bounds.restype = None
        L.sr_tie_bounds.argtypes = [dp, dp, i64, ctypes.c_int, dp, dp]
        L.sr_pow_15_25.restype = None
        L.sr_pow_15_25.argtypes = [dp, i64, dp, dp]
        L.sr_pairs.restype = ctypes.c_int
        L.sr_pairs.argtypes = [dp, dp, dp, i64, ctypes.c_int, ctypes.c_double, ctypes.c_double, dp, dp, i64, dp,
                               ctypes.c_int]
        L.sr_compact_ok.restype = ctypes.c_int
        L.sr_compact_ok.argtypes = [dp, dp, i64, ctypes.c_int, ctypes.c_double, ctypes.c_double]
        _lib = L
    return _lib


# arithmetic of the kernels' bit model: 'exact' = NumPy's evaluation order rounding for rounding,
# 'compact' = the regrouped form (stein_ref.c header) the d <= 8 kernels use by default
ARITH = {'exact': 0, 'compact': 1}
DEFAULT_ARITH = 'compact'


def _a(arith):
    return ARITH[arith or DEFAULT_ARITH]


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def greedy(x, g, w, l, tr, m, arith=None):
    """Bit-model greedy run: returns (idx uint32, running sums A)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.float64)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    n, d = x.shape
    idx = np.empty(m, dtype=np.uint32)
    A = np.empty(n, dtype=np.float64)
    rc = lib().sr_greedy(_p(x), _p(g), _p(w), n, d, l, tr, m, _p(idx), _p(A), _a(arith))
    assert rc == 0
    return idx, A


def host_threads():
    """Threads for the checker: the box's CPU share (OMP_NUM_THREADS is 16 on the GPU box, while
    os.cpu_count() there reports the whole machine)."""
    return max(1, min(int(os.environ.get('OMP_NUM_THREADS', 0)) or (os.cpu_count() or 1), 16))


def greedy_mt(x, g, w, l, tr, m, nthreads=None, arith=None):
    """sr_greedy over row blocks on host threads: same indices and bit-identical A as greedy()."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.float64)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    n, d = x.shape
    idx = np.empty(m, dtype=np.uint32)
    A = np.empty(n, dtype=np.float64)
    rc = lib().sr_greedy_mt(_p(x), _p(g), _p(w), n, d, l, tr, m, _p(idx), _p(A), nthreads or host_threads(),
                            _a(arith))
    assert rc == 0
    return idx, A


def tie_bounds(g, w):
    """(max_i |g_i|^2, max_i w_i^2) as the kernels compute them for the near-tie threshold."""
    g = np.ascontiguousarray(g, dtype=np.float64)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    g2, w2 = ctypes.c_double(), ctypes.c_double()
    lib().sr_tie_bounds(_p(g), _p(w), g.shape[0], g.shape[1], ctypes.byref(g2), ctypes.byref(w2))
    return g2.value, w2.value


def greedy_ties(x, g, w, l, tr, m, nthreads=None, arith=None, winner_sums=False):
    """greedy_mt plus the kernels' near-tie guard model (stein_ref.c sr_greedy_mt_ties): (idx, A, gap, thr,
    flagged) where gap[t] = the smallest running sum of any row other than the step-t winner and its bitwise
    duplicates minus the winner's (other exact ties count: 0), thr[t] the guard's threshold and
    flagged[t] = gap[t] <= thr[t] (only
    with the compact arithmetic, d <= 8).  winner_sums=True appends wv[t], the step-t winner's sum."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.float64)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    n, d = x.shape
    idx = np.empty(m, dtype=np.uint32)
    A = np.empty(n, dtype=np.float64)
    gap, thr, wv = (np.empty(m, dtype=np.float64) for _ in range(3))
    rc = lib().sr_greedy_mt_ties(_p(x), _p(g), _p(w), n, d, l, tr, m, _p(idx), _p(A), nthreads or host_threads(),
                                 _a(arith), _p(gap), _p(thr), _p(wv))
    assert rc == 0
    with np.errstate(invalid='ignore'):
        flagged = (gap <= thr) & (_a(arith) == 1) & (d <= 8)
    if winner_sums:
        return idx, A, gap, thr, flagged, wv
    return idx, A, gap, thr, flagged


def pairs(x, g, w, l, tr, i1, i2, arith=None):
    x = np.ascontiguousarray(x, dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.float64)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    i1 = np.ascontiguousarray(i1, dtype=np.int64)
    i2 = np.ascontiguousarray(i2, dtype=np.int64)
    out = np.empty(i1.shape[0], dtype=np.float64)
    rc = lib().sr_pairs(_p(x), _p(g), _p(w), x.shape[0], x.shape[1], l, tr, _p(i1), _p(i2), i1.shape[0], _p(out), _a(arith))
    assert rc == 0
    return out


def compact_ok(x, g, l, tr):
    """1 if the compact arithmetic applies (every coordinate 0 or in [2^-60, 2^60], l and tr in range)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    g = np.ascontiguousarray(g, dtype=np.float64)
    return bool(lib().sr_compact_ok(_p(x), _p(g), x.shape[0], x.shape[1], l, tr))


def pow_15_25(q):
    q = np.ascontiguousarray(q, dtype=np.float64)
    p15, p25 = np.empty_like(q), np.empty_like(q)
    lib().sr_pow_15_25(_p(q), q.shape[0], _p(p15), _p(p25))
    return p15, p25
