"""CPU stand-in for HipShardBackend (test infrastructure): same candidate-record format and the same
winner / tie-break rules the HIP step kernel implements, with the C bit-model doing the arithmetic.
Lets the gloo tests drive stein_thinning.distributed.run_sharded on CPU ranks."""
import numpy as np
import torch

from tests import oracle_c

HEADER = 2


def stride(d):
    return ((HEADER + 2 * d + 1) + 1) & ~1


def _better(a, ia, b, ib):
    if np.isnan(a):
        return (not np.isnan(b)) or ia < ib
    if np.isnan(b):
        return False
    return a < b or (a == b and ia < ib)


def _bits(i):
    return np.array([i], dtype=np.int64).view(np.float64)[0]


def _unbits(v):
    return int(np.array([v], dtype=np.float64).view(np.int64)[0])


class CpuShardBackend:
    def __init__(self, s, gs, w, l, tr, r0, r1, nranks, n_points):
        self.x, self.g = s[r0:r1], gs[r0:r1]
        self.w = None if w is None else w[r0:r1]
        self.l, self.tr, self.r0, self.nranks = l, tr, r0, nranks
        self.n, self.d = self.x.shape
        self.stride = stride(self.d)
        self.send = torch.zeros(self.stride, dtype=torch.float64)
        self.recv = torch.zeros(self.stride * nranks, dtype=torch.float64)
        self.idx = np.zeros(n_points, dtype=np.uint32)
        self.A = None

    def _winner(self):
        rec = self.recv.numpy().reshape(self.nranks, self.stride)
        best = 0
        for r in range(1, self.nranks):
            if _better(rec[r, 0], _unbits(rec[r, 1]), rec[best, 0], _unbits(rec[best, 1])):
                best = r
        return _unbits(rec[best, 1]), rec[best, HEADER:]

    def step(self, t):
        from stein_thinning import _native as nat
        arith = nat.arithmetic()   # the kernels' arithmetic for this thread (an exact re-run included)
        ar = np.arange(self.n)
        if t == 0:
            A = oracle_c.pairs(self.x, self.g, None, self.l, self.tr, ar, ar, arith=arith)
            if self.w is not None:
                A = (A * self.w) * self.w
        else:
            gidx, row = self._winner()
            self.idx[t - 1] = gidx
            d = self.d
            xs = np.vstack([self.x, row[:d][None]])
            gs = np.vstack([self.g, row[d:2 * d][None]])
            col = oracle_c.pairs(xs, gs, None, self.l, self.tr, ar, np.full(self.n, self.n), arith=arith)
            if self.w is not None:
                col = (col * self.w) * row[2 * d]
            A = self.A + 2.0 * col
        self.A = A
        li = int(np.argmin(A))
        rec = np.zeros(self.stride)
        rec[0] = A[li]
        rec[1] = _bits(self.r0 + li)
        rec[HEADER:HEADER + self.d] = self.x[li]
        rec[HEADER + self.d:HEADER + 2 * self.d] = self.g[li]
        rec[HEADER + 2 * self.d] = 1.0 if self.w is None else self.w[li]
        self.send.copy_(torch.from_numpy(rec))

    def finalize(self, t):
        self.idx[t] = self._winner()[0]

    def indices(self):
        return self.idx.copy()


def from_integrand(integrand, r0, r1, nranks, n_points, mailboxes=None, rank=0):
    """Drop-in for stein_thinning.distributed.HipShardBackend(integrand, r0, r1, nranks, n_points):
    lets a gloo test run the product's thin() -> thin_across_ranks -> sharded_runner chain on CPU."""
    assert mailboxes is None
    return CpuShardBackend(integrand.sample, integrand.gradient, integrand.weights, integrand.linv_scale,
                           integrand.linv_trace, r0, r1, nranks, n_points)


class CpuKsdBackend:
    """CPU stand-in for HipKsdBackend: column sums of the lower triangle over a row range with the
    C bit model's pair values (same per-column sequential order as the HIP kernel)."""

    def __init__(self, s, gs, w, l, tr, n):
        self.s, self.gs, self.w, self.l, self.tr, self.n = s[:n], gs[:n], w, l, tr, n

    def colsum(self, a0, a1):
        c = np.zeros(self.n)
        for i in range(a0 + 1, self.n):
            a = np.arange(a0, min(i, a1))
            if a.size == 0:
                continue
            kv = oracle_c.pairs(self.s, self.gs, None, self.l, self.tr, np.full(a.size, i), a)
            if self.w is not None:
                kv = (kv * self.w[i]) * self.w[a]
            acc = 0.0
            for v in kv:
                acc += v
            c[i] = acc
        return torch.from_numpy(c)

    def finish(self, c):
        ar = np.arange(self.n)
        kd = oracle_c.pairs(self.s, self.gs, None, self.l, self.tr, ar, ar)
        if self.w is not None:
            kd = (kd * self.w[:self.n]) * self.w[:self.n]
        S = np.cumsum(2.0 * c.numpy() + kd)
        return np.sqrt(S) / (ar + 1)
