"""``stein_thinning.kernel`` -- IMQ Stein kernel and preconditioners.

Mirrors the reference dependency's module (imported at
``code/notebooks/Kernel_Stein_discrepancy.ipynb`` cell 2 and ``JAX_Stein_Thinning.ipynb`` cells 15,
26): ``vfk0_imq(a, b, sa, sb, linv)``, ``make_imq(sample, preconditioner)``,
``make_precon(sample, preconditioner)``.  ``vfk0_imq`` evaluates on the GPU (HIP pair kernel);
the preconditioner is O(1000^2) host preprocessing exactly as the reference computes it.
"""
from __future__ import annotations

from typing import Callable

import numpy as np
from numpy.linalg import inv
from scipy.spatial.distance import pdist

MED_SUBSAMPLE = 1000


def make_precon(sample: np.ndarray, preconditioner='id') -> np.ndarray:
    """Gamma^-1 for the IMQ kernel (reference usage: ``make_precon(s, 'id')``,
    ``JAX_Stein_Thinning.ipynb`` cell 28; median heuristic ``report.tex:432``).

    'id' -> I; 'med' -> inv(med^2 I), med = median pairwise distance of the (standardised) sample,
    sub-sampled at ``linspace(0, n-1, 1000)`` rows when n > 1000 (sub-sampling rule: parity
    unpinned); 'sclmed' -> inv(med^2 / log(min(1000, n)) I); a number s -> inv(s I).
    """
    sample = np.asarray(sample, dtype=np.float64)
    n, d = sample.shape

    def med2():
        sub = sample[np.linspace(0, n - 1, MED_SUBSAMPLE, dtype=int)] if n > MED_SUBSAMPLE else sample
        return np.median(pdist(sub)) ** 2

    if isinstance(preconditioner, str):
        if preconditioner == 'id':
            return np.identity(d)
        if preconditioner == 'med':
            m2 = med2()
            if m2 == 0:
                raise ValueError('Too few unique samples in smp.')
            return inv(m2 * np.identity(d))
        if preconditioner == 'sclmed':
            m2 = med2()
            if m2 == 0:
                raise ValueError('Too few unique samples in smp.')
            return inv(m2 / np.log(np.minimum(MED_SUBSAMPLE, n)) * np.identity(d))
    try:
        scale = float(preconditioner)
    except (TypeError, ValueError):
        raise ValueError('Incorrect preconditioner type.') from None
    return inv(scale * np.identity(d))


def vfk0_imq(a: np.ndarray, b: np.ndarray, sa: np.ndarray, sb: np.ndarray, linv: np.ndarray) -> np.ndarray:
    """IMQ Langevin Stein kernel k_P(a_i, b_i) (c = 1, beta = -1/2), evaluated by the HIP pair kernel.

    Same broadcasting as the reference (row-wise pairs; either side may have a single row).
    Only isotropic preconditioners (linv = l I: 'id', 'med', 'sclmed', scalar) run on the engine.
    """
    from .device import DeviceProblem, isotropic_scale
    a = np.atleast_2d(np.asarray(a, dtype=np.float64))
    b = np.atleast_2d(np.asarray(b, dtype=np.float64))
    sa = np.atleast_2d(np.asarray(sa, dtype=np.float64))
    sb = np.atleast_2d(np.asarray(sb, dtype=np.float64))
    if a.shape != sa.shape or b.shape != sb.shape or a.shape[1] != b.shape[1]:
        raise ValueError('inconsistent shapes for vfk0_imq')
    iso = isotropic_scale(linv)
    if iso is None:
        raise NotImplementedError('vfk0_imq on the HIP engine supports isotropic preconditioners only')
    na, nb = a.shape[0], b.shape[0]
    ia, ib = np.broadcast_arrays(np.arange(na), np.arange(nb))
    prob = DeviceProblem(np.vstack([a, b]), np.vstack([sa, sb]), None, iso[0], iso[1])
    return prob.pairs(ia.astype(np.int64), ib.astype(np.int64) + na)


def make_imq(sample: np.ndarray, preconditioner='id') -> Callable:
    linv = make_precon(sample, preconditioner)

    def vfk0(a, b, sa, sb):
        return vfk0_imq(a, b, sa, sb, linv)
    vfk0.linv = linv
    return vfk0
