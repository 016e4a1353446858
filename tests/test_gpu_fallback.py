"""Persistent greedy kernel next to other work on the device.

The persistent kernel needs its whole grid co-resident (every block waits for every other block's
record each step) but is launched with a plain launch after an occupancy query
(csrc/persistent.hip launch_p), which cannot see kernels on other streams.  A grid that is not
co-resident aborts at step 0 after a bounded wait and ``DeviceProblem.greedy`` re-runs the thin
on the launch-per-step kernels: the indices must still be right and the fallback reported.
"""
import ctypes
import os
import time
import warnings

import numpy as np
import pytest

from tests import oracle_c

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import thinning as st  # noqa: E402
from stein_thinning.device import DeviceProblem  # noqa: E402

HELPER = os.path.join(os.path.dirname(os.path.abspath(__file__)), '_build', 'libst_occupy.so')


def _rw(n, d, seed):
    rng = np.random.default_rng(seed)
    x = np.cumsum(rng.normal(size=(n, d)) * 0.3, axis=0) / np.sqrt(n) * 40 + rng.normal(size=(n, d))
    return x, -x


def test_persistent_grid_not_coresident_falls_back():
    n, d, m = 2_000_000, 4, 50
    x, g = _rw(n, d, 5)
    integ = st._make_stein_integrand(x, g, preconditioner='med')
    prob = integ.device_problem()
    want, want_A = prob.greedy(m, return_sums=True)
    assert prob.fallback is None
    cidx, cA = oracle_c.greedy_mt(integ.sample, integ.gradient, None, integ.linv_scale, integ.linv_trace, m)
    np.testing.assert_array_equal(want, cidx)

    lib = ctypes.CDLL(HELPER)
    lib.st_test_occupy.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1, dtype=torch.int32, device='cuda')
    # a high-priority stream: HIP gives it a hardware queue of its own (a normal-priority pool stream
    # can share the default stream's queue, which would serialise the two kernels instead)
    side = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
    # 64 CUs held for 0.4 s by blocks that take all of a CU's LDS: 64 of the persistent kernel's
    # one-block-per-CU grid (each ~160 KB of LDS at this n) cannot start until they leave
    assert lib.st_test_occupy(64, 163840, 40_000_000, ctypes.c_void_p(sink.data_ptr()),
                              ctypes.c_void_p(side.cuda_stream)) == 0
    time.sleep(0.05)
    t0 = time.perf_counter()
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter('always')
        idx, A = prob.greedy(m, return_sums=True)
    secs = time.perf_counter() - t0
    torch.cuda.synchronize()
    assert prob.fallback is not None, f'no fallback: the grid was co-resident ({secs:.3f} s)'
    assert any('launch-per-step' in str(w.message) for w in caught)
    np.testing.assert_array_equal(idx, want)
    assert np.array_equal(A, want_A)
    assert secs < 5.0, secs
    # the next thin on an idle device takes the persistent path again
    np.testing.assert_array_equal(prob.greedy(m), want)
    assert prob.fallback is None
