"""The reference's plug-in pattern on the GPU (F6, ``JAX_Stein_Thinning.ipynb`` cells 4-19, json
~201-244): a user-written integrand closure over ``make_imq(s, 'id')`` driven by ``_greedy_search``
must select what ``thin`` selects (the notebook's own ``np.testing.assert_array_equal(idx2, idx)``),
with the shim's ``vfk0`` keeping the n-row operand resident (one row uploaded per step)."""
import time

import numpy as np
import pytest
from scipy.stats import multivariate_normal as mvn

from oracle import stein_numpy as o

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import kernel as sk  # noqa: E402
from stein_thinning.kernel import make_imq  # noqa: E402
from stein_thinning.thinning import _greedy_search, _validate_and_standardize, thin  # noqa: E402


@pytest.fixture(scope='module')
def notebook_sample():
    """JAX_Stein_Thinning.ipynb cells 4-7: seed 12345, N(0, [[1, .8], [.8, 1]]), n_max = 5e6 draws, the
    first n = 1e5 used."""
    rng = np.random.default_rng(12345)
    mean = np.array([0., 0.])
    cov = np.array([[1., 0.8], [0.8, 1.]])
    sample = mvn.rvs(mean=mean, cov=cov, size=5_000_000, random_state=rng)
    grad = (np.linalg.inv(cov) @ (mean - sample).T).T
    n = 100_000
    return sample[:n].copy(), grad[:n].copy()


def test_f6_plugin_closure_equals_thin(notebook_sample):
    x, grad = notebook_sample
    m = 100
    idx = thin(x, grad, m)                                   # cell 10
    np.testing.assert_array_equal(idx, o.thin(x, grad, m))
    s, g = _validate_and_standardize(x, grad, True)          # cell 16
    vfk0 = make_imq(s, 'id')

    def integrand(ind1, ind2):                               # cell 17
        return vfk0(s[ind1], s[ind2], g[ind1], g[ind2])
    _greedy_search(3, integrand)                             # warm: the operand becomes resident
    t0 = time.perf_counter()
    idx2 = _greedy_search(m, integrand)                      # cell 18
    per_step = (time.perf_counter() - t0) / m
    np.testing.assert_array_equal(idx2, idx)                 # cell 19
    assert per_step < 1e-3, f'{per_step * 1e3:.3f} ms per plug-in step'
    # the same with a fresh make_imq closure inside every call: the resident rows are shared
    idx3 = _greedy_search(m, lambda i1, i2: make_imq(s, 'id')(s[i1], s[i2], g[i1], g[i2]))
    np.testing.assert_array_equal(idx3, idx)


def test_vfk0_resident_rows_follow_in_place_changes(notebook_sample):
    """A resident operand is re-validated on every call: changing the caller's array in place gives
    the new values, never a stale device copy; pair values equal the oracle's to the bit-model
    tolerance of the pow rounding (1e-12)."""
    x, grad = notebook_sample
    s, g = _validate_and_standardize(x[:20_000], grad[:20_000], True)
    s, g = s.copy(), g.copy()
    linv = np.identity(2) * 0.7
    for step in range(3):
        j = [7 + step]
        got = sk.vfk0_imq(s, s[j], g, g[j], linv)
        want = o.vfk0_imq(s, s[j], g, g[j], linv)
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12 * np.max(np.abs(want)))
        got_r = sk.vfk0_imq(s[j], s, g[j], g, linv)         # the single row on the left
        np.testing.assert_array_equal(got_r, got)
        diag = sk.vfk0_imq(s, s, g, g, linv)
        np.testing.assert_allclose(diag, o.vfk0_imq(s, s, g, g, linv), rtol=1e-12)
        s[100 * step:100 * step + 50] += 0.25                 # in place: must be seen next call
