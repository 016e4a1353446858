"""Lotka-Volterra inputs on the GPU (csrc/lv.hip) against scipy (oracle/lv_numpy.py: the
reference module's model + the notebook's gradient on scipy's solve_ivp) and against the values of
the reference module itself (tests/golden/lv_reference.json, made by tests/golden/make_lv_golden.py).

Tolerance: scipy's RK45 takes the same steps as the kernel, but the stage combinations and dense
output are BLAS dot products whose summation order differs, so values agree to rounding amplified
by the integration (rtol 1e-8 here); a step-size decision that falls the other way on a last-bit
difference would show as a ~1e-4 discrepancy and fail the test."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from oracle import lv_numpy as ol  # noqa: E402
from stein_thinning import lotka_volterra as lv  # noqa: E402

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'lv_reference.json')))
RTOL = 1e-8   # observed: 1.7e-10 (gradient), 6.7e-10 (log density) on MI355X


@pytest.fixture(scope='module')
def data():
    return lv.reference_data()


def _points(n, scale, seed):
    rng = np.random.default_rng(seed)
    base = np.log(lv.THETA)
    return np.exp(base + scale * rng.normal(size=(n, 4)))


def _thetas():
    pts = [lv.THETA[None, :], np.exp(np.array(GOLDEN['log_theta']))]
    pts += [_points(40, 0.02, 1), _points(40, 0.1, 2), _points(20, 0.4, 3)]
    return np.concatenate(pts)


def test_grad_log_posterior_matches_scipy(data):
    th = _thetas()
    got = lv.grad_log_posterior(th, data)
    want = np.stack([ol.grad_log_posterior(t, data.t, data.y, data.cov) for t in th])
    scale = np.abs(want).max(axis=1, keepdims=True)
    err = np.abs(got - want) / scale
    print('max rel err', err.max(), 'median', np.median(err))
    assert err.max() < RTOL, (np.argmax(err.max(axis=1)), err.max())


def test_log_target_density_matches_reference_module(data):
    lt = np.array(GOLDEN['log_theta'])
    got = lv.log_target_density(lt, data)
    want = np.array(GOLDEN['log_target_density'])
    np.testing.assert_allclose(got, want, rtol=RTOL)


def test_log_target_density_matches_scipy(data):
    lt = np.log(_thetas())
    got = lv.log_target_density(lt, data)
    want = np.array([ol.log_target_density(x, data.t, data.y, data.cov) for x in lt])
    err = np.abs(got - want) / np.abs(want)
    print('max rel err', err.max())
    assert err.max() < RTOL


def test_for_unique_matches_rowwise(data):
    th = _points(30, 0.05, 4)
    sample = th[np.random.default_rng(5).integers(0, 30, size=100)]
    got = lv.for_unique(lambda s: lv.grad_log_posterior(s, data), sample)
    want = lv.grad_log_posterior(sample, data)
    np.testing.assert_array_equal(got, want)


def test_single_point_and_empty(data):
    g1 = lv.grad_log_posterior(lv.THETA, data)
    assert g1.shape == (1, 4)
    assert lv.grad_log_posterior(np.zeros((0, 4)), data).shape == (0, 4)
    assert lv.log_target_density(np.zeros((0, 4)), data).shape == (0,)
