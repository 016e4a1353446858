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


def _single_phase(th, data, rtol=lv.RTOL, atol=lv.ATOL):
    """st_lv_grad_log_posterior: the one-kernel path (each thread integrates and evaluates)."""
    from stein_thinning import _native as nat
    th = np.ascontiguousarray(th, dtype=np.float64)
    t, y, s = lv._settings(data, rtol, atol)
    cinv = np.ascontiguousarray(np.linalg.inv(np.asarray(data.cov, dtype=np.float64)))
    dev = nat.require_device()
    n = th.shape[0]
    out = torch.empty((n, 4), dtype=torch.float64, device=dev)
    status = torch.zeros(n, dtype=torch.int32, device=dev)
    thd, td, yd = (torch.from_numpy(a).to(dev) for a in (th, t, y))
    nat.check(nat.lib().st_lv_grad_log_posterior(
        nat.ptr(thd), n, nat.ptr(td), t.size, nat.ptr(yd), s.ctypes.data, cinv.ctypes.data, lv.MAX_STEPS,
        nat.ptr(out), nat.ptr(status), nat.stream_handle()), 'st_lv_grad_log_posterior')
    assert int((status != 0).sum()) == 0
    return out.cpu().numpy()


def test_two_phase_matches_single_phase(data):
    """The two-phase gradient (recorded steps, one wave per point) reassociates only the dense
    output and the sum over observation points: same step sequence, values to ~1e-13."""
    th = _thetas()
    got = lv.grad_log_posterior(th, data)
    want = _single_phase(th, data)
    err = np.abs(got - want) / np.abs(want).max(axis=1, keepdims=True)
    print('max rel diff', err.max())
    assert err.max() < 1e-11


def test_two_phase_step_table_overflow_falls_back(data):
    """rtol 1e-9 needs far more than the 64 recorded steps per point: every point overflows the
    step table and is recomputed by the single-phase kernel -- bitwise its result."""
    th = _points(70, 0.05, 6)
    got = lv.grad_log_posterior(th, data, rtol=1e-9, atol=1e-12)
    want = _single_phase(th, data, rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(got, want)


def test_two_phase_chunks(data):
    th = _points(50, 0.05, 7)
    np.testing.assert_array_equal(lv.grad_log_posterior(th, data, chunk=7), lv.grad_log_posterior(th, data))


@pytest.mark.parametrize('pieces', [1, 2, 3])
def test_phase_b_pieces_per_lane(data, pieces):
    """st_tune key 18: 1, 2 or 3 observation pieces per lane in phase B only regroup the per-point
    sum (pieces, then the wave tree): against scipy within RTOL and against the single-phase kernel
    within 1e-11, like the default."""
    from stein_thinning import _native as nat
    L = nat.lib()
    assert L.st_tune(18, pieces) == 0
    try:
        th = _thetas()
        got = lv.grad_log_posterior(th, data)
    finally:
        L.st_tune(18, -1)
    want = _single_phase(th, data)
    err = np.abs(got - want) / np.abs(want).max(axis=1, keepdims=True)
    assert err.max() < 1e-11, err.max()
    ref = np.stack([ol.grad_log_posterior(t, data.t, data.y, data.cov) for t in th[:12]])
    assert (np.abs(got[:12] - ref) / np.abs(ref).max(axis=1, keepdims=True)).max() < RTOL


@pytest.mark.parametrize('t_n', [2643, 2644, 2700, 2731, 4000])
def test_phase_b_observation_count_at_the_lds_boundary(data, t_n):
    """Phase B stages the observations in LDS when 3 t_n doubles fit next to its static LDS in 64 KB
    (t_n <= 2643), else reads them from global memory (the static part is counted); either
    side of the boundary agrees with the single-phase kernel."""
    t = np.linspace(0.0, 25.0, t_n)
    y = np.stack([np.interp(t, data.t, data.y[:, 0]), np.interp(t, data.t, data.y[:, 1])], axis=1)
    custom = lv.LvData(t=t, y=y)
    th = _points(24, 0.05, 11)
    got = lv.grad_log_posterior(th, custom)
    want = _single_phase(th, custom)
    err = np.abs(got - want) / np.abs(want).max(axis=1, keepdims=True)
    assert err.max() < 1e-11, err.max()
