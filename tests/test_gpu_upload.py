"""The drop-in thin's upload path (round 4): the standardised, page-locked host arrays go to the device
asynchronously while the 'med' preconditioner is computed on the host (thinning._early_upload), and the
integrand waits for the copy before it is handed out, so it is safe to use from any stream."""
import numpy as np
import pytest

from oracle import stein_numpy as o

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import thinning as st  # noqa: E402


def _data(n=30_000, d=4, seed=5):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d)) * np.linspace(0.5, 2, d)
    g = -x / np.linspace(0.5, 2, d) ** 2 + 0.1 * rng.normal(size=(n, d))
    return x, g


def test_med_integrand_uploads_early_and_works_on_another_stream():
    x, g = _data()
    integ = st._make_stein_integrand(x, g, preconditioner='med')
    prob = integ._problem
    assert prob is not None and prob._upload_event is None       # uploaded early, and waited for
    want = o.thin(x, g, 40, preconditioner='med')
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        got = integ.device_problem().greedy(40)
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(st.thin(x, g, 40, preconditioner='med'), want)


def test_gf_med_integrand_uploads_weights_early():
    x, g = _data(seed=6)
    log_p = -0.5 * np.sum(x * x, axis=1)
    log_q = -0.45 * np.sum(x * x, axis=1)
    integ = st._make_stein_gf_integrand(x, log_p, log_q, g, preconditioner='med')
    assert integ._problem is not None and integ._problem.w is not None
    np.testing.assert_array_equal(integ.device_problem().greedy(30),
                                  o.thin_gf(x, log_p, log_q, g, 30, preconditioner='med'))


@pytest.mark.parametrize('d', [2, 3, 4, 8])
def test_device_standardisation_bit_identical(d):
    """n >= 65536, d <= 8: the raw arrays go up while the host computes loc / scl
    (st_standardize_upload) and the device applies x / scl, g * scl (st_layout_soa_scaled): the
    device arrays, the 'med' preconditioner and the deferred host arrays are bit-identical to the
    host route's, and the integrand is handed out with its upload finished."""
    n = 100_003
    x, g = _data(n=n, d=d, seed=d)
    integ = st._make_stein_integrand(x, g, preconditioner='med')
    prob = integ._problem
    assert prob is not None and prob._upload_event is None and prob._raw is None
    assert integ._sample is None                     # host arrays deferred
    s, gs = st._validate_and_standardize(x, g, True)
    assert np.array_equal(prob.x[:, :n].cpu().numpy().T, s)
    assert np.array_equal(prob.g[:, :n].cpu().numpy().T, gs)
    assert not prob.x[:, n:].any() and not prob.g[:, n:].any()
    from stein_thinning.kernel import make_precon
    assert np.array_equal(integ.linv, make_precon(s, 'med'))
    assert np.array_equal(integ.sample, s) and np.array_equal(integ.gradient, gs)
    np.testing.assert_array_equal(integ.device_problem().greedy(25), o.thin(x, g, 25, preconditioner='med'))


def test_device_standardisation_gradient_free():
    n = 70_001
    x, g = _data(n=n, seed=8)
    log_p = -0.5 * np.sum(x * x, axis=1)
    log_q = -0.45 * np.sum(x * x, axis=1)
    integ = st._make_stein_gf_integrand(x, log_p, log_q, g, preconditioner='med')
    assert integ._sample is None and integ._problem.w is not None
    w = np.exp(st._log_weights(log_p, log_q, None))
    assert np.array_equal(integ._problem.w[:n].cpu().numpy(), w)
    np.testing.assert_array_equal(integ.device_problem().greedy(20),
                                  o.thin_gf(x, log_p, log_q, g, 20, preconditioner='med'))


def test_device_standardisation_errors():
    """The reference's ValueErrors, NaN before inf, as _validate_and_standardize raises them."""
    n = 70_000
    x, g = _data(n=n)
    cases = []
    a, b = x.copy(), g.copy(); a[5, 1] = np.nan; cases.append((a, b, 'NaNs'))
    a, b = x.copy(), g.copy(); b[n - 1, 3] = np.inf; cases.append((a, b, 'infs'))
    a, b = x.copy(), g.copy(); a[7, 0] = -np.inf; b[60_000, 2] = np.nan; cases.append((a, b, 'NaNs'))
    a, b = x.copy(), g.copy(); a[:, 2] = 1.5; cases.append((a, b, 'Too few unique samples'))
    for a, b, msg in cases:
        with pytest.raises(ValueError, match=msg):
            st._make_stein_integrand(a, b, preconditioner='med')
        with pytest.raises(ValueError, match=msg):
            st._validate_and_standardize(a, b, True)


def test_device_standardisation_input_kinds():
    """The device route takes what _validate_and_standardize takes: float32 arrays, Fortran-ordered
    arrays and torch tensors (CPU or on the GPU) give the float64 NumPy route's indices."""
    n = 70_001
    x, g = _data(n=n, seed=11)
    want = st.thin(x, g, 15, preconditioner='med')
    np.testing.assert_array_equal(want, o.thin(x, g, 15, preconditioner='med'))
    x32, g32 = x.astype(np.float32), g.astype(np.float32)
    np.testing.assert_array_equal(st.thin(x32, g32, 15, preconditioner='med'),
                                  o.thin(x32.astype(np.float64), g32.astype(np.float64), 15, preconditioner='med'))
    np.testing.assert_array_equal(st.thin(np.asfortranarray(x), np.asfortranarray(g), 15, preconditioner='med'), want)
    np.testing.assert_array_equal(st.thin(torch.from_numpy(x), torch.from_numpy(g), 15, preconditioner='med'), want)
    np.testing.assert_array_equal(st.thin(torch.from_numpy(x).cuda(), torch.from_numpy(g).cuda(), 15,
                                          preconditioner='med'), want)
