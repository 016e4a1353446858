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
