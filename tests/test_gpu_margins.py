"""Near-tie diagnostics on the GPU: DeviceProblem.greedy(m, margins=True) runs
the launch-per-step kernels one step at a time and reports every step's argmin margin against the
arithmetic's error band (stein_thinning/diagnostics.py).  Checked against the NumPy restatement over
the C bit model (tests/margins_ref.py): identical selections and margins (the kernels' running sums
are the bit model's bits), the same flagged steps, and on the near-tie construction the compact run's
departure from NumPy flagged while the exact arithmetic reproduces NumPy's indices."""
import numpy as np
import pytest

from oracle import stein_numpy as o
from tests import margins_ref as mr

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

import stein_thinning  # noqa: E402
from stein_thinning import diagnostics as dg  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402


@pytest.mark.parametrize('arith', ['compact', 'exact'])
def test_margins_match_bit_model_and_flag_the_near_tie(arith):
    X, G, steps = mr.near_tie_twins(0)
    want = o.thin(X, G, 30)
    stein_thinning.set_arithmetic(arith)
    try:
        integrand = st._make_stein_integrand(X, G)
        idx, gm = integrand.device_problem().greedy(30, margins=True)
        np.testing.assert_array_equal(idx, integrand.device_problem().greedy(30))   # same selection
    finally:
        stein_thinning.set_arithmetic('compact')
    ref = mr.margins(integrand.sample, integrand.gradient, None, integrand.linv_scale, integrand.linv_trace,
                     30, arith)
    np.testing.assert_array_equal(idx, ref['indices'])
    np.testing.assert_array_equal(gm.margin_ulps, ref['margin_ulps'])
    np.testing.assert_allclose(gm.band_ulps, ref['band_ulps'], rtol=1e-6)
    np.testing.assert_array_equal(gm.flagged, ref['flagged'])
    np.testing.assert_array_equal(gm.flagged_steps(), steps)
    if arith == 'exact':
        np.testing.assert_array_equal(idx, want)
    else:
        bad = np.flatnonzero(idx != want)
        assert bad.size and gm.flagged[bad[0]]


def test_thin_margins_gf_golden_problem_unflagged():
    from oracle import models
    sample, gradient, log_p, _, _ = models.bivariate_reference_sample(1000)
    log_q, gq, _, _ = models.gaussian_proxy(sample, 2)
    gm = dg.thin_gf_margins(sample, log_p, log_q, gq, 20, preconditioner='med')
    np.testing.assert_array_equal(gm.indices, o.thin_gf(sample, log_p, log_q, gq, 20, preconditioner='med'))
    assert not gm.flagged.any() and gm.margin_ulps.min() > 1e6
