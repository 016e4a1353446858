"""Small-shard plans (round 5, csrc/persistent_small.hip): blocks of at most 256 / 512 rows run the
256-thread persistent kernel with ONE / TWO register rows per thread instead of four.  The selection
and the running sums must not depend on the plan: each run is compared bit for bit with the same thin
forced onto four register rows (st_tune key 3) and with the C bit model (oracle/stein_ref.c)."""
import numpy as np
import pytest

from oracle import stein_ref_c as oc

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import _native as nat  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402


def _run(prob, m, rt=None):
    if rt is not None:
        nat.check(nat.lib().st_tune(3, rt), 'st_tune')
    try:
        idx, a, ws = prob.greedy_buffers(m)
        prob.greedy_launch(m, idx, a, ws)
        torch.cuda.synchronize()
        return idx.cpu().numpy().view(np.uint32).copy(), a[:prob.n].cpu().numpy().copy()
    finally:
        if rt is not None:
            nat.check(nat.lib().st_tune(3, -1), 'st_tune')


def _problem(n, d, gf, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d))
    g = -x + 0.1 * rng.normal(size=(n, d))
    if gf:
        log_p = -0.5 * np.sum(x * x, axis=1)
        log_q = -0.45 * np.sum(x * x, axis=1)
        return st._make_stein_gf_integrand(x, log_p, log_q, g, preconditioner='med')
    return st._make_stein_integrand(x, g, preconditioner='med')


@pytest.mark.parametrize('n', [3000, 47_279, 65_536, 65_537, 100_003, 131_072])
@pytest.mark.parametrize('d,gf', [(4, False), (4, True), (2, False)])
@pytest.mark.parametrize('arith', ['compact', 'exact'])
def test_small_plans_bit_identical(n, d, gf, arith):
    with nat.arithmetic_override(arith):
        integrand = _problem(n, d, gf, seed=n % 97 + d)
        prob = integrand.device_problem()
        m = 60
        idx, a = _run(prob, m)
        idx4, a4 = _run(prob, m, rt=4)
        np.testing.assert_array_equal(idx, idx4)
        np.testing.assert_array_equal(a, a4)
        cidx, ca = oc.greedy_mt(integrand.sample, integrand.gradient, integrand.weights, integrand.linv_scale,
                                integrand.linv_trace, m, arith=arith)
        np.testing.assert_array_equal(idx, cidx)
        np.testing.assert_array_equal(a, ca)


def test_small_plan_guarded_flags_like_the_model():
    """The guarded small-shard kernel: its first flagged step equals the model's on the near-tie twins."""
    from tests import margins_ref as mr
    X, G, steps = mr.near_tie_twins(2)
    integrand = st._make_stein_integrand(X, G)
    prob = integrand.device_problem()
    idx, a, ws = prob.greedy_buffers(30)
    prob.greedy_launch(30, idx, a, ws)
    assert nat.near_tie_step(ws) == steps[0]
