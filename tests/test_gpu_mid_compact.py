"""Mid-size compact-only plans (round 5, csrc/persistent_cmp.hip): 512-thread blocks of 1 280 .. 4 095
rows run the compact-only persistent kernel with four / six / eight register rows per thread, where
the general kernel keeps four in registers and the rest in LDS.  The plan must not change a bit:
each run equals the general kernel's (st_tune key 12 = 0), the forced register counts and the C bit
model (oracle/stein_ref.c)."""
import numpy as np
import pytest

from oracle import stein_ref_c as oc

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import _native as nat  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402


def _run(prob, m, cmp=None):
    L = nat.lib()
    if cmp is not None:
        nat.check(L.st_tune(12, cmp), 'st_tune')
    try:
        idx, a, ws = prob.greedy_buffers(m)
        prob.greedy_launch(m, idx, a, ws)
        torch.cuda.synchronize()
        return idx.cpu().numpy().view(np.uint32).copy(), a[:prob.n].cpu().numpy().copy(), ws
    finally:
        if cmp is not None:
            L.st_tune(12, -1)


def _problem(n, d, gf, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d))
    g = -x + 0.1 * rng.normal(size=(n, d))
    if gf:
        log_p = -0.5 * np.sum(x * x, axis=1)
        log_q = -0.45 * np.sum(x * x, axis=1)
        return st._make_stein_gf_integrand(x, log_p, log_q, g, preconditioner='med')
    return st._make_stein_integrand(x, g, preconditioner='med')


@pytest.mark.parametrize('n', [340_001, 474_297, 500_000, 700_003, 950_000, 1_048_575])
@pytest.mark.parametrize('d,gf', [(4, False), (4, True), (2, False)])
def test_mid_plans_bit_identical(n, d, gf):
    integrand = _problem(n, d, gf, seed=n % 89 + d)
    prob = integrand.device_problem()
    m = 50
    idx, a, _ = _run(prob, m)
    gidx, ga, _ = _run(prob, m, cmp=0)
    np.testing.assert_array_equal(idx, gidx)
    np.testing.assert_array_equal(a, ga)
    for rt in (6, 8):
        fidx, fa, _ = _run(prob, m, cmp=rt)
        np.testing.assert_array_equal(idx, fidx)
        np.testing.assert_array_equal(a, fa)
    cidx, ca = oc.greedy_mt(integrand.sample, integrand.gradient, integrand.weights, integrand.linv_scale,
                            integrand.linv_trace, m)
    np.testing.assert_array_equal(idx, cidx)
    np.testing.assert_array_equal(a, ca)


def test_mid_plan_guarded_flags_like_the_general_kernel():
    """The guarded mid-size kernel: on twins planted in a 5e5-row problem its first flagged step
    equals the general kernel's."""
    rng = np.random.default_rng(5)
    n = 500_000
    x = rng.normal(size=(n, 4))
    g = -x + 0.1 * rng.normal(size=(n, 4))
    x[n - 1] = x[17] * (1 + 2.0 ** -52)          # a near-twin of row 17, far apart in the grid
    g[n - 1] = g[17]
    integrand = st._make_stein_integrand(x, g)
    prob = integrand.device_problem()
    idx, _, ws = _run(prob, 200)
    gidx, _, gws = _run(prob, 200, cmp=0)
    np.testing.assert_array_equal(idx, gidx)
    assert nat.near_tie_step(ws) == nat.near_tie_step(gws)
