"""The 'med' preconditioner on the GPU (st_pdist + a device sort, the drop-in thin's path): every
distance bit-identical to scipy.spatial.distance.pdist, the median identical to np.median(pdist(.)),
and make_precon(..., on_device=True) identical to the host make_precon."""
import numpy as np
import pytest
from scipy.spatial.distance import pdist

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import _native as nat  # noqa: E402
from stein_thinning.device import pdist_median  # noqa: E402
from stein_thinning.kernel import make_precon  # noqa: E402


@pytest.mark.parametrize('k,d', [(2, 1), (3, 4), (1000, 4), (1001, 2), (777, 8), (300, 50), (64, 128)])
def test_pdist_bit_identical_to_scipy(k, d):
    rng = np.random.default_rng(k * 131 + d)
    rows = rng.normal(size=(k, d)) * rng.uniform(0.01, 100.0, size=d)
    rows[k // 2] = rows[0]                      # a zero distance
    t = torch.from_numpy(rows).cuda()
    out = torch.empty(k * (k - 1) // 2, dtype=torch.float64, device='cuda')
    nat.check(nat.lib().st_pdist(nat.ptr(t), k, d, nat.ptr(out), nat.stream_handle()), 'st_pdist')
    got = out.cpu().numpy()
    want = pdist(rows)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), np.flatnonzero(got != want)[:10]


@pytest.mark.parametrize('k', [2, 3, 4, 999, 1000])
def test_pdist_median_equals_numpy(k):
    rng = np.random.default_rng(k)
    sub = rng.normal(size=(k, 4))
    sub[1:k // 3] = sub[0]                      # many equal distances around the middle
    assert pdist_median(sub) == np.median(pdist(sub))
    assert type(pdist_median(sub)) is type(np.median(pdist(sub)))


def test_make_precon_on_device_matches_host():
    from bench import lv_surrogate
    from stein_thinning import thinning as st
    x, g, _, _ = lv_surrogate(200_000, 12347)
    s, _ = st._validate_and_standardize(x, g, True)
    for pre in ('med', 'sclmed'):
        assert np.array_equal(make_precon(s, pre, on_device=True), make_precon(s, pre)), pre
    small = s[:700]
    assert np.array_equal(make_precon(small, 'med', on_device=True), make_precon(small, 'med'))
