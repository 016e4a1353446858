"""Energy distance on the GPU (K7) against the reference's printed values and the oracle
(``pytest -m gpu``).

F2: the six energy distances printed in Gaussian_mixture.ipynb (40-point prefixes of the naive,
Stein and gradient-free selections against both samples; 6 decimals).  F3: the energy-distance
curves of report/figures/gaussian-mixture-comparison.pdf (1 000 prefixes, PDF precision).
Random data: within 1e-12 relative of oracle.stein_numpy.energy_distance (scipy cdist + means).
"""
import numpy as np
import pytest

from oracle import models
from oracle import stein_numpy as o

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import energy as se  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402

CURVE_RTOL = 1.5e-8   # the oracle itself is 1.406e-8 from the PDF-extracted curve at k = 1


@pytest.fixture(scope='module')
def gm_sel(gm):
    sample, sample2, logpdf, score = gm
    gradient = score(sample)
    log_p = logpdf(sample)
    log_q, gq, _, _ = models.gaussian_proxy(sample, ddof=1)
    return dict(s=sample, s2=sample2, idx_st=st.thin(sample, gradient, 1000, preconditioner='med'),
                idx_gf=st.thin_gf(sample, log_p, log_q, gq, 1000, preconditioner='med'))


def test_f2_printed_energy_distances(gm_sel, golden):
    f = golden['F2_gaussian_mixture']
    s, s2 = gm_sel['s'], gm_sel['s2']
    naive = np.linspace(0, 999, 40).astype(int)
    for name, idx in [('naive', naive), ('stein', gm_sel['idx_st']), ('gf_simple_gaussian', gm_sel['idx_gf'])]:
        assert round(np.sqrt(se.energy_distance(s[idx[:40]], s)), 6) == pytest.approx(
            f['energy_distance_vs_sample'][name], abs=1e-6)
        assert round(np.sqrt(se.energy_distance(s[idx[:40]], s2)), 6) == pytest.approx(
            f['energy_distance_vs_sample2'][name], abs=1e-6)


def test_f3_energy_distance_curves(gm_sel, curves):
    s, s2 = gm_sel['s'], gm_sel['s2']
    for name in ['stein', 'gf_simple_gaussian']:
        idx = gm_sel['idx_st'] if name == 'stein' else gm_sel['idx_gf']
        c = np.array(curves['ed/' + name])
        got = se.energy_distance_curve(s2, s, idx, c[:, 0].astype(int))
        np.testing.assert_allclose(got, c[:, 1], rtol=CURVE_RTOL)


@pytest.mark.parametrize('d', [1, 2, 4, 9])
def test_random_against_oracle(d):
    rng = np.random.default_rng(d)
    x = rng.normal(size=(1500, d))
    y = rng.normal(size=(333, d)) * 1.3 + 0.2
    np.testing.assert_allclose(se.energy_distance(x, y), o.energy_distance(x, y), rtol=1e-12)
    sizes = np.array([1, 2, 17, 100, 333])
    idx = np.arange(333)
    want = [np.sqrt(o.energy_distance(x, y[:k])) for k in sizes]
    np.testing.assert_allclose(se.energy_distance_curve(x, y, idx, sizes), want, rtol=1e-10)


def test_one_dimensional_input_and_errors():
    rng = np.random.default_rng(0)
    x, y = rng.normal(size=300), rng.normal(size=100) + 0.5
    np.testing.assert_allclose(se.energy_distance(x, y), o.energy_distance(x[:, None], y[:, None]), rtol=1e-12)
    with pytest.raises(ValueError):
        se.energy_distance(np.zeros((3, 2)), np.zeros((3, 3)))
    with pytest.raises(ValueError):
        se.energy_distance_curve(x, y, np.arange(100), [101])


@pytest.mark.parametrize('d', [3, 4, 11])
def test_chunked_ranges_against_oracle(d):
    """A short A against a long B (the selection against the validation sample) and a long
    triangle: both split over blockIdx.y chunks of B with the workspace reduction; the same value
    as the oracle, and the chunked column sums equal the unsplit kernel's to rounding."""
    from stein_thinning import _native as nat
    rng = np.random.default_rng(d + 40)
    x = rng.normal(size=(6011, d))
    y = rng.normal(size=(301, d)) * 0.7 + 0.1
    assert nat.lib().st_distance_workspace_bytes(301, 0, 6011) > 0
    np.testing.assert_allclose(se.energy_distance(x, y), o.energy_distance(x, y), rtol=1e-12)
    sizes = np.array([1, 5, 150, 301])
    want = [np.sqrt(o.energy_distance(x, y[:k])) for k in sizes]
    np.testing.assert_allclose(se.energy_distance_curve(x, y, np.arange(301), sizes), want, rtol=1e-10)
    dev = torch.device('cuda', 0)
    ys, ny, _, ldy = se._soa(y, dev)
    xs, nx, _, ldx = se._soa(x, dev)
    split = se._colsum(ys, ny, ldy, xs, nx, ldx, d, 0, nx, False, dev)
    whole = torch.zeros(ny, dtype=torch.float64, device=dev)
    nat.check(nat.lib().st_distance_colsum(nat.ptr(ys), ldy, ny, nat.ptr(xs), ldx, nx, d, 0, nx, 0, nat.ptr(whole),
                                           nat.stream_handle()), 'st_distance_colsum')
    np.testing.assert_allclose(split, whole.cpu().numpy(), rtol=1e-13)
