"""Pin the CPU oracle (oracle/stein_numpy.py) to the reference's own golden outputs.

F1: Gradient_free_Stein_thinning.ipynb printed index vectors; F2: Gaussian_mixture.ipynb printed
moments / unique counts / energy distances / Laplace collapse; F3: the vector curves of
report/figures/gaussian-mixture-comparison.pdf (tests/golden/extract_pdf_curves.py); F4: the kmat
extreme value; F5: code/tests/test_ksd.py (kmat protocol).
"""
import warnings

import numpy as np
import pytest
from scipy.stats import multivariate_normal as mvn

from oracle import models
from oracle import stein_numpy as o

# the PDF stores 6-decimal point coordinates on a log axis of ~135 pt/decade: <= ~2e-8 relative
CURVE_RTOL = 1e-7


@pytest.fixture(scope='module')
def biv():
    return models.bivariate_reference_sample(1000)


def test_f1a_thin(biv, golden):
    sample, gradient, _, _, _ = biv
    idx = o.thin(sample, gradient, 20)
    assert idx.dtype == np.uint32
    np.testing.assert_array_equal(idx, golden['F1a_thin_bivariate_m20']['indices'])


def test_f1b_gf_with_true_density_equals_thin(biv):
    sample, gradient, log_p, _, _ = biv
    np.testing.assert_array_equal(o.thin_gf(sample, log_p, log_p, gradient, 20), o.thin(sample, gradient, 20))


def test_f1c_gf_simple_gaussian(biv, golden):
    sample, _, log_p, _, _ = biv
    log_q, gq, mean, cov = models.gaussian_proxy(sample, ddof=2)
    f = golden['F1c_thin_gf_simple_gaussian_ddof2']
    np.testing.assert_allclose(mean, f['sample_mean'], atol=5e-9)
    np.testing.assert_allclose(cov, f['sample_cov'], atol=5e-9)
    np.testing.assert_array_equal(o.thin_gf(sample, log_p, log_q, gq, 20), f['indices'])


@pytest.fixture(scope='module')
def gm_runs(gm):
    sample, sample2, logpdf, score = gm
    gradient = score(sample)
    log_p = logpdf(sample)
    log_q, gq, mean, cov = models.gaussian_proxy(sample, ddof=1)
    idx_st = o.thin(sample, gradient, 1000, preconditioner='med')
    idx_gf = o.thin_gf(sample, log_p, log_q, gq, 1000, preconditioner='med')
    return dict(sample=sample, sample2=sample2, gradient=gradient, log_p=log_p, log_q=log_q, gq=gq,
                mean=mean, cov=cov, idx_st=idx_st, idx_gf=idx_gf)


def test_f2_moments_and_unique_counts(gm_runs, golden):
    f = golden['F2_gaussian_mixture']
    np.testing.assert_allclose(gm_runs['mean'], f['sample_mean'], atol=5e-9)
    np.testing.assert_allclose(gm_runs['cov'], f['sample_cov'], atol=5e-9)
    assert len(np.unique(gm_runs['idx_st'])) == f['unique_counts']['stein']
    assert len(np.unique(gm_runs['idx_gf'])) == f['unique_counts']['gf_simple_gaussian']


def test_f2_energy_distances(gm_runs, golden):
    f = golden['F2_gaussian_mixture']
    s, s2 = gm_runs['sample'], gm_runs['sample2']
    naive = np.linspace(0, 999, 40).astype(int)
    for name, idx in [('naive', naive), ('stein', gm_runs['idx_st']), ('gf_simple_gaussian', gm_runs['idx_gf'])]:
        assert round(np.sqrt(o.energy_distance(s[idx[:40]], s)), 6) == pytest.approx(f['energy_distance_vs_sample'][name], abs=1e-6)
        assert round(np.sqrt(o.energy_distance(s[idx[:40]], s2)), 6) == pytest.approx(f['energy_distance_vs_sample2'][name], abs=1e-6)


def test_f2_laplace_collapse_and_warning(gm, golden):
    sample, _, logpdf, _ = gm
    f = golden['F2_gaussian_mixture']
    lm, lc = np.array(f['laplace_mean']), np.array(f['laplace_cov'])
    log_p = logpdf(sample)
    log_q = mvn.logpdf(sample, mean=lm, cov=lc)
    gq = -np.einsum('ij,kj->ki', np.linalg.inv(lc), sample - lm)
    assert np.min((log_q - log_p) / np.log(10)) == pytest.approx(f['laplace_min_log10_ratio'], rel=1e-5)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        idx = o.thin_gf(sample, log_p, log_q, gq, 1000, preconditioner='med')
    assert any('log_q differs from log_p by more than 10' in str(x.message) for x in w)
    assert set(np.unique(idx).tolist()) == {f['laplace_all_selected']}


def test_f2_simple_gaussian_no_warning(gm_runs):
    with warnings.catch_warnings():
        warnings.simplefilter('error')
        o._make_stein_gf_integrand(gm_runs['sample'], gm_runs['log_p'], gm_runs['log_q'], gm_runs['gq'])


def test_f3_ksd_curves(gm_runs, curves):
    for name in ['stein', 'gf_simple_gaussian']:
        idx = gm_runs['idx_st'] if name == 'stein' else gm_runs['idx_gf']
        ks = o.calculate_ksd(gm_runs['sample'], gm_runs['gradient'], idx)
        c = np.array(curves['ksd/' + name])
        np.testing.assert_allclose(ks[c[:, 0].astype(int) - 1], c[:, 1], rtol=CURVE_RTOL)


def test_f3_energy_distance_curves(gm_runs, curves):
    s, s2 = gm_runs['sample'], gm_runs['sample2']
    for name in ['stein', 'gf_simple_gaussian']:
        idx = gm_runs['idx_st'] if name == 'stein' else gm_runs['idx_gf']
        c = np.array(curves['ed/' + name])[::7]
        ed = np.array([np.sqrt(o.energy_distance(s[idx[:k]], s2)) for k in c[:, 0].astype(int)])
        np.testing.assert_allclose(ed, c[:, 1], rtol=CURVE_RTOL)


def test_f3_kde_proxy_curves(gm_runs, curves):
    """The gradient-free KDE curves of report/figures/gaussian-mixture-comparison.pdf
    (Gaussian_mixture.ipynb cells 42-48: jax gaussian_kde, silverman, thin_gf with 'med', 1 000
    points) reproduced by oracle.proxy_numpy.kde_proxy (fp64) + the NumPy thin_gf: KSD and energy
    distance at the PDF's precision.  The reference evaluated the KDE in JAX's default fp32; the
    selection does not depend on the difference."""
    from oracle import proxy_numpy as op
    s, s2 = gm_runs['sample'], gm_runs['sample2']
    log_q, gq = op.kde_proxy(s, bw_method='silverman')
    idx = o.thin_gf(s, gm_runs['log_p'], log_q, gq, 1000, preconditioner='med')
    ks = o.calculate_ksd(s, gm_runs['gradient'], idx)
    c = np.array(curves['ksd/gf_kde'])
    np.testing.assert_allclose(ks[c[:, 0].astype(int) - 1], c[:, 1], rtol=CURVE_RTOL)
    c = np.array(curves['ed/gf_kde'])[::13]
    ed = np.array([np.sqrt(o.energy_distance(s[idx[:k]], s2)) for k in c[:, 0].astype(int)])
    np.testing.assert_allclose(ed, c[:, 1], rtol=CURVE_RTOL)


def test_f4_kmat_extremes(gm, golden):
    sample, _, _, _ = gm
    f = golden['F2_gaussian_mixture']
    lm, lc = np.array(f['laplace_mean']), np.array(f['laplace_cov'])
    gq = -np.einsum('ij,kj->ki', np.linalg.inv(lc), sample - lm)
    km = o.kmat(o._make_stein_integrand(sample, gq), sample.shape[0])
    v = np.abs(km[np.triu_indices_from(km)])
    # printed moments carry 8 significant digits -> compare to 1e-7 relative
    assert np.max(v) == pytest.approx(f['kmat_laplace_abs_max'], rel=1e-7)
    # the minimum is a near-cancellation: its value moves with the 8th digit of the moments
    assert np.min(v) == pytest.approx(f['kmat_laplace_abs_min'], rel=2e-2)


def test_f5_kmat_protocol(golden):
    f = golden['F5_test_ksd']
    mat = np.array(f['mat'])

    def integrand(ind1, ind2):
        return mat[ind1, ind2]
    res = o.kmat(o.reindex_integrand(integrand, np.array(f['indices'])), 5)
    np.testing.assert_array_equal(res, f['expected'])
