"""Pin the compact arithmetic of the d <= 8 kernels (oracle/stein_ref.c header, arith = 1) to the
reference's outputs: its bit model selects exactly the golden / NumPy-restatement indices on every
fixture the reference holds for the greedy loop (F1 printed index vectors, F2 1 000-step runs and the
10 000-step Laplace collapse, the KDE proxy run behind the F3 curves) and on BASELINE configs 2 and 3.
Config 4 at full length is pinned in tests/test_oracle_bitmodel.py (the bit model's default is the
compact arithmetic; the exact one is checked there too).

The compact value is a few ulps from NumPy's evaluation of vfk0_imq (JAX_Stein_Thinning.ipynb cell 27,
json ~354-361), so index parity rests on argmin margins, as it already does for NumPy itself across
CPUs (1-ulp SIMD pow differences, DESIGN.md "pow")."""
import warnings

import numpy as np
import pytest
from scipy.stats import multivariate_normal as mvn

from oracle import models
from oracle import stein_numpy as o
from tests import oracle_c


def _inputs(x, g, pre='id', log_p=None, log_q=None):
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, pre)
    w = None if log_p is None else np.exp(o._log_weights(log_p, log_q, None))
    return s, gs, w, float(linv[0, 0]), float(np.trace(linv))


def _compact(x, g, m, pre='id', log_p=None, log_q=None):
    s, gs, w, l, tr = _inputs(x, g, pre, log_p, log_q)
    assert oracle_c.compact_ok(s, gs, l, tr)
    idx, A = oracle_c.greedy_mt(s, gs, w, l, tr, m, arith='compact')
    idx_e, A_e = oracle_c.greedy_mt(s, gs, w, l, tr, m, arith='exact')
    return idx, A, idx_e, A_e


def test_compact_f1_golden_indices(golden):
    sample, gradient, log_p, _, _ = models.bivariate_reference_sample(1000)
    idx, _, _, _ = _compact(sample, gradient, 20)
    np.testing.assert_array_equal(idx, golden['F1a_thin_bivariate_m20']['indices'])
    log_q, gq, _, _ = models.gaussian_proxy(sample, ddof=2)
    idx, _, _, _ = _compact(sample, gq, 20, log_p=log_p, log_q=log_q)
    np.testing.assert_array_equal(idx, golden['F1c_thin_gf_simple_gaussian_ddof2']['indices'])


@pytest.fixture(scope='module')
def gm_inputs(gm):
    sample, _, logpdf, score = gm
    return sample, score(sample), logpdf(sample)


def test_compact_f2_gaussian_mixture_1000_steps(gm_inputs, golden):
    sample, gradient, log_p = gm_inputs
    f = golden['F2_gaussian_mixture']
    idx, A, idx_e, A_e = _compact(sample, gradient, 1000, 'med')
    np.testing.assert_array_equal(idx, o.thin(sample, gradient, 1000, preconditioner='med'))
    np.testing.assert_array_equal(idx, idx_e)
    assert len(np.unique(idx)) == f['unique_counts']['stein']
    # running sums a few ulps of the summed magnitudes from the exact arithmetic's
    assert np.max(np.abs(A - A_e) / np.maximum(np.abs(A_e), 1.0)) < 1e-12
    log_q, gq, _, _ = models.gaussian_proxy(sample, ddof=1)
    idx, _, _, _ = _compact(sample, gq, 1000, 'med', log_p, log_q)
    np.testing.assert_array_equal(idx, o.thin_gf(sample, log_p, log_q, gq, 1000, preconditioner='med'))
    assert len(np.unique(idx)) == f['unique_counts']['gf_simple_gaussian']


def test_compact_f2_laplace_collapse_10000_steps(gm_inputs, golden):
    sample, _, log_p = gm_inputs
    f = golden['F2_gaussian_mixture']
    lm, lc = np.array(f['laplace_mean']), np.array(f['laplace_cov'])
    log_q = mvn.logpdf(sample, mean=lm, cov=lc)
    gq = -np.einsum('ij,kj->ki', np.linalg.inv(lc), sample - lm)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        idx, _, _, _ = _compact(sample, gq, 10_000, 'med', log_p, log_q)
    assert set(np.unique(idx).tolist()) == {f['laplace_all_selected']}


def test_compact_kde_proxy_run(gm_inputs):
    """The gradient-free KDE run behind the report's gf_kde curves (Gaussian_mixture.ipynb cells
    42-48; pinned to the PDF in tests/test_oracle_golden.py::test_f3_kde_proxy_curves)."""
    from oracle import proxy_numpy as op
    sample, _, log_p = gm_inputs
    log_q, gq = op.kde_proxy(sample, bw_method='silverman')
    idx, _, _, _ = _compact(sample, gq, 1000, 'med', log_p, log_q)
    np.testing.assert_array_equal(idx, o.thin_gf(sample, log_p, log_q, gq, 1000, preconditioner='med'))


@pytest.mark.parametrize('gf', [False, True])
def test_compact_configs_2_3(gf):
    """BASELINE configs 2 (Langevin) and 3 (gradient-free): n = 2e5, d = 4, 'med', m = 100."""
    from bench import lv_surrogate
    x, g, log_p, (log_q, gq) = lv_surrogate(200_000, 12348 if gf else 12347)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        if gf:
            idx, _, idx_e, _ = _compact(x, gq, 100, 'med', log_p, log_q)
            want = o.thin_gf(x, log_p, log_q, gq, 100, preconditioner='med')
        else:
            idx, _, idx_e, _ = _compact(x, g, 100, 'med')
            want = o.thin(x, g, 100, preconditioner='med')
    np.testing.assert_array_equal(idx, want)
    np.testing.assert_array_equal(idx_e, want)


def test_compact_pair_values_close_to_numpy():
    """Per pair: the compact value against NumPy's vfk0_imq -- within 8 ulps of the sum of the
    magnitudes the value is built from (t1 + t2 + t3 and the sums inside t2 and t3 cancel, so it is
    the absolute error that both evaluations bound)."""
    rng = np.random.default_rng(3)
    for d in (1, 2, 4, 8):
        n = 4000
        x = rng.normal(size=(n, d)) * rng.choice([0.01, 1, 30], size=(n, 1))
        g = -x + rng.normal(size=(n, d))
        l = 0.37
        linv = l * np.eye(d)
        i1, i2 = rng.integers(0, n, size=5000), rng.integers(0, n, size=5000)
        got = oracle_c.pairs(x, g, None, l, l * d, i1, i2, arith='compact')
        want = o.vfk0_imq(x[i1], x[i2], g[i1], g[i2], linv)
        amb = (x[i1] - x[i2]).T
        qf = 1 + np.sum(l * amb * amb, axis=0)
        scale = (np.abs(3 * l * l * np.sum(amb * amb, axis=0)) / qf ** 2.5
                 + (l * d + l * np.sum(np.abs((g[i1] - g[i2]).T * amb), axis=0)) / qf ** 1.5
                 + np.sum(np.abs(g[i1] * g[i2]), axis=1) / qf ** 0.5)
        assert np.all(np.abs(got - want) <= 8 * np.spacing(scale)), d


def test_compact_applies_per_pair_in_range():
    """The rule is per pair: a row with a coordinate outside [2^-60, 2^60] (here 1e-300) makes every
    pair it is part of take the exact arithmetic (its values equal the exact model's bit for bit),
    while all other pairs stay compact; l outside the range makes every pair exact."""
    rng = np.random.default_rng(5)
    x = rng.normal(size=(500, 4))
    g = -x + 0.3 * rng.normal(size=(500, 4))
    assert oracle_c.compact_ok(x, g, 0.5, 2.0)
    x[17, 2] = 1e-300
    assert not oracle_c.compact_ok(x, g, 0.5, 2.0)
    i1 = np.repeat(np.arange(500), 3)
    i2 = np.concatenate([np.full(500, 17), rng.integers(0, 500, size=1000)])
    i2 = i2[rng.permutation(i2.size)]
    pc = oracle_c.pairs(x, g, None, 0.5, 2.0, i1, i2, arith='compact')
    pe = oracle_c.pairs(x, g, None, 0.5, 2.0, i1, i2, arith='exact')
    bad = (i1 == 17) | (i2 == 17)
    assert np.array_equal(pc[bad], pe[bad])
    assert np.any(pc[~bad] != pe[~bad])
    x[17, 2] = 0.0
    assert oracle_c.compact_ok(x, g, 0.5, 2.0) and not oracle_c.compact_ok(x, g, 2.0 ** 61, 2.0)
    ic, Ac = oracle_c.greedy(x, g, None, 2.0 ** 61, 2.0, 30, arith='compact')
    ie, Ae = oracle_c.greedy(x, g, None, 2.0 ** 61, 2.0, 30, arith='exact')
    np.testing.assert_array_equal(ic, ie)
    assert np.array_equal(Ac, Ae)
