"""The C bit model (oracle/stein_ref.c) restates NumPy's evaluation order of the reference vfk0_imq.

(1) a scalar Python model with NumPy's own power() reproduces oracle.vfk0_imq bit for bit
    (sequential sums for qf/t1/t2, NumPy pairwise_sum for t3) at d = 1, 2, 4, 9, 50;
(2) the C model equals that scalar model with correctly rounded powers, bit for bit;
(3) C-model greedy indices equal the NumPy oracle's on seeded inputs.
"""
import decimal

import numpy as np
import pytest

from oracle import stein_numpy as o
from tests import oracle_c

decimal.getcontext().prec = 80


def _seq(v):
    acc = v[0]
    for x in v[1:]:
        acc = acc + x
    return acc


def _pairwise(v):
    n = len(v)
    if n < 8:
        r = np.float64(0.0)
        for x in v:
            r = r + x
        return r
    r = list(v[:8])
    i = 8
    while i < n - (n % 8):
        for j in range(8):
            r[j] = r[j] + v[i + j]
        i += 8
    res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    while i < n:
        res = res + v[i]
        i += 1
    return res


def _cr_pow(q, e):
    d = decimal.Decimal(float(q))
    v = d * d.sqrt() if e == 1.5 else d * d * d.sqrt()
    return np.float64(float(v))


def _model(xi, xj, gi, gj, l, tr, powf):
    l2 = l * l
    dl = xi - xj
    gd = gi - gj
    qf = np.float64(1.0) + _seq((l * dl) * dl)
    t1 = (-3 * _seq((l2 * dl) * dl)) / powf(qf, 2.5)
    t2 = (tr + _seq((l * gd) * dl)) / powf(qf, 1.5)
    t3 = _pairwise(gi * gj) / np.sqrt(qf)
    return (t1 + t2) + t3


def _problem(d, n=150, seed=0):
    rng = np.random.default_rng(seed + d)
    x = rng.normal(size=(n, d)) * rng.uniform(0.2, 3, size=d)
    g = rng.normal(size=(n, d)) * 2
    return x, g


@pytest.mark.parametrize('d', [1, 2, 4, 9, 50])
@pytest.mark.parametrize('pre', ['id', 'med'])
def test_scalar_model_matches_numpy_oracle(d, pre):
    x, g = _problem(d)
    linv = o.make_precon(x, pre)
    l, tr = linv[0, 0], np.trace(linv)
    j = 3
    ref = o.vfk0_imq(x, x[[j]], g, g[[j]], linv)
    got = np.array([_model(x[i], x[j], g[i], g[j], l, tr, np.power) for i in range(x.shape[0])])
    np.testing.assert_array_equal(got, ref)
    refd = o.vfk0_imq(x, x, g, g, linv)
    gotd = np.array([_model(x[i], x[i], g[i], g[i], l, tr, np.power) for i in range(x.shape[0])])
    np.testing.assert_array_equal(gotd, refd)


@pytest.mark.parametrize('d', [1, 2, 4, 9, 50])
def test_c_model_is_scalar_model_with_correct_rounding(d):
    x, g = _problem(d, n=60)
    linv = o.make_precon(x, 'med')
    l, tr = linv[0, 0], np.trace(linv)
    i1 = np.arange(60)
    i2 = np.full(60, 5)
    got = oracle_c.pairs(x, g, None, l, tr, i1, i2, arith='exact')
    want = np.array([_model(x[i], x[5], g[i], g[5], l, tr, _cr_pow) for i in i1])
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize('d,pre,gf', [(2, 'id', False), (4, 'med', False), (4, 'med', True), (9, 'id', True)])
def test_c_model_greedy_matches_numpy_oracle(d, pre, gf):
    rng = np.random.default_rng(7)
    n, m = 3000, 60
    x = rng.normal(size=(n, d))
    x[1000:1300] = x[:300]          # duplicated rows: exact ties, lowest index wins
    g = -x + 0.1 * rng.normal(size=(n, d))
    g[1000:1300] = g[:300]
    if gf:
        log_p = -0.5 * np.sum(x * x, axis=1)
        log_q = -0.45 * np.sum(x * x, axis=1)
        want = o.thin_gf(x, log_p, log_q, g, m, preconditioner=pre)
        s, gs = o._validate_and_standardize(x, g, True)
        w = np.exp(o._log_weights(log_p, log_q, None))
    else:
        want = o.thin(x, g, m, preconditioner=pre)
        s, gs = o._validate_and_standardize(x, g, True)
        w = None
    linv = o.make_precon(s, pre)
    idx, _ = oracle_c.greedy(s, gs, w, linv[0, 0], np.trace(linv), m)
    np.testing.assert_array_equal(idx, want)


@pytest.mark.parametrize('d,gf', [(2, True), (4, False), (9, False), (50, True)])
def test_threaded_bit_model_equals_sequential(d, gf):
    """sr_greedy_mt (the checker of the full-size GPU tests) equals sr_greedy for any thread count:
    same indices (lowest index among exact ties across thread blocks, first NaN) and bit-identical
    running sums."""
    from tests import oracle_c
    rng = np.random.default_rng(d)
    n, m = 3_001, 40
    x = rng.normal(size=(n, d))
    x[2_000:2_200] = x[10:210]                 # exact ties across thread-block boundaries
    g = -x + 0.1 * rng.normal(size=(n, d))
    g[2_000:2_200] = g[10:210]
    w = None
    if gf:
        lw = rng.normal(size=n)
        lw[[7, 2_500]] = 800.0                   # exp overflow -> inf weights -> NaN sums
        with np.errstate(over='ignore'):
            w = np.exp(lw - lw.min())
    want_idx, want_A = oracle_c.greedy(x, g, w, 0.7, 0.7 * d, m)
    for nt in (1, 2, 3, 7, 16):
        idx, A = oracle_c.greedy_mt(x, g, w, 0.7, 0.7 * d, m, nt)
        np.testing.assert_array_equal(idx, want_idx)
        assert np.array_equal(A, want_A, equal_nan=True)


def test_bit_model_powers_are_correctly_rounded():
    """qf^1.5 and qf^2.5 of the bit model (double-double to ~2^-105, q^2.5 as q times the q^1.5
    pair, then rounded once) against 80-digit Decimal powers: correctly rounded on 20 000
    log-uniform qf in [1, 2^120]; at values built to sit within 2^-106 of a rounding midpoint
    (qf just below a power of four: (4 - 2^-51)^1.5 = 8 - 1.5 2^-50 + 3 2^-106) the double-double
    cannot decide and the result may be the other neighbour -- within one ulp, as NumPy's own pow."""
    rng = np.random.default_rng(7)
    q = np.exp2(rng.uniform(0, 120, size=20_000)) * (1 + rng.uniform(0, 1e-3, size=20_000))
    p15, p25 = oracle_c.pow_15_25(q)
    want15 = np.array([_cr_pow(v, 1.5) for v in q])
    want25 = np.array([_cr_pow(v, 2.5) for v in q])
    assert np.array_equal(p15, want15), np.flatnonzero(p15 != want15)[:5]
    assert np.array_equal(p25, want25), np.flatnonzero(p25 != want25)[:5]
    edge = np.array([1.0, np.nextafter(1.0, 2.0), 2.0, 4.0, np.nextafter(4.0, 0.0), 2.0 ** 100])
    e15, e25 = oracle_c.pow_15_25(edge)
    for got, e in ((e15, 1.5), (e25, 2.5)):
        want = np.array([_cr_pow(v, e) for v in edge])
        assert np.all(np.abs(got - want) <= np.spacing(want))


# ------------------------------------------------------------------------------------------
# BASELINE configs 4 / 5 at full length: the C bit model (what the GPU parity tests compare the
# running sums with) selects exactly the reference NumPy path's indices
# (tests/golden/config{4,5}_numpy_indices.json, tests/golden/make_config_golden.py)
# ------------------------------------------------------------------------------------------
def _golden_config(name):
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', name)) as f:
        return json.load(f)


def _config_inputs(x, g, log_p=None, log_q=None):
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    w = None if log_p is None else np.exp(o._log_weights(log_p, log_q, None))
    return s, gs, w, float(linv[0, 0]), float(np.trace(linv))


@pytest.mark.parametrize('mode', ['compact', 'exact'])
def test_bitmodel_config4_full_length_equals_numpy_fixture(mode):
    """Both arithmetics of the d <= 8 kernels select all 1 000 indices of the NumPy fixture."""
    from bench import lv_surrogate
    fx = _golden_config('config4_numpy_indices.json')
    x, g, _, _ = lv_surrogate(2_000_000, 12345)
    s, gs, _, l, tr = _config_inputs(x, g)
    assert oracle_c.compact_ok(s, gs, l, tr)
    idx, _ = oracle_c.greedy_mt(s, gs, None, l, tr, 1000, arith=mode)
    np.testing.assert_array_equal(idx, fx['indices'])
    assert fx['min_margin_ulps'] > 1e3   # no step is a near tie that 1-ulp pow differences could flip


def test_bitmodel_config5_full_length_equals_numpy_fixture():
    import warnings
    from bench import gaussian_d50
    fx = _golden_config('config5_numpy_indices.json')
    x, log_p, log_q, gq = gaussian_d50(500_000, 12349)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        s, gs, w, l, tr = _config_inputs(x, gq, log_p, log_q)
    idx, _ = oracle_c.greedy_mt(s, gs, w, l, tr, 500)
    np.testing.assert_array_equal(idx, fx['indices'])
    assert fx['min_margin_ulps'] > 1e3
