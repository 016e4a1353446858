"""Full-sample KSD on the GPU (K6: column sums of the lower triangle + prefix scan), its row-sharded
form (the n-length column-sum all-reduce) and the multi-process run (``pytest -m gpu``).

Bar: within 1e-12 relative of the NumPy oracle's ``ksd`` (oracle/stein_numpy.py, restating
stein_thinning.stein.ksd; north_star tolerance 1e-6).  The GPU sums each column sequentially over
the rows and scans in 1024 chunks; the reference sums with NumPy's pairwise sum and scans
sequentially, so agreement is to rounding, not bitwise.
"""
import os
import socket
import warnings

import numpy as np
import pytest

from oracle import stein_numpy as o
from tests import oracle_c

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import stein as ss  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402
from stein_thinning.distributed import HipKsdBackend, run_ksd_sharded, triangle_row_bounds  # noqa: E402


def _problem(n, d, gf, seed=3, pre='med'):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d)) @ np.diag(np.linspace(0.5, 2.0, d))
    x[n // 3:n // 3 + 20] = x[:20]                      # duplicated rows
    g = -x / np.linspace(0.5, 2.0, d) ** 2 + 0.1 * rng.normal(size=(n, d))
    g[n // 3:n // 3 + 20] = g[:20]
    if gf:
        log_p = -0.5 * np.sum(x * x, axis=1)
        log_q = -0.45 * np.sum(x * x, axis=1) + 0.01 * rng.normal(size=n)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            dev = st._make_stein_gf_integrand(x, log_p, log_q, g, preconditioner=pre)
            ref = o._make_stein_gf_integrand(x, log_p, log_q, g, preconditioner=pre)
        return dev, ref
    return st._make_stein_integrand(x, g, preconditioner=pre), o._make_stein_integrand(x, g, preconditioner=pre)


@pytest.mark.parametrize('d,gf', [(1, False), (2, False), (4, False), (4, True), (8, True), (9, False),
                                  (50, True)])
def test_ksd_matches_oracle(d, gf):
    n = 700
    dev, ref = _problem(n, d, gf)
    got = ss.ksd(dev, n)
    want = o.ksd(ref, n)
    np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)


def test_ksd_prefix_of_longer_run_and_subsets():
    dev, ref = _problem(3000, 4, False, seed=9, pre='id')
    full = ss.ksd(dev, 3000)
    np.testing.assert_allclose(full[:500], ss.ksd(dev, 500), rtol=1e-14)
    np.testing.assert_allclose(full[-5:], o.ksd(ref, 3000)[-5:], rtol=1e-12)
    idx = np.random.default_rng(1).permutation(3000)[:400]
    np.testing.assert_allclose(ss.ksd(o.reindex_integrand(dev, idx), 400),
                               o.ksd(o.reindex_integrand(ref, idx), 400), rtol=1e-12)


@pytest.mark.parametrize('world', [2, 3, 8])
def test_row_shards_sum_to_full(world):
    """Column sums over disjoint triangle row blocks, added on the host, = the one-range sums."""
    n = 2500
    dev, _ = _problem(n, 4, True, seed=4)
    be = HipKsdBackend(dev, n)
    full = be.colsum(0, n).clone()
    parts = torch.zeros_like(full)
    for r in range(world):
        a0, a1 = triangle_row_bounds(n, r, world)
        parts += be.colsum(a0, a1)
    np.testing.assert_allclose(parts.cpu().numpy(), full.cpu().numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(be.finish(parts), run_ksd_sharded(be, n), rtol=1e-12)


def test_large_n_against_c_bit_model_pairs():
    """n = 20 000 (2e8 pairs): the last cumulative KSD value against a host sum of the C bit-model
    pair values (column sums in the kernel's order, so the only difference is the final scan)."""
    n = 20_000
    rng = np.random.default_rng(7)
    x = rng.normal(size=(n, 4))
    g = -x + 0.05 * rng.normal(size=(n, 4))
    dev = st._make_stein_integrand(x, g, preconditioner='med')
    ks = ss.ksd(dev, n)
    s, gs, linv = dev.sample, dev.gradient, dev.linv_scale
    cols = np.arange(n - 200, n)          # the last 200 columns' full sums, bit model
    tot = 0.0
    for i in cols:
        a = np.arange(i)
        tot += 2.0 * np.sum(oracle_c.pairs(s, gs, None, linv, dev.linv_trace, np.full(i, i), a, arith='exact'))
    diag = oracle_c.pairs(s, gs, None, linv, dev.linv_trace, cols, cols, arith='exact')
    tail = tot + np.sum(diag)
    S = (ks[-1] * n) ** 2 - (ks[n - 201] * (n - 200)) ** 2
    np.testing.assert_allclose(S, tail, rtol=1e-9)


def _free_port():
    with socket.socket() as so:
        so.bind(('127.0.0.1', 0))
        return so.getsockname()[1]


def _ksd_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning.distributed import ksd_sharded
        dev, _ = _problem(1800, 4, True, seed=5)
        np.save(os.path.join(out_dir, f'ks{rank}.npy'), ksd_sharded(dev, 1800))
    finally:
        dist.destroy_process_group()


def test_ksd_sharded_processes(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_ksd_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    dev, ref = _problem(1800, 4, True, seed=5)
    want = o.ksd(ref, 1800)
    for r in range(2):
        np.testing.assert_allclose(np.load(tmp_path / f'ks{r}.npy'), want, rtol=1e-12)


@pytest.mark.parametrize('gf', [False, True])
def test_colsum_per_pair_rule_independent_of_row_shards(gf):
    """Compact setting with a few rows outside [2^-60, 2^60] (tiny gradient coordinates): every pair
    takes the arithmetic the per-pair rule gives it (stein_math.hpp pair_value_sel) whatever tile or
    row shard it falls in, so each shard's column sums equal, bit for bit, the sequential sums of the
    C bit model's compact-rule pair values over that shard's rows."""
    from stein_thinning import _native as nat
    if nat.arithmetic() != 'compact':
        pytest.skip('compact arithmetic not selected')
    n, d = 900, 4
    rng = np.random.default_rng(21)
    x = rng.normal(size=(n, d))
    g = -x + 0.1 * rng.normal(size=(n, d))
    for r in (10, 300, 301, 777):
        g[r, 1] = 1e-25          # standardised: ~1e-25 < 2^-60 -> these rows' pairs take the exact form
    if gf:
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            dev = st._make_stein_gf_integrand(x, -0.5 * np.sum(x * x, 1), -0.45 * np.sum(x * x, 1), g,
                                              preconditioner='med')
    else:
        dev = st._make_stein_integrand(x, g, preconditioner='med')
    s, gs, w = dev.sample, dev.gradient, dev.weights
    assert not oracle_c.compact_ok(s[[10]], gs[[10]], dev.linv_scale, dev.linv_trace)
    be = HipKsdBackend(dev, n)
    ii, aa = np.tril_indices(n, -1)            # column i, row a < i (row-major: a increasing per i)
    kv = oracle_c.pairs(s, gs, None, dev.linv_scale, dev.linv_trace, ii, aa, arith='compact')
    if gf:
        kv = (kv * w[ii]) * w[aa]
    for a0, a1 in [(0, n)] + [triangle_row_bounds(n, r, 3) for r in range(3)] + [(5, 301), (301, 302)]:
        got = be.colsum(a0, a1).cpu().numpy()
        want = np.zeros(n)
        sel = (aa >= a0) & (aa < a1)
        for i in range(n):
            v = kv[sel & (ii == i)]
            if v.size:
                want[i] = np.cumsum(v)[-1]     # sequential, in increasing a (the kernel's order)
        np.testing.assert_array_equal(got, want, err_msg=f'rows [{a0}, {a1})')
