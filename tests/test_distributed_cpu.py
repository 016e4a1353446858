"""N > 1 orchestration of stein_thinning.distributed on CPU ranks (gloo, world_size 2 and 3):
row shards + per-step all-gather of candidate records give exactly the single-process indices,
including exact ties across shard boundaries (lowest global index wins)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import stein_numpy as o
from stein_thinning.distributed import combine_near_tie, run_ksd_sharded, run_sharded, shard_bounds, triangle_row_bounds


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _data(gf):
    rng = np.random.default_rng(11)
    n, d = 1501, 3
    x = rng.normal(size=(n, d))
    x[900:1000] = x[100:200]          # duplicates living in different shards
    g = -x + 0.05 * rng.normal(size=(n, d))
    g[900:1000] = g[100:200]
    if gf:
        log_p = -0.5 * np.sum(x * x, axis=1)
        log_q = -0.4 * np.sum(x * x, axis=1)
        return x, g, log_p, log_q
    return x, g, None, None


def _worker(rank, world, port, gf, m, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from tests.cpu_shard_backend import CpuShardBackend
        x, g, log_p, log_q = _data(gf)
        s, gs = o._validate_and_standardize(x, g, True)
        w = np.exp(o._log_weights(log_p, log_q, None)) if gf else None
        linv = o.make_precon(s, 'med')
        r0, r1 = shard_bounds(s.shape[0], rank, world)
        be = CpuShardBackend(s, gs, w, linv[0, 0], np.trace(linv), r0, r1, world, m)
        idx = run_sharded(be, m)
        np.save(os.path.join(out_dir, f'idx{rank}.npy'), idx)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,gf', [(2, False), (2, True), (3, False)])
def test_sharded_equals_single_process(tmp_path, world, gf):
    m = 40
    mp.spawn(_worker, args=(world, _free_port(), gf, m, str(tmp_path)), nprocs=world, join=True)
    x, g, log_p, log_q = _data(gf)
    want = o.thin_gf(x, log_p, log_q, g, m, preconditioner='med') if gf else o.thin(x, g, m, preconditioner='med')
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}.npy'), want)


def _dropin_worker(rank, world, port, m, out_dir, differ):
    """The drop-in stein_thinning.thinning.thin / thin_gf called on every rank of a gloo group: rows
    sharded across the ranks (thin_across_ranks), CPU stand-in for the HIP shard backend."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE='rccl',
                      ST_SHARD_THIN='1')
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning import distributed as sd
        from stein_thinning import thinning as st
        from tests import cpu_shard_backend
        sd.HipShardBackend = cpu_shard_backend.from_integrand
        x, g, log_p, log_q = _data(True)
        if differ:
            try:
                st.thin(x + rank, g, m, preconditioner='med')
            except ValueError as e:
                np.save(os.path.join(out_dir, f'err{rank}.npy'), np.array(['different problems' in str(e)]))
            return
        idx = st.thin(x, g, m, preconditioner='med')
        mode = sd.last_mode
        idx_gf = st.thin_gf(x, log_p, log_q, g, m, preconditioner='med')
        np.save(os.path.join(out_dir, f'idx{rank}.npy'), idx)
        np.save(os.path.join(out_dir, f'gf{rank}.npy'), idx_gf)
        np.save(os.path.join(out_dir, f'mode{rank}.npy'), np.array([mode]))
    finally:
        dist.destroy_process_group()


def test_dropin_thin_shards_under_multi_rank_launch(tmp_path):
    m, world = 30, 2
    mp.spawn(_dropin_worker, args=(world, _free_port(), m, str(tmp_path), False), nprocs=world, join=True)
    x, g, log_p, log_q = _data(True)
    want = o.thin(x, g, m, preconditioner='med')
    want_gf = o.thin_gf(x, log_p, log_q, g, m, preconditioner='med')
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}.npy'), want)
        np.testing.assert_array_equal(np.load(tmp_path / f'gf{r}.npy'), want_gf)
        assert str(np.load(tmp_path / f'mode{r}.npy')[0]) == 'records-all-gather'


def test_dropin_thin_rejects_different_problems_per_rank(tmp_path):
    mp.spawn(_dropin_worker, args=(2, _free_port(), 10, str(tmp_path), True), nprocs=2, join=True)
    for r in range(2):
        assert bool(np.load(tmp_path / f'err{r}.npy')[0])


def _optin_worker(rank, world, port, out_dir):
    """Row sharding of the drop-in thin is opt-in: off by default under a multi-rank launch (a rank
    may thin alone -- nothing collective runs), on with ST_SHARD_THIN=1 or set_rank_sharding(True)."""
    os.environ.pop('ST_SHARD_THIN', None)
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning import thinning as st
        got = [st._rank_sharding()]
        os.environ['ST_SHARD_THIN'] = '1'
        got.append(st._rank_sharding())
        st.set_rank_sharding(False)
        got.append(st._rank_sharding())
        os.environ.pop('ST_SHARD_THIN')
        st.set_rank_sharding(True)
        got.append(st._rank_sharding())
        st.set_rank_sharding(None)
        got.append(st._rank_sharding())
        np.save(os.path.join(out_dir, f'optin{rank}.npy'), np.array(got))
    finally:
        dist.destroy_process_group()


def test_dropin_row_sharding_is_opt_in(tmp_path):
    mp.spawn(_optin_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert np.load(tmp_path / f'optin{r}.npy').tolist() == [False, True, False, True, False]


def test_shard_bounds_cover_rows():
    for n in [1, 7, 100, 2_000_001]:
        for world in [1, 2, 3, 8]:
            if world > n:
                continue
            b = [shard_bounds(n, r, world) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in b]
            assert max(sizes) - min(sizes) <= 1


def _ksd_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from tests.cpu_shard_backend import CpuKsdBackend
        x, g, log_p, log_q = _data(True)
        s, gs = o._validate_and_standardize(x, g, True)
        w = np.exp(o._log_weights(log_p, log_q, None))
        linv = o.make_precon(s, 'med')
        n = 400
        ks = run_ksd_sharded(CpuKsdBackend(s, gs, w, linv[0, 0], np.trace(linv), n), n)
        np.save(os.path.join(out_dir, f'ks{rank}.npy'), ks)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_ksd_row_sharded_all_reduce(tmp_path, world):
    """Row-sharded KSD: triangle row blocks + gloo all-reduce of the column-sum vector reproduce
    the reference's cumulative KSD (oracle ksd over the gradient-free integrand)."""
    mp.spawn(_ksd_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    x, g, log_p, log_q = _data(True)
    want = o.ksd(o._make_stein_gf_integrand(x, log_p, log_q, g, preconditioner='med'), 400)
    for r in range(world):
        np.testing.assert_allclose(np.load(tmp_path / f'ks{r}.npy'), want, rtol=1e-12)


def test_triangle_row_bounds_balance():
    for n in [1, 2, 5, 1000, 2_000_000]:
        for world in [1, 2, 3, 8]:
            b = [triangle_row_bounds(n, r, world) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            pairs = [sum(n - 1 - a for a in range(a0, a1)) if n < 5000 else
                     (a1 - a0) * (n - 1) - (a1 * (a1 - 1) - a0 * (a0 - 1)) // 2 for a0, a1 in b]
            assert sum(pairs) == n * (n - 1) // 2
            if n >= 1000:
                assert max(pairs) - min(pairs) <= 2 * n


def rank_first_flag(s, g, w, l, tr, m, r0, r1):
    """The kernels' near-tie check restricted to one rank's rows [r0, r1) -- what that rank's blocks flag
    (persistent_kernel.hpp tie_check): per step, the smallest running sum of its rows other than the global
    winner and the winner's bitwise duplicates, against the global winner's sum and the threshold thr(t)
    the rank computes from bounds over all n rows.  The first such step, or -1.  (A restatement over the C
    bit model's sums: test infrastructure.)"""
    from tests import oracle_c
    idx, _, _, thr, _, wv = oracle_c.greedy_ties(s, g, w, l, tr, m, winner_sums=True)
    rows = np.arange(r0, r1)
    for t in range(m):
        _, A = oracle_c.greedy(s, g, w, l, tr, t + 1)   # the sums whose argmin is idx[t]
        j = int(idx[t])
        dup = np.all(s[rows] == s[j], axis=1) & np.all(g[rows] == g[j], axis=1)
        same = dup & (np.all(s[rows].view(np.uint64) == s[j].view(np.uint64), axis=1) &
                      np.all(g[rows].view(np.uint64) == g[j].view(np.uint64), axis=1))
        if w is not None:
            same &= w[rows].view(np.uint64) == w[j].view(np.uint64)
        cand = rows[~same]
        if cand.size and A[cand].min() - wv[t] <= thr[t]:
            return t
    return -1


def _tie_data(kind):
    from tests import margins_ref as mr
    if kind == 'twins':
        X, G, _ = mr.near_tie_twins(1)
    elif kind == 'pooled':
        X, G, _ = mr.near_tie_twins(6)
        X, G = np.vstack([X, X]), np.vstack([G, G])
    else:   # duplicates only: no step is a near tie
        rng = np.random.default_rng(2)
        X = rng.normal(size=(300, 2))
        X, G = np.vstack([X, X[::-1]]), -np.vstack([X, X[::-1]])
    return X, G


def _tie_worker(rank, world, port, kind, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        X, G = _tie_data(kind)
        s, gs = o._validate_and_standardize(X, G, True)
        linv = o.make_precon(s, 'id')
        r0, r1 = shard_bounds(s.shape[0], rank, world)
        own = rank_first_flag(s, gs, None, linv[0, 0], np.trace(linv), 30, r0, r1)
        np.save(os.path.join(out_dir, f'tie{rank}.npy'), np.array([own, combine_near_tie(own)]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,kind', [(2, 'twins'), (3, 'twins'), (2, 'pooled'), (3, 'dups')])
def test_rank_level_tie_rule_equals_the_model(tmp_path, world, kind):
    """each rank flags its own rows against the global winner and the global threshold,
    one all-reduce MIN combines the words (distributed.combine_near_tie); the combined first flagged step
    equals the single-device model's (oracle/stein_ref.c sr_greedy_mt_ties) on near-tie twins, twins pooled
    with their own copy (the winners' duplicates in other shards must not flag) and duplicates only."""
    from tests import oracle_c
    mp.spawn(_tie_worker, args=(world, _free_port(), kind, str(tmp_path)), nprocs=world, join=True)
    X, G = _tie_data(kind)
    s, gs = o._validate_and_standardize(X, G, True)
    linv = o.make_precon(s, 'id')
    *_, flagged = oracle_c.greedy_ties(s, gs, None, linv[0, 0], np.trace(linv), 30)
    want = int(np.flatnonzero(flagged)[0]) if flagged.any() else -1
    got = [np.load(tmp_path / f'tie{r}.npy') for r in range(world)]
    assert all(int(v[1]) == want for v in got)
    assert min((int(v[0]) for v in got if v[0] >= 0), default=-1) == want
    if kind == 'dups':
        assert want == -1


def test_combine_near_tie_single_process():
    assert combine_near_tie(-1) == -1 and combine_near_tie(7) == 7 and combine_near_tie(-2) == -2
