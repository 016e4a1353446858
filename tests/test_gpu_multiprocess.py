"""Multi-process sharded thinning on the GPU box: 2-3 ranks (processes) on the one visible GPU
(RCCL cannot place two ranks on one device, so the group is gloo): the record all-gather path, the
persistent device-exchange engine (d = 2, 4) and the launch-per-step device-exchange engine (other
d) through IPC-mapped mailboxes, and a 1-rank RCCL run of the HIP-graph-captured loop."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from oracle import stein_numpy as o  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _data(d=4):
    rng = np.random.default_rng(5)
    n = 40_003
    x = rng.normal(size=(n, d))
    x[30_000:30_400] = x[2_000:2_400]      # exact ties across the shard boundary
    g = -x + 0.1 * rng.normal(size=(n, d))
    g[30_000:30_400] = g[2_000:2_400]
    log_p = -0.5 * np.sum(x * x, axis=1)
    log_q = -0.45 * np.sum(x * x, axis=1)
    return x, g, log_p, log_q


def _worker(rank, world, port, backend, gf, out_dir, exchange='device', runs=1, d=4):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE=exchange)
    torch.cuda.set_device(0)
    kw = dict(device_id=torch.device('cuda', 0)) if backend == 'nccl' else {}
    dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    try:
        from stein_thinning import distributed as sd
        x, g, log_p, log_q = _data(d)
        for run in range(runs):
            gf_run = gf if run % 2 == 0 else not gf   # alternate kernels on the same mailboxes
            if gf_run:
                idx = sd.thin_gf_sharded(x, log_p, log_q, g, 80, preconditioner='med')
            else:
                idx = sd.thin_sharded(x, g, 80, preconditioner='med')
            np.save(os.path.join(out_dir, f'idx{rank}_{run}.npy'), idx)
            with open(os.path.join(out_dir, f'mode{rank}_{run}.txt'), 'w') as f:
                f.write(str(sd.last_mode))
    finally:
        dist.destroy_process_group()


def _want(gf, d=4):
    x, g, log_p, log_q = _data(d)
    return o.thin_gf(x, log_p, log_q, g, 80, preconditioner='med') if gf else o.thin(x, g, 80, preconditioner='med')


@pytest.mark.parametrize('gf', [False, True])
def test_two_processes_one_gpu_gloo_rccl_records(tmp_path, gf):
    """Per-step record all-gather path (forced), two ranks exchanging through gloo."""
    mp.spawn(_worker, args=(2, _free_port(), 'gloo', gf, str(tmp_path), 'rccl'), nprocs=2, join=True)
    want = _want(gf)
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}_0.npy'), want)
        assert (tmp_path / f'mode{r}_0.txt').read_text() == 'records-all-gather'


@pytest.mark.parametrize('world,gf', [(2, False), (3, True)])
def test_device_exchange_processes_share_one_gpu(tmp_path, world, gf):
    """Persistent multi-rank kernel: `world` processes on the one visible GPU, IPC-mapped device
    mailboxes (the same code path as one rank per GPU over xGMI), three consecutive runs on the
    same mailboxes (sequence numbers / tags carry over), both kernels."""
    mp.spawn(_worker, args=(world, _free_port(), 'gloo', gf, str(tmp_path), 'device', 3), nprocs=world,
             join=True)
    for run in range(3):
        want = _want(gf if run % 2 == 0 else not gf)
        for r in range(world):
            assert (tmp_path / f'mode{r}_{run}.txt').read_text() == 'device-exchange'
            np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}_{run}.npy'), want)


@pytest.mark.parametrize('world,gf,d', [(2, False, 3), (3, True, 10)])
def test_step_device_exchange_processes_share_one_gpu(tmp_path, world, gf, d):
    """Launch-per-step engine with the mailbox exchange kernel (d outside the persistent kernel's
    set; compile-time-d and runtime-d step kernels): graph-captured loop, three consecutive runs on
    the same mailboxes (the device-side exchange counter carries over replays), both kernels."""
    mp.spawn(_worker, args=(world, _free_port(), 'gloo', gf, str(tmp_path), 'device', 3, d), nprocs=world,
             join=True)
    for run in range(3):
        want = _want(gf if run % 2 == 0 else not gf, d)
        for r in range(world):
            assert (tmp_path / f'mode{r}_{run}.txt').read_text() == 'device-exchange-steps-graph'
            np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}_{run}.npy'), want)


@pytest.mark.parametrize('world,gf', [(2, True), (3, False)])
def test_wide_persistent_device_exchange_share_one_gpu(tmp_path, world, gf):
    """d = 50 shards of at most 256 rows per CU: the wide persistent kernel per rank with the
    in-kernel mailbox exchange (engine 'persistent' -> mode 'device-exchange'), three runs."""
    mp.spawn(_worker, args=(world, _free_port(), 'gloo', gf, str(tmp_path), 'device', 3, 50), nprocs=world,
             join=True)
    for run in range(3):
        want = _want(gf if run % 2 == 0 else not gf, 50)
        for r in range(world):
            assert (tmp_path / f'mode{r}_{run}.txt').read_text() == 'device-exchange'
            np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}_{run}.npy'), want)


def test_replicated_engine_processes_share_one_gpu(tmp_path):
    """ST_SHARDED_EXCHANGE=replicated (also the d = 2, 4 fallback when the device exchange is
    unavailable): every rank thins the whole sample with the single-GPU kernel, indices agree."""
    mp.spawn(_worker, args=(2, _free_port(), 'gloo', False, str(tmp_path), 'replicated', 2), nprocs=2, join=True)
    for run in range(2):
        want = _want(run % 2 == 1)
        for r in range(2):
            assert (tmp_path / f'mode{r}_{run}.txt').read_text() == 'replicated'
            np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}_{run}.npy'), want)


def _dropin_worker(rank, world, port, out_dir):
    """The reference's call surface, unchanged, on every rank of a 2-process group that opted in to
    row sharding (ST_SHARD_THIN=1): thin / thin_gf shard their rows across the ranks
    (thinning._greedy_search -> distributed.thin_across_ranks)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE='device',
                      ST_SHARD_THIN='1')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning import distributed as sd
        from stein_thinning import thinning as st
        x, g, log_p, log_q = _data()
        for run, gf in enumerate([False, True]):
            sd.last_mode = None
            idx = st.thin_gf(x, log_p, log_q, g, 80, preconditioner='med') if gf else \
                st.thin(x, g, 80, preconditioner='med')
            np.save(os.path.join(out_dir, f'idx{rank}_{run}.npy'), idx)
            with open(os.path.join(out_dir, f'mode{rank}_{run}.txt'), 'w') as f:
                f.write(str(sd.last_mode))
    finally:
        dist.destroy_process_group()


def _chain_data(n=60_001, d=4):
    """Random-walk chain with ~70 % of its rows repeating the row before (the repeated-row path)."""
    rng = np.random.default_rng(17)
    x = np.empty((n, d))
    x[0] = rng.normal(size=d)
    acc = rng.random(n) < 0.3
    for i in range(1, n):
        x[i] = x[i - 1] + 0.3 * rng.normal(size=d) if acc[i] else x[i - 1]
    return x, -x * np.linspace(0.5, 2.0, d)


def _dropin_dedup_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE='device',
                      ST_SHARD_THIN='1')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning import distributed as sd
        from stein_thinning import thinning as st
        x, g = _chain_data()
        idx = st.thin(x, g, 60, preconditioner='med')
        np.save(os.path.join(out_dir, f'didx{rank}.npy'), idx)
        with open(os.path.join(out_dir, f'dkept{rank}.txt'), 'w') as f:
            f.write(str(sd.last_rows_kept))
    finally:
        dist.destroy_process_group()


def test_dropin_sharded_thin_drops_repeated_rows(tmp_path):
    """The row-sharded drop-in thin compacts a chain's repeated rows on the host before sharding
    (SteinIntegrand.run_starts_view): every rank returns the NumPy path's indices."""
    mp.spawn(_dropin_dedup_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    x, g = _chain_data()
    want = o.thin(x, g, 60, preconditioner='med')
    for r in range(2):
        kept = int((tmp_path / f'dkept{r}.txt').read_text())
        assert 0 < kept < 0.5 * x.shape[0]
        np.testing.assert_array_equal(np.load(tmp_path / f'didx{r}.npy'), want)


def test_dropin_thin_shards_across_two_processes(tmp_path):
    mp.spawn(_dropin_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for run, gf in enumerate([False, True]):
        want = _want(gf)
        for r in range(2):
            assert (tmp_path / f'mode{r}_{run}.txt').read_text() == 'device-exchange'
            np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}_{run}.npy'), want)


def test_single_rank_rccl_graph_capture(tmp_path):
    mp.spawn(_worker, args=(1, _free_port(), 'nccl', False, str(tmp_path)), nprocs=1, join=True)
    x, g, _, _ = _data()
    np.testing.assert_array_equal(np.load(tmp_path / 'idx0_0.npy'), o.thin(x, g, 80, preconditioner='med'))


def _small_worker(rank, world, port, out_dir, exchange, d):
    """Tiny shards (n = 901 over `world` ranks: one block per rank) and m > n (2 000 points, the
    Gaussian_mixture.ipynb m = 10 000 > n = 1 000 regime): repeated selections, both kernels."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE=exchange)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning import distributed as sd
        rng = np.random.default_rng(3)
        x = rng.normal(size=(901, d))
        g = -x
        idx = sd.thin_sharded(x, g, 2000, preconditioner='med')
        np.save(os.path.join(out_dir, f'small{rank}.npy'), idx)
        with open(os.path.join(out_dir, f'smallmode{rank}.txt'), 'w') as f:
            f.write(str(sd.last_mode))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,exchange,d', [(3, 'device', 2), (3, 'device', 5), (2, 'rccl', 2)])
def test_tiny_shards_and_more_points_than_rows(tmp_path, world, exchange, d):
    mp.spawn(_small_worker, args=(world, _free_port(), str(tmp_path), exchange, d), nprocs=world, join=True)
    rng = np.random.default_rng(3)
    x = rng.normal(size=(901, d))
    want = o.thin(x, -x, 2000, preconditioner='med')
    expect = {'rccl': 'records-all-gather', 'device': 'device-exchange' if d in (2, 4) else
              'device-exchange-steps-graph'}[exchange]
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f'small{r}.npy'), want)
        assert (tmp_path / f'smallmode{r}.txt').read_text() == expect


def _large_worker(rank, world, port, out_dir, n, m):
    """One rank of a device-exchange run whose shards exceed 1 280 rows per block (the 512-thread,
    dynamic-chunk persistent kernel with LDS and streamed rows); grids capped so that the ranks'
    one-block-per-CU grids co-reside on the shared GPU (as bench.py's rehearsal mode does)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE='device')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning import _native as nat
        from stein_thinning import distributed as sd
        assert nat.lib().st_tune(5, 256 // world) == 0
        x, g = _rw_data(n)
        idx = sd.thin_sharded(x, g, m, preconditioner='med')
        np.save(os.path.join(out_dir, f'idx{rank}.npy'), idx)
        with open(os.path.join(out_dir, f'mode{rank}.txt'), 'w') as f:
            f.write(str(sd.last_mode))
    finally:
        dist.destroy_process_group()


def _rw_data(n, d=4):
    rng = np.random.default_rng(23)
    x = np.cumsum(0.05 * rng.normal(size=(n, d)), axis=0)   # random-walk chain: near-duplicate rows
    x[n // 2:n // 2 + 500] = x[1_000:1_500]                  # exact ties across the shard boundary
    g = -x + 0.1 * rng.normal(size=(n, d))
    g[n // 2:n // 2 + 500] = g[1_000:1_500]
    return x, g


def test_device_exchange_512_thread_shards_share_one_gpu(tmp_path):
    """Two ranks, 2e5 rows each on 128 blocks (1 563 rows per block > 1 280): the 512-thread
    persistent kernel under the device exchange, against the NumPy oracle."""
    n, m, world = 400_003, 30, 2
    mp.spawn(_large_worker, args=(world, _free_port(), str(tmp_path), n, m), nprocs=world, join=True)
    x, g = _rw_data(n)
    want = o.thin(x, g, m, preconditioner='med')
    for r in range(world):
        assert (tmp_path / f'mode{r}.txt').read_text() == 'device-exchange'
        np.testing.assert_array_equal(np.load(tmp_path / f'idx{r}.npy'), want)


def _config4_worker(rank, world, port, out_dir, data_path, m):
    """One of `world` ranks of config 4 on the shared GPU, grid 256 / world blocks each (bench.py's
    rehearsal mode): the raw host arrays go through thin_sharded exactly as on one GPU per rank."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE='device')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from stein_thinning import _native as nat
        from stein_thinning import distributed as sd
        assert nat.lib().st_tune(5, 256 // world) == 0
        data = np.load(data_path)
        idx = sd.thin_sharded(data['x'], data['g'], m, preconditioner='med')
        np.save(os.path.join(out_dir, f'c4idx{rank}.npy'), idx)
        with open(os.path.join(out_dir, f'c4mode{rank}.txt'), 'w') as f:
            f.write(str(sd.last_mode))
    finally:
        dist.destroy_process_group()


def test_config4_eight_ranks_share_one_gpu(tmp_path, config4):
    """Config 4 (n = 2e6, m = 1000) split over 8 ranks as on an 8-GPU node (2.5e5 rows per rank),
    the 8 processes sharing the one visible GPU with 32 blocks each: all 1000 indices identical to
    the C bit model on every rank, through the in-kernel mailbox exchange."""
    world = 8
    data_path = str(tmp_path / 'c4.npz')
    np.savez(data_path, x=config4['x'], g=config4['g'])
    mp.spawn(_config4_worker, args=(world, _free_port(), str(tmp_path), data_path, config4['m']),
             nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f'c4mode{r}.txt').read_text() == 'device-exchange'
        np.testing.assert_array_equal(np.load(tmp_path / f'c4idx{r}.npy'), config4['idx'])


def _config5_worker(rank, world, port, out_dir, m):
    """One of `world` ranks of config 5 (n = 5e5, d = 50, gradient-free) on the shared GPU through the
    drop-in thin_gf; grids capped to 256 / world blocks, so each rank's 62 500 rows exceed the wide
    persistent kernel's 256 rows per block and the launch-per-step engine with the mailbox exchange
    kernel runs (on an 8-GPU node every rank has its own 256 CUs and the wide persistent kernel).
    Row sharding of the drop-in call is opted in (ST_SHARD_THIN=1)."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE='device',
                      ST_SHARD_THIN='1')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import warnings
        from bench import gaussian_d50
        from stein_thinning import _native as nat
        from stein_thinning import distributed as sd
        from stein_thinning import thinning as st
        assert nat.lib().st_tune(5, 256 // world) == 0
        x, log_p, log_q, gq = gaussian_d50(500_000, 12349)
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            idx = st.thin_gf(x, log_p, log_q, gq, m, preconditioner='med')
        np.save(os.path.join(out_dir, f'c5idx{rank}.npy'), idx)
        with open(os.path.join(out_dir, f'c5mode{rank}.txt'), 'w') as f:
            f.write(str(sd.last_mode))
    finally:
        dist.destroy_process_group()


def test_config5_eight_ranks_share_one_gpu(tmp_path):
    """Config 5 split over 8 processes as one job: all 500 indices identical to
    the reference NumPy path's (tests/golden/config5_numpy_indices.json) on every rank."""
    import json
    world, m = 8, 500
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'config5_numpy_indices.json')) as f:
        want = np.asarray(json.load(f)['indices'])
    mp.spawn(_config5_worker, args=(world, _free_port(), str(tmp_path), m), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f'c5mode{r}.txt').read_text() == 'device-exchange-steps-graph'
        np.testing.assert_array_equal(np.load(tmp_path / f'c5idx{r}.npy'), want)


def test_sharded_supported_query_matches_launcher():
    """st_greedy_sharded_supported evaluates the persistent launcher's own eligibility: d = 2, 4 any
    shard; d = 50 only while a rank's block has at most 256 rows (so the grid cap st_tune key 5
    matters: config 5 at 8 ranks with 32 blocks per rank does NOT fit); other d never."""
    from stein_thinning import _native as nat
    L = nat.lib()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = 500_000
    assert L.st_greedy_sharded_supported(2_000_000, 4, 0, 0, 250_000, 0, 8, 1000) == 1
    assert L.st_greedy_sharded_supported(n, 50, 1, 0, n // 8, 0, 8, 500) == (1 if n // 8 <= 256 * cus else 0)
    assert L.st_greedy_sharded_supported(n, 9, 1, 0, n // 8, 0, 8, 500) == 0
    assert L.st_tune(5, 32) == 0
    try:
        assert L.st_greedy_sharded_supported(n, 50, 1, 0, n // 8, 0, 8, 500) == 0
        assert L.st_greedy_sharded_supported(2_000_000, 4, 0, 0, 250_000, 0, 8, 1000) == 1
    finally:
        L.st_tune(5, -1)
    assert L.st_greedy_sharded_supported(n, 50, 1, 10, 5, 0, 8, 500) < 0


def _near_tie_worker(rank, world, port, out_dir):
    """Every rank of a `world`-process group on the one GPU: the near-tie twins (tests/margins_ref.py, 10
    seeds: a runner-up a few ulps of its running sum from the winner at steps 8-12, the twins in another
    shard than most winners) through thin_sharded and through the drop-in thin() with ST_SHARD_THIN=1
    (VERDICT r05 next #1): the ranks' words are combined after the run and the flagged thin re-runs in the
    exact arithmetic on every rank.  Also the twins pooled with their own copy (exact ties with the
    winner's duplicates, in another shard: must not flag) and an exact tie between different rows."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), ST_SHARDED_EXCHANGE='device',
                      ST_SHARD_THIN='1')
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from tests import margins_ref as mr
        from stein_thinning import distributed as sd
        from stein_thinning import thinning as st
        out = {}
        for seed in range(10):
            X, G, _ = mr.near_tie_twins(seed)
            a = sd.thin_sharded(X, G, 30)
            out[f'sharded{seed}'] = (a.tolist(), sd.last_near_tie, sd.last_mode)
            b = st.thin(X, G, 30)
            out[f'dropin{seed}'] = (b.tolist(), sd.last_near_tie, sd.last_mode)
        X, G, _ = mr.near_tie_twins(5)
        c = sd.thin_sharded(np.vstack([X, X]), np.vstack([G, G]), 30)
        out['pooled'] = (c.tolist(), sd.last_near_tie, sd.last_mode)
        rng = np.random.default_rng(8)
        Z = rng.normal(size=(300, 2))
        Z = Z[np.sum(Z * Z, axis=1) > 0.5]
        Z[3] = [0.125, -0.25]
        Z[200] = -Z[3]
        e = sd.thin_sharded(Z, -Z, 3, standardize=False)
        out['mirror'] = (e.tolist(), sd.last_near_tie, sd.last_mode)
        import json
        with open(os.path.join(out_dir, f'nt{rank}.json'), 'w') as f:
            json.dump(out, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_near_tie_guard_across_processes(tmp_path, world):
    import json
    from tests import margins_ref as mr
    mp.spawn(_near_tie_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [json.loads((tmp_path / f'nt{r}.json').read_text()) for r in range(world)]
    for seed in range(10):
        X, G, steps = mr.near_tie_twins(seed)
        want = o.thin(X, G, 30)
        for r in range(world):
            for key in (f'sharded{seed}', f'dropin{seed}'):
                idx, tie, mode = res[r][key]
                np.testing.assert_array_equal(np.asarray(idx, dtype=np.uint32), want, err_msg=f'{key} rank {r}')
                assert tie == steps[0], (key, r, tie)   # the model's first flagged step (test_near_tie_cpu.py)
                assert mode == 'device-exchange'
    X, G, _ = mr.near_tie_twins(5)
    X2, G2 = np.vstack([X, X]), np.vstack([G, G])
    rng = np.random.default_rng(8)
    Z = rng.normal(size=(300, 2))
    Z = Z[np.sum(Z * Z, axis=1) > 0.5]
    Z[3] = [0.125, -0.25]
    Z[200] = -Z[3]
    for r in range(world):
        idx, tie, _ = res[r]['pooled']
        np.testing.assert_array_equal(np.asarray(idx, dtype=np.uint32), o.thin(X2, G2, 30))
        assert tie == 8   # the twins flag; the winners' exact copies in the other half do not
        idx, tie, _ = res[r]['mirror']
        np.testing.assert_array_equal(np.asarray(idx, dtype=np.uint32), o.thin(Z, -Z, 3, standardize=False))
        assert tie == 0
