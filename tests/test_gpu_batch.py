"""Batch launch (st_greedy_batch; device.greedy_concurrent's first choice): independent thins in ONE
persistent launch, each problem on its own group of #CU / count blocks.  Indices and running sums
must equal each problem's own st_greedy run bit for bit -- including a compact-only batch whose
gated general kernel takes over one problem only -- and the C model's.
"""
import numpy as np
import pytest

from oracle import stein_numpy as o
from tests import oracle_c

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import device  # noqa: E402
from stein_thinning.device import DeviceProblem  # noqa: E402


def _problem(n, d, seed, gf=False, tiny=False):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d)) @ np.diag(np.linspace(0.7, 1.6, d))
    g = -x / np.linspace(0.7, 1.6, d) ** 2
    s, gs = o._validate_and_standardize(x, g, True)
    s, gs = s.copy(), gs.copy()
    if tiny:   # rows out of the compact range in one block: the compact-only run hands over
        s[n // 2:n // 2 + 10, 1] = 1e-30
    linv = o.make_precon(s, 'med')
    w = np.exp(0.1 * np.tanh(s[:, 0])) if gf else None
    return s, gs, w, float(linv[0, 0]), float(np.trace(linv))


def _batch(probs, m):
    bufs = [p.greedy_buffers(m) for p in probs]
    applied = device._launch_batch(probs, m, bufs)
    torch.cuda.synchronize()
    return applied, [(b[0].cpu().numpy().view(np.uint32).astype(np.int64), b[1][:p.n].cpu().numpy())
                     for p, b in zip(probs, bufs)]


@pytest.mark.parametrize('d', [2, 4])
@pytest.mark.parametrize('gf', [False, True])
def test_batch_equals_one_by_one(d, gf):
    """Four problems of different n (150k .. 250k rows: the 512-thread general kernel at 64 blocks
    each) in one launch: each gives its own st_greedy indices and running sums."""
    m = 40
    inputs = [_problem(n, d, seed=10 * d + k, gf=gf) for k, n in enumerate((150_001, 181_337, 230_000, 250_003))]
    probs = [DeviceProblem(*inp) for inp in inputs]
    applied, got = _batch(probs, m)
    assert applied
    for p, (idx, A) in zip(probs, got):
        want, want_A = p.greedy(m, return_sums=True, dedup=False)
        np.testing.assert_array_equal(idx, want)
        assert np.array_equal(A, want_A), np.flatnonzero(A != want_A)[:10]
    cidx, cA = oracle_c.greedy(*inputs[1], m)
    np.testing.assert_array_equal(got[1][0], cidx)
    assert np.array_equal(got[1][1], cA)


def test_batch_compact_only_and_handoff():
    """Two problems of 600k rows (the compact-only kernel at 128 blocks each); the second has rows
    out of the compact range, so its group hands over to the gated general batch kernel while the
    first group's compact run completes: both equal their own runs and the C model."""
    m = 30
    inputs = [_problem(600_000, 4, seed=3), _problem(600_000, 4, seed=4, tiny=True)]
    probs = [DeviceProblem(*inp) for inp in inputs]
    applied, got = _batch(probs, m)
    assert applied
    for inp, p, (idx, A) in zip(inputs, probs, got):
        want, want_A = p.greedy(m, return_sums=True, dedup=False)
        np.testing.assert_array_equal(idx, want)
        assert np.array_equal(A, want_A), np.flatnonzero(A != want_A)[:10]
        cidx, cA = oracle_c.greedy_mt(*inp, m)
        np.testing.assert_array_equal(idx, cidx)
        assert np.array_equal(A, cA)


@pytest.mark.parametrize('gf', [False, True])
def test_batch_small_problems_256_thread_kernel(gf):
    """Small problems (20k .. 60k rows: a few hundred rows per block, the 256-thread kernel) batch
    too: indices and running sums equal each problem's own run."""
    m = 25
    inputs = [_problem(n, 2, seed=200 + k, gf=gf) for k, n in enumerate((20_000, 33_333, 47_001, 60_000))]
    probs = [DeviceProblem(*inp) for inp in inputs]
    applied, got = _batch(probs, m)
    assert applied
    for p, (idx, A) in zip(probs, got):
        want, want_A = p.greedy(m, return_sums=True, dedup=False)
        np.testing.assert_array_equal(idx, want)
        assert np.array_equal(A, want_A), np.flatnonzero(A != want_A)[:10]


def test_batch_declines_mixed_or_unsupported_problems():
    """Problems that plan onto different kernels (a 2e4-row problem next to a 2e5-row one, or
    different register rows), or a d the persistent kernel does not take, return ST_ERR_UNSUPPORTED
    with nothing enqueued."""
    m = 20
    for sizes, d in [((200_000, 20_000), 4), ((150_000, 900_000), 4), ((100_000, 100_000), 3)]:
        probs = [DeviceProblem(*_problem(n, d, seed=k)) for k, n in enumerate(sizes)]
        applied, _ = _batch(probs, m)
        assert not applied, (sizes, d)


def test_greedy_concurrent_batches_by_d(monkeypatch):
    """greedy_concurrent groups the problems by d: the d = 2 and d = 4 groups each go out as one
    batch launch, the small ones through the streams; every result equals the problem's own run."""
    calls = []
    real = device._launch_batch

    def spy(runs, n_points, bufs):
        ok = real(runs, n_points, bufs)
        calls.append((runs[0].d, len(runs), ok))
        return ok
    monkeypatch.setattr(device, '_launch_batch', spy)
    m = 35
    probs = [DeviceProblem(*_problem(n, d, seed=100 + k)) for k, (n, d) in
             enumerate([(200_000, 4), (170_000, 2), (215_000, 4), (180_000, 2), (20_000, 4)])]
    got = device.greedy_concurrent(probs, m, dedup=False)
    want = [p.greedy(m, dedup=False) for p in probs]
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)
    # the d = 4 group holds the small problem too: that batch is declined and runs on the streams
    assert sorted(calls) == [(2, 2, True), (4, 3, False)]
    calls.clear()
    got = device.greedy_concurrent(probs[:4], m, dedup=False)
    for a, b in zip(got, want[:4]):
        np.testing.assert_array_equal(a, b)
    assert sorted(calls) == [(2, 2, True), (4, 2, True)]


def test_thin_chains_raises_the_loops_error():
    """thin_chains builds the chains one after the other and raises what the loop of thin() calls
    raises: the first failing chain's error (here chain 1's NaN, not chain 2's shape mismatch); a bad
    n_points after chain 0's input (the loop's first thin() checks it there); mismatched list lengths."""
    import re
    import stein_thinning
    rng = np.random.default_rng(9)
    xs = [rng.normal(size=(70_000, 4)) for _ in range(4)]
    gs = [-x for x in xs]
    gs[1] = gs[1].copy()
    gs[1][123, 2] = np.nan
    gs[2] = gs[2][:, :3]
    with pytest.raises(Exception) as want:
        [stein_thinning.thin(x, g, 10, preconditioner='med') for x, g in zip(xs, gs)]
    with pytest.raises(type(want.value), match=re.escape(str(want.value))):
        stein_thinning.thin_chains(xs, gs, 10, preconditioner='med')
    for m in (0, -1):   # chain 0 valid, chain 1 NaN: the loop raises the n_points error first
        with pytest.raises(Exception) as want:
            [stein_thinning.thin(x, g, m, preconditioner='med') for x, g in zip(xs, gs)]
        with pytest.raises(type(want.value), match=re.escape(str(want.value))):
            stein_thinning.thin_chains(xs, gs, m, preconditioner='med')
    gs0 = [-xs[0].copy()]
    gs0[0][5, 1] = np.inf   # chain 0 invalid and n_points bad: the loop raises chain 0's input error
    with pytest.raises(Exception) as want:
        stein_thinning.thin(xs[0], gs0[0], 0, preconditioner='med')
    with pytest.raises(type(want.value), match=re.escape(str(want.value))):
        stein_thinning.thin_chains(xs[:1], gs0, 0, preconditioner='med')
    with pytest.raises(ValueError, match='one entry per chain'):
        stein_thinning.thin_chains(xs, gs[:2], 10)
    got = stein_thinning.thin_chains(xs[:1] + xs[3:], gs[:1] + gs[3:], 10, preconditioner='med')
    for x, g, idx in zip(xs[:1] + xs[3:], gs[:1] + gs[3:], got):
        np.testing.assert_array_equal(idx, stein_thinning.thin(x, g, 10, preconditioner='med'))


def test_greedy_concurrent_splits_a_declined_batch(monkeypatch):
    """Two large and two small problems of one d plan onto different kernels as one batch; the
    declined group is split by size and each half goes out as its own batch launch."""
    calls = []
    real = device._launch_batch

    def spy(runs, n_points, bufs):
        ok = real(runs, n_points, bufs)
        calls.append((len(runs), tuple(sorted(p.n for p in runs)), ok))
        return ok
    monkeypatch.setattr(device, '_launch_batch', spy)
    m = 30
    probs = [DeviceProblem(*_problem(n, 4, seed=300 + k)) for k, n in
             enumerate([200_000, 20_000, 215_000, 25_000])]
    got = device.greedy_concurrent(probs, m, dedup=False)
    for p, idx in zip(probs, got):
        np.testing.assert_array_equal(idx, p.greedy(m, dedup=False))
    assert calls == [(4, (20_000, 25_000, 200_000, 215_000), False), (2, (20_000, 25_000), True),
                     (2, (200_000, 215_000), True)]
