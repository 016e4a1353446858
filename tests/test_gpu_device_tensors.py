"""The drop-in thin on ROCm tensors: inputs already on the GPU are used in place.
Only x travels to the host (st_standardize_download: its sequential column sums, bit-identical to NumPy's
mean / mean |x - loc|, and the 'med' subsample); g is checked and scaled on the device and never copied
to the host.  Indices, the standardised device arrays and the ValueErrors equal the NumPy route's."""
import contextlib

import numpy as np
import pytest

from oracle import stein_numpy as o

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

import stein_thinning  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402


def _data(n, d, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, d)) * np.linspace(0.5, 2, d)
    g = -x / np.linspace(0.5, 2, d) ** 2 + 0.1 * rng.normal(size=(n, d))
    return x, g


@contextlib.contextmanager
def no_host_copy(*tensors):
    """Fails the test if any host copy of these tensors is asked for (.cpu(), .numpy(), .to('cpu'),
    .tolist(), np.asarray) inside the block."""
    ptrs = {t.data_ptr() for t in tensors}
    saved = {name: getattr(torch.Tensor, name) for name in ('cpu', 'numpy', 'to', 'tolist', '__array__')}

    def guard(name):
        orig = saved[name]

        def f(self, *args, **kwargs):
            if self.data_ptr() in ptrs and (name != 'to' or _to_host(args, kwargs)):
                raise AssertionError(f'host copy of an input tensor: .{name}()')
            return orig(self, *args, **kwargs)
        return f
    try:
        for name in saved:
            setattr(torch.Tensor, name, guard(name))
        yield
    finally:
        for name, orig in saved.items():
            setattr(torch.Tensor, name, orig)


def _to_host(args, kwargs):
    dev = kwargs.get('device', args[0] if args else None)
    return dev is not None and not isinstance(dev, torch.dtype) and torch.device(dev).type == 'cpu'


@pytest.mark.parametrize('d,n', [(1, 100_003), (1, 777), (2, 100_003), (4, 100_003), (4, 999), (8, 100_003),
                                 (50, 20_001)])
def test_download_statistics_bit_identical(d, n):
    x, g = _data(n, d, seed=d)
    xd, gd = torch.from_numpy(x).cuda(), torch.from_numpy(g).cuda()
    with no_host_copy(xd, gd):
        up = st._download_standardized(xd, gd)
    n_, d_, scl, stage_x, stage_g, x_raw, g_raw = up
    loc = np.mean(x, axis=0)
    assert np.array_equal(scl, np.mean(np.abs(x - loc), axis=0))
    assert np.array_equal(stage_x, x) and stage_g is None
    assert x_raw.data_ptr() == xd.data_ptr() and g_raw.data_ptr() == gd.data_ptr()   # used in place
    with no_host_copy(xd, gd):
        integ = st._make_stein_integrand(xd, gd, preconditioner='med')
    prob = integ._problem
    s, gs = st._validate_and_standardize(x, g, True)
    assert np.array_equal(prob.x[:, :n].cpu().numpy().T, s)
    assert np.array_equal(prob.g[:, :n].cpu().numpy().T, gs)
    from stein_thinning.kernel import make_precon
    assert np.array_equal(integ.linv, make_precon(s, 'med'))
    assert integ._sample is None
    assert np.array_equal(integ.gradient, gs)   # the deferred host arrays (g fetched only here)


def test_thin_on_device_tensors_never_copies_g():
    n = 120_000
    x, g = _data(n, 4, seed=21)
    xd, gd = torch.from_numpy(x).cuda(), torch.from_numpy(g).cuda()
    want = o.thin(x, g, 30, preconditioner='med')
    with no_host_copy(gd):
        got = stein_thinning.thin(xd, gd, 30, preconditioner='med')
    np.testing.assert_array_equal(got, want)
    with no_host_copy(xd, gd):   # x comes down through the native download, not through torch
        np.testing.assert_array_equal(stein_thinning.thin(xd, gd, 30, preconditioner='med'), want)


def test_thin_on_device_tensors_with_repeats_and_near_ties():
    """MCMC-like input (runs of repeated rows): the guarded drop-in thins the run starts on the device."""
    n = 80_000
    rng = np.random.default_rng(3)
    base = rng.normal(size=(n // 4, 4))
    x = np.repeat(base, 4, axis=0)
    g = -x
    xd, gd = torch.from_numpy(x).cuda(), torch.from_numpy(g).cuda()
    with no_host_copy(xd, gd):
        got = stein_thinning.thin(xd, gd, 25)
    np.testing.assert_array_equal(got, o.thin(x, g, 25))


def test_thin_gf_on_device_tensors():
    n = 70_001
    x, g = _data(n, 4, seed=8)
    log_p = -0.5 * np.sum(x * x, axis=1)
    log_q = -0.45 * np.sum(x * x, axis=1)
    xd, gd = torch.from_numpy(x).cuda(), torch.from_numpy(g).cuda()
    lp, lq = torch.from_numpy(log_p).cuda(), torch.from_numpy(log_q).cuda()   # n-length: host weights
    with no_host_copy(xd, gd):
        got = stein_thinning.thin_gf(xd, lp, lq, gd, 20, preconditioner='med')
    np.testing.assert_array_equal(got, o.thin_gf(x, log_p, log_q, g, 20, preconditioner='med'))


def test_device_tensor_errors():
    """The reference's ValueErrors, NaN before inf, either array, as _validate_and_standardize raises them."""
    n = 70_000
    x, g = _data(n, 4, seed=1)
    cases = []
    a, b = x.copy(), g.copy(); a[5, 1] = np.nan; cases.append((a, b, 'NaNs'))
    a, b = x.copy(), g.copy(); b[n - 1, 3] = np.inf; cases.append((a, b, 'infs'))
    a, b = x.copy(), g.copy(); a[7, 0] = -np.inf; b[60_000, 2] = np.nan; cases.append((a, b, 'NaNs'))
    a, b = x.copy(), g.copy(); b[9, 0] = np.nan; a[:, 2] = 1.5; cases.append((a, b, 'NaNs'))
    a, b = x.copy(), g.copy(); a[:, 2] = 1.5; cases.append((a, b, 'Too few unique samples'))
    for a, b, msg in cases:
        with pytest.raises(ValueError, match=msg):
            o.thin(a, b, 5)
        ad, bd = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
        with pytest.raises(ValueError, match=msg):
            with no_host_copy(bd):
                stein_thinning.thin(ad, bd, 5)


def test_device_tensor_other_kinds():
    """A non-contiguous tensor (a device copy), small n, float32 (the host route): the same indices."""
    x, g = _data(70_001, 4, seed=11)
    want = o.thin(x, g, 12, preconditioner='med')
    xd, gd = torch.from_numpy(x).cuda(), torch.from_numpy(g).cuda()
    xt = torch.from_numpy(np.ascontiguousarray(x.T)).cuda().T   # non-contiguous view: a device copy
    gt = torch.from_numpy(np.ascontiguousarray(g.T)).cuda().T
    with no_host_copy(xt, gt):
        np.testing.assert_array_equal(stein_thinning.thin(xt, gt, 12, preconditioner='med'), want)
    assert st._download_standardized(xd.float(), gd.float()) is None
    small = _data(1000, 3, seed=2)
    xs, gs = torch.from_numpy(small[0]).cuda(), torch.from_numpy(small[1]).cuda()
    with no_host_copy(xs, gs):
        np.testing.assert_array_equal(stein_thinning.thin(xs, gs, 10), o.thin(small[0], small[1], 10))
    x1, g1 = _data(5001, 1, seed=4)
    x1d, g1d = torch.from_numpy(x1).cuda(), torch.from_numpy(g1).cuda()
    with no_host_copy(x1d, g1d):
        np.testing.assert_array_equal(stein_thinning.thin(x1d, g1d, 10), o.thin(x1, g1, 10))


def test_thin_gf_d50_on_device_tensors():
    """Config 5's shape (d = 50, gradient-free), smaller n: the wide kernels on in-place tensors."""
    x, g = _data(20_001, 50, seed=50)
    log_p = -0.5 * np.sum(x * x, axis=1)
    log_q = -0.45 * np.sum(x * x, axis=1)
    xd, gd = torch.from_numpy(x).cuda(), torch.from_numpy(g).cuda()
    with no_host_copy(xd, gd):
        got = stein_thinning.thin_gf(xd, log_p, log_q, gd, 10, preconditioner='med')
    np.testing.assert_array_equal(got, o.thin_gf(x, log_p, log_q, g, 10, preconditioner='med'))


def test_thin_chains_on_device_tensors():
    xs, gs = [], []
    for s in range(3):
        x, g = _data(70_000 + s, 2, seed=30 + s)
        xs.append(x)
        gs.append(g)
    xd = [torch.from_numpy(x).cuda() for x in xs]
    gd = [torch.from_numpy(g).cuda() for g in gs]
    with no_host_copy(*gd):
        got = stein_thinning.thin_chains(xd, gd, 15)
    for x, g, idx in zip(xs, gs, got):
        np.testing.assert_array_equal(idx, o.thin(x, g, 15))
