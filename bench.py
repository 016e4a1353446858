"""Benchmark of the Stein-thinning hot path on MI355X (BASELINE.json metric).

metric: Stein-kernel pair-evals/s + wall-clock to thin n=2e6 -> m=1e3, 1/2/4/8 GPU.
A "step" = one complete greedy thin of the HBM-resident standardised sample (diagonal + m-1 fused
kernel steps + argmin), i.e. n*m pair-evals; ms_per_step is the wall-clock of one thin.
N = 1 workload: config 4 of BASELINE.json (LV surrogate, d=4, n=2e6, Langevin IMQ, 'med', m=1000),
one launch of the persistent on-chip-resident kernel per thin (csrc/persistent.hip).
N > 1 (torchrun, one rank per GPU): the same n rows sharded across ranks (strong scaling); d = 2, 4:
one persistent launch per rank per thin, the ranks' per-step winners exchanged through IPC-mapped
device mailboxes over xGMI (stein_thinning/distributed.py PersistentShardedGreedy); other d (or if
the device exchange is unavailable): per-step kernels + RCCL all-gather of the rank records, the loop
captured in a HIP graph.  The mode used is reported in config.parallelism.

Synthetic data (no network): the LV posterior chains of the reference live only in S3, so the
"LV surrogate" is a seeded random-walk Metropolis chain on N(mu, Sigma) with mu, Sigma the
reference's printed LV chain-0 moments (Gradient_free.ipynb cells 42-43), isotropic step 0.0052
tuned to the reference chains' acceptance rate 0.23 (Sampling.ipynb cells 16, 28: ~77% duplicated
rows), ten pooled chains of 2e5 for n=2e6.
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd')
for _p in (ROOT, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

with open(os.path.join(ROOT, 'BASELINE.json')) as _f:
    BASELINE = json.load(_f)
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
LV_FLOP_PER_OBS = 106   # dense output per observation: 10 x quartic (8) + x (2) + residual (2) + C^-1 (6) + 4 x 4
FP64_VALU_PEAK_TFS = 78.6  # MI355X spec fp64 vector (256 CU x 4 SIMD x 16 FMA lanes x 2 x 2.4 GHz)

LV_MEAN = np.array([-0.38261842, 0.29176476, -0.02010969, -0.01824518])
LV_COV = np.array([
    [2.12987627e-04, 1.62995182e-04, -1.91636668e-04, -1.72343118e-04],
    [1.62995182e-04, 1.97250184e-04, -1.02375977e-04, -6.37599091e-05],
    [-1.91636668e-04, -1.02375977e-04, 2.16947410e-04, 2.13353024e-04],
    [-1.72343118e-04, -6.37599091e-05, 2.13353024e-04, 2.30906788e-04],
])
CHAIN_LEN = 200_000
RW_STEP = 0.0052   # acceptance ~0.23 as the reference RW-MH chains (Sampling.ipynb cell 28)


def lv_surrogate(n: int, seed: int, chain_len: int = CHAIN_LEN):
    """Pooled seeded RW-MH chains on N(LV_MEAN, LV_COV) -> (x, grad log p, log p, (log q, grad log q))."""
    from scipy.stats import multivariate_normal as mvn
    rng = np.random.default_rng(seed)
    chains = max(1, (n + chain_len - 1) // chain_len)
    steps = (n + chains - 1) // chains
    prec = np.linalg.inv(LV_COV)
    d = LV_MEAN.shape[0]

    def logp(z):
        zc = z - LV_MEAN
        return -0.5 * np.einsum('ij,jk,ik->i', zc, prec, zc)
    cur = LV_MEAN + rng.multivariate_normal(np.zeros(d), LV_COV, size=chains)
    lp = logp(cur)
    out = np.empty((steps, chains, d))
    noise = rng.normal(size=(steps, chains, d)) * RW_STEP
    logu = np.log(rng.random(size=(steps, chains)))
    for t in range(steps):
        prop = cur + noise[t]
        lpp = logp(prop)
        acc = logu[t] < lpp - lp
        cur = np.where(acc[:, None], prop, cur)
        lp = np.where(acc, lpp, lp)
        out[t] = cur
    x = np.ascontiguousarray(out.transpose(1, 0, 2).reshape(-1, d)[:n])
    grad = -(x - LV_MEAN) @ prec
    log_p = mvn.logpdf(x, mean=LV_MEAN, cov=LV_COV)
    mean = np.mean(x, axis=0)
    cov = np.cov(x, rowvar=False, ddof=d)      # Gradient_free.ipynb cell 41 (ddof = d)
    log_q = mvn.logpdf(x, mean=mean, cov=cov)
    grad_q = -np.einsum('ij,kj->ki', np.linalg.inv(cov), x - mean)
    return x, grad, log_p, (log_q, grad_q)


def lv_call_shape(n: int, seed: int, shape: str):
    """The reference's own LV thinning calls on one RW-MH chain (Stein_thinning.ipynb cells 12, 14;
    n ~ 5e5 per chain, Sampling.ipynb cells 16-18): the chain lives on the log-parameters s and the
    gradients on theta = exp(s), so
      shape 'exp': thin(np.exp(s), grads, 10_000, preconditioner='med')          (json :204)
      shape 'log': thin(s, np.exp(s) * grads, 10_000, preconditioner='med')     (json :264)
    Surrogate: s = one RW-MH chain on N(LV_MEAN, LV_COV) (log space) and grads = d log p / d theta =
    (d log p / d s) / theta (the log-space score divided by the chain rule's factor).  Returns the
    (sample, gradient) pair the call passes."""
    s, gs, _, _ = lv_surrogate(n, seed, chain_len=n)
    theta = np.exp(s)
    grads = gs / theta
    if shape == 'exp':
        return theta, grads
    if shape == 'log':
        return s, np.exp(s) * grads
    raise ValueError(shape)


def gaussian_d50(n: int, seed: int, d: int = 50, rho: float = 0.5):
    """Config 5: iid N(0, AR(1) rho) in d=50; gradient-free with q = N(mean, 1.2 cov)."""
    from scipy.stats import multivariate_normal as mvn
    rng = np.random.default_rng(seed)
    cov = rho ** np.abs(np.subtract.outer(np.arange(d), np.arange(d)))
    x = rng.multivariate_normal(np.zeros(d), cov, size=n, method='cholesky')
    log_p = mvn.logpdf(x, mean=np.zeros(d), cov=cov)
    mean = np.mean(x, axis=0)
    qcov = 1.2 * np.cov(x, rowvar=False)
    log_q = mvn.logpdf(x, mean=mean, cov=qcov)
    grad_q = -np.einsum('ij,kj->ki', np.linalg.inv(qcov), x - mean)
    return x, log_p, log_q, grad_q


CONFIGS = {
    'c2': dict(desc='LV-surrogate d=4 n=2e5 Langevin IMQ med m=100', n=200_000, m=100, gf=False, seed=12347),
    'c3': dict(desc='LV-surrogate d=4 n=2e5 gradient-free IMQ med m=100', n=200_000, m=100, gf=True, seed=12348),
    'c4': dict(desc='LV-surrogate pooled d=4 n=2e6 Langevin IMQ med m=1000', n=2_000_000, m=1000, gf=False, seed=12345),
    'c5': dict(desc='Gaussian AR(1) d=50 n=5e5 gradient-free IMQ med m=500', n=500_000, m=500, gf=True, seed=12349,
               d50=True),
    # one rank's share of an 8-GPU config-4 run (2.5e5 rows, m = 1000): the per-GPU load of that run,
    # for the same-device rehearsals of the rank exchange (DESIGN.md section 5 cost model)
    'c4r8': dict(desc='LV-surrogate d=4 n=2.5e5 (one rank of 8 of config 4) Langevin IMQ med m=1000', n=250_000,
                 m=1000, gf=False, seed=12345),
    # the reference's LV call (not a BASELINE config): one chain of 5e5, m = 10 000, 'med'
    'lv': dict(desc="LV call shape: thin(np.exp(s), grads, 10_000, 'med') on one RW-MH chain n=5e5 "
                    "(Stein_thinning.ipynb:204)", n=500_000, m=10_000, gf=False, seed=12350, lv_shape='exp'),
    'lvlog': dict(desc="LV call shape, log space: thin(s, np.exp(s) * grads, 10_000, 'med'), n=5e5 "
                       "(Stein_thinning.ipynb:264)", n=500_000, m=10_000, gf=False, seed=12350, lv_shape='log'),
}


def _persistent_nt(n_shard: int, d: int) -> int:
    """Threads per block the persistent kernel picks by default (persistent.hip,
    launch_greedy_persistent: 512 above kNt512MinRows = 1280 rows per block, one block per CU)."""
    rows_per_block = -(-n_shard // 256)
    return 512 if d in (2, 4) and rows_per_block > 1280 else 256


def _persistent_label(n_shard: int, d: int, gf: bool, arithmetic: str, world: int) -> str:
    """The persistent kernel launch_greedy_persistent enqueues by default (persistent.hip): one device,
    512-thread blocks and at least 4 096 rows per block under the compact arithmetic -> the
    compact-only kernel (9 register rows per thread) with the general kernel gated behind it."""
    nt = _persistent_nt(n_shard, d)
    rows = -(-n_shard // 256)
    g = str(gf).lower()
    if world == 1 and nt == 512 and arithmetic == 'compact' and rows >= 8 * 512:
        return (f'greedy_persistent<{d},{g},9,512,1,compact,compact-only> (+ the general kernel gated behind '
                f'it: returns at once)')
    return f'greedy_persistent<{d},{g},RT,{nt}>'


def make_integrand(cfg):
    import warnings
    from stein_thinning import thinning as st
    if cfg.get('d50'):
        x, log_p, log_q, gq = gaussian_d50(cfg['n'], cfg['seed'])
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            return st._make_stein_gf_integrand(x, log_p, log_q, gq, preconditioner='med'), x, None
    if cfg.get('lv_shape'):
        x, g = lv_call_shape(cfg['n'], cfg['seed'], cfg['lv_shape'])
        return st._make_stein_integrand(x, g, preconditioner='med'), x, g
    x, g, log_p, (log_q, gq) = lv_surrogate(cfg['n'], cfg['seed'])
    if cfg['gf']:
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            return st._make_stein_gf_integrand(x, log_p, log_q, gq, preconditioner='med'), x, (log_p, log_q, gq)
    return st._make_stein_integrand(x, g, preconditioner='med'), x, g


def cpu_baseline(cfg, integrand, steps: int, gpu_idx=None, arith='compact'):
    """Host baselines on the same standardised input (test-infrastructure code, timed only):
    * primary (`value`): the NumPy restatement of the reference path (oracle/stein_numpy.py: the (d, n)
      transposed vfk0_imq, A += 2 col, np.argmin -- JAX_Stein_Thinning.ipynb:281-295, 354-361) for the
      diagonal + `steps` steps on one core (NumPy ufuncs are single-threaded), its rate extrapolated
      linearly in m (every step costs the same n pair-evaluations);
    * `c_port`: the C restatement (oracle/stein_ref.c sr_greedy_mt -- the kernels' bit model, rows split
      over host threads like the reference's process fan-out, code/src/utils/parallel.py:48-52) running the
      FULL m-step thin on the box's CPU share; its indices are compared with the GPU's."""
    from oracle import stein_numpy as ref
    from oracle import stein_ref_c
    s, g, w = integrand.sample, integrand.gradient, integrand.weights
    vfk0 = ref.make_imq(s, 'med')
    if w is None:
        def f(i1, i2):
            return vfk0(s[i1], s[i2], g[i1], g[i2])
    else:
        def f(i1, i2):
            return vfk0(s[i1], s[i2], g[i1], g[i2]) * w[i1] * w[i2]
    steps = min(steps, cfg['m'] - 1)
    t0 = time.perf_counter()
    np_idx = ref._greedy_search(steps + 1, f)
    dt = time.perf_counter() - t0
    pairs = cfg['n'] * (steps + 1)
    full = cfg['n'] * cfg['m']
    nt = stein_ref_c.host_threads()
    t0 = time.perf_counter()
    cidx, _ = stein_ref_c.greedy_mt(s, g, w, integrand.linv_scale, integrand.linv_trace, cfg['m'], nt, arith=arith)
    dt_c = time.perf_counter() - t0
    host = f"{platform.processor() or platform.machine()} ({os.cpu_count()} logical CPUs visible)"
    share = ('the box\'s CPU share for its one GPU: the pool sets OMP_NUM_THREADS=16 and allows '
             '16 CPUs per GPU, while os.cpu_count() reports the whole host' if os.environ.get('OMP_NUM_THREADS') == '16'
             else f'OMP_NUM_THREADS / os.cpu_count() on this host')
    return {'value': pairs / dt, 'unit': 'pair-evals/s', 'cores': 1, 'kind': 'port',
            'sample': (f"oracle.stein_numpy._greedy_search (NumPy restatement of the reference path, "
                       f"JAX_Stein_Thinning.ipynb:281-295) on the same standardised sample: diagonal + {steps} steps "
                       f"= {pairs:.3g} pair-evals in {dt:.1f} s on one core (NumPy ufuncs are single-threaded); the "
                       f"full n={cfg['n']}, m={cfg['m']} thin extrapolated linearly: {full * dt / pairs:.0f} s; NumPy "
                       f"{np.__version__}; host {host}"),
            'same_indices_as_gpu_prefix': None if gpu_idx is None else bool(np.array_equal(np_idx, gpu_idx[:steps + 1])),
            'c_port': {'value': full / dt_c, 'unit': 'pair-evals/s', 'cores': nt, 'cores_reason': share,
                       'sample': (f"oracle/stein_ref.c sr_greedy_mt (C restatement of the reference greedy loop, "
                                  f"the kernels' bit model, {arith} arithmetic) on {nt} host threads: the full "
                                  f"thin ({full:.3g} pair-evals) in {dt_c:.1f} s"),
                       'same_indices_as_gpu': None if gpu_idx is None else bool(np.array_equal(cidx, gpu_idx))}}


def kernel_timing(prob, n_points: int, repeats: int = 5):
    """Average duration of the fused step kernel: HIP events on the launch stream bracket a run of
    back-to-back single-step launches (st_greedy_steps t = 1 .. n_points-1, no other work in
    between), averaged per launch -- the quantity rocprofv3's kernel-trace average reports."""
    import torch
    from stein_thinning import _native as nat
    L = nat.lib()
    idx, a, ws = prob.greedy_buffers(n_points)
    stream = torch.cuda.current_stream()

    def steps(t0, t1):
        nat.check(L.st_greedy_steps(nat.ptr(prob.x), nat.ptr(prob.g), nat.ptr(prob.w), prob.n, prob.d, prob.ld,
                                    prob.l, prob.tr, t0, t1, n_points, nat.ptr(idx), nat.ptr(a), nat.ptr(ws),
                                    ws.numel() * 8, nat.stream_handle()), 'st_greedy_steps')
    per = []
    for _ in range(repeats):
        steps(0, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        steps(1, n_points - 1)
        e1.record(stream)
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) * 1e-3 / (n_points - 2))
    return float(np.mean(per)), float(np.median(per))


def dedup_timing(prob, m: int, want_idx, stream, repeats: int = 5):
    """The drop-in thin's repeated-row path on the resident problem (DeviceProblem.dedup_view; not
    `value`, which evaluates all n m pairs): run detection + compaction timed with the host clock
    around a synchronised call (second of two, caches reset), then the thin of the run starts timed
    with HIP events like the headline run, and whether its mapped-back indices equal the timed run's."""
    import torch
    det = []
    for _ in range(2):
        prob._dedup = False
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        view = prob.dedup_view()
        torch.cuda.synchronize()
        det.append(time.perf_counter() - t0)
    if view is None:
        return {'rows_kept': prob.n, 'of': prob.n, 'used': False, 'detect_s': round(det[-1], 6),
                'note': 'fewer than 10 % of the rows repeat their predecessor: the drop-in thin evaluates all rows'}
    sp = view.problem
    idx, a, ws = sp.greedy_buffers(m)
    sp.greedy_launch(m, idx, a, ws)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(repeats)]
    for e0, e1 in evs:
        e0.record(stream)
        sp.greedy_launch(m, idx, a, ws)
        e1.record(stream)
    torch.cuda.synchronize()
    med = float(np.median([e0.elapsed_time(e1) * 1e-3 for e0, e1 in evs]))
    got = view.to_rows(idx.cpu().numpy().view(np.uint32))
    from stein_thinning import _native as nat
    try:   # the near-tie guard's verdict on the run starts (the drop-in's path): -1 = no step flagged
        tie = nat.near_tie_step(ws)
    except nat.HipExtensionError:   # an older A/B build (ST_HIP_LIB) without the guard
        tie = None
    # the drop-in's own rule (DeviceProblem.greedy: dedup_pays before and after detection; the guard does not
    # force it since round 6 -- repeated rows never flag a step)
    return {'used': True, 'drop_in_takes_it': bool(prob.dedup_pays(m) and prob.dedup_pays(m, sp.n)),
            'near_tie_step': tie,
            'rows_kept': sp.n, 'of': prob.n, 'detect_s': round(det[-1], 6),
            'thin_s': round(med, 6), 's_per_thin_incl_detect': det[-1] + med,
            'pair_evals_per_thin': sp.n * m,
            'same_indices_as_timed_run': bool(np.array_equal(got, want_idx)),
            'note': 'rows that repeat their predecessor bit for bit (rejected MCMC proposals) tie with their run '
                    'start in every evaluation and lose the tie to its lower index, so the thin of the run '
                    'starts selects the same rows (stein_thinning.device.DeviceProblem.dedup_view)'}


def _set_guard(enabled) -> bool:
    """stein_thinning's near-tie guard switch; False when the library predates it (an A/B build loaded
    through ST_HIP_LIB), which then runs unguarded whatever is asked."""
    from stein_thinning import _native as nat
    try:
        nat.set_near_tie_guard(enabled)
        return True
    except ValueError:
        return False


def rank_local_ms(integrand, m: int, rank: int, world: int, reps: int = 3):
    """ms per thin of this rank's shard ALONE on its GPU: the persistent kernel the rank runs (the
    single-device compact-only variant switched off) over rows shard_bounds(n, rank, world), no rank
    exchange (HIP events on the launch stream, median) -- T_local of DESIGN.md section 5's cost model
    T(N) = T_local(n / N) + H(N) + X."""
    import torch
    from stein_thinning import distributed as sd
    from stein_thinning import _native as nat
    lo, hi = sd.shard_bounds(integrand.n, rank, world)
    prob = integrand.device_problem().subset(np.arange(lo, hi))
    idx, a, ws = prob.greedy_buffers(m)
    L = nat.lib()
    prev = L.st_tune_get(12)
    # the kernel a rank runs: the compact-only variant is single-device only (st_tune key 12 off here)
    nat.check(L.st_tune(12, 0), 'st_tune')
    try:
        prob.greedy_launch(m, idx, a, ws)
        stream = torch.cuda.current_stream()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for e0, e1 in evs:
            e0.record(stream)
            prob.greedy_launch(m, idx, a, ws)
            e1.record(stream)
        torch.cuda.synchronize()
    finally:
        nat.check(L.st_tune(12, prev), 'st_tune')
    return float(np.median([e0.elapsed_time(e1) for e0, e1 in evs]))


def rank_hop(ms_sharded: float, integrand, m: int, rank: int, world: int, dev):
    """The measured rank level per step: (the sharded thin - the slowest rank's shard alone) / m -- H(N) + X
    of DESIGN.md section 5 (the rank winner's push over xGMI, the peers' polls, the candidate rows and the
    R-way pick), in one number, on the hardware the run is on.  Collective."""
    local = _max_over_ranks([rank_local_ms(integrand, m, rank, world)], dev)[0]
    return {'us_per_step': round((ms_sharded - local) / m * 1e3, 3), 'local_ms_per_thin': round(local, 4),
            'sharded_ms_per_thin': round(ms_sharded, 4),
            'note': '(sharded thin - the slowest rank\'s shard thinned alone on its GPU) / m: the rank exchange '
                    '(H + X of DESIGN.md section 5) per step' +
                    (' -- ranks SHARE one GPU here (rehearsal): no xGMI in it' if SHARE_DEVICE else '')}


def config5_sharded(rank: int, world: int, dev, steps: int = 3):
    """Config 5 (d = 50, gradient-free, n = 5e5, m = 500: the workload that shards)
    on the same ranks: ms per thin (max over ranks, barrier-bracketed), the per-rank launch median, its
    fp64 VALU fraction and the measured rank hop.  Collective; nulls at one rank."""
    nulls = {'ms_per_thin': None, 'kernel_median_us': None, 'frac': None, 'engine': None, 'rank_hop': None,
             'note': 'measured only when bench.py runs on N > 1 ranks'}
    if world == 1:
        return nulls
    import torch
    import torch.distributed as dist
    from stein_thinning import distributed as sd
    cfg = CONFIGS['c5']
    n, m = cfg['n'], cfg['m']
    integrand, _, _ = make_integrand(cfg)
    runner = sd.sharded_runner(integrand, m)   # collective; one validated run
    runner.launch()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        runner.launch()
        e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    dist.barrier()
    med = float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])) * 1e-3
    elapsed, med = _max_over_ranks([elapsed, med], dev)
    flop = algorithmic_flop_per_pair(50, True)
    tflops = n * m / world * flop / med / 1e12
    ms = elapsed / steps * 1e3
    return {'ms_per_thin': round(ms, 4), 'kernel_median_us': round(med * 1e6, 1),
            'frac': round(tflops / FP64_VALU_PEAK_TFS, 4), 'achieved_TFs': round(tflops, 2),
            'engine': runner.mode, 'n': n, 'd': 50, 'm': m, 'steps': steps,
            'rank_hop': rank_hop(ms, integrand, m, rank, world, dev) if runner.mode == 'device-exchange' else None,
            'note': f"config 5 ({cfg['desc']}) row-sharded over the same ranks; frac = algorithmic fp64 "
                    f"({flop} flop per pair) per rank / the rank's launch median / {FP64_VALU_PEAK_TFS} TF"}


def lv_chains(count: int, n: int, seed: int):
    """`count` RW-MH surrogate chains of n rows each in the reference's LV call shape ('exp', lv_call_shape),
    generated side by side (one vectorised lv_surrogate pool, chain-major): [(sample, gradient), ...]."""
    s, gs, _, _ = lv_surrogate(count * n, seed, chain_len=n)
    out = []
    for c in range(count):
        sc, gc = s[c * n:(c + 1) * n], gs[c * n:(c + 1) * n]
        theta = np.exp(sc)
        out.append((theta, gc / theta))
    return out


def chains_over_gpus(rank: int, world: int, dev, chains: int = 5, reps: int = 3):
    """The reference's own multi-device split: its notebook thins each of the 5 LV
    chains (n ~ 5e5 -> m = 10 000, 'med', Stein_thinning.ipynb:202-204) in a worker per chain
    (code/src/utils/parallel.py:48-52).  Here chain c goes to rank c % world; every rank thins its chains
    with the drop-in path on its own GPU (device.greedy_concurrent: repeated rows dropped, near-tie guard
    on, one batch launch per GPU).  Timed barrier to barrier, max over ranks, median of `reps`; beside it
    ONE GPU thinning all the chains in one batch launch (rank 0 alone), and the indices of both compared
    with the per-chain loop (rank 0: DeviceProblem.greedy one chain after the other).  Collective; nulls
    at one rank."""
    nulls = {'ms_per_chains': None, 'one_gpu_batch_ms': None, 'speedup_vs_one_gpu': None,
             'same_indices_as_loop': None, 'note': 'measured only when bench.py runs on N > 1 ranks'}
    if world == 1:
        return nulls
    import torch
    import torch.distributed as dist
    from stein_thinning import device as sdev
    from stein_thinning import thinning as st
    from stein_thinning import _native as nat
    n, m = 500_000, 10_000
    mine = [c for c in range(chains) if c % world == rank]
    data = lv_chains(chains, n, 20_500) if rank == 0 else None
    if rank != 0:   # the same chains on every rank (one seeded pool; generated where needed)
        data = lv_chains(chains, n, 20_500) if mine else []
    probs = {c: st._make_stein_integrand(*data[c], preconditioner='med').device_problem() for c in mine}
    guard = nat.near_tie_guard()

    import contextlib
    # rehearsal (ranks sharing one GPU): each rank's batch grid within its 256 / world CUs, so the ranks'
    # persistent grids co-reside
    share = nat.grid_cap(max(1, 256 // world // max(1, len(mine)))) if SHARE_DEVICE else contextlib.nullcontext()

    def run_mine():
        for p in probs.values():
            p._dedup = False   # run detection inside the timed region
        with share:
            return sdev.greedy_concurrent([probs[c] for c in mine], m, dedup=True, guard=guard) if mine else []
    got = dict(zip(mine, run_mine()))   # warm-up
    times = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got = dict(zip(mine, run_mine()))
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        dist.barrier()
    ms = _max_over_ranks([float(np.median(times)) * 1e3], dev)[0]
    parts = [None] * world
    dist.all_gather_object(parts, {c: v.tolist() for c, v in got.items()})
    one_ms, same = None, None
    if rank == 0:
        allp = [probs[c] if c in probs else st._make_stein_integrand(*data[c], preconditioner='med').device_problem()
                for c in range(chains)]
        loop = [p.greedy(m, dedup=True, guard=guard) for p in allp]
        one = []
        for _ in range(2):
            for p in allp:
                p._dedup = False
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            batch_idx = sdev.greedy_concurrent(allp, m, dedup=True, guard=guard)
            torch.cuda.synchronize()
            one.append(time.perf_counter() - t0)
        one_ms = float(np.median(one)) * 1e3
        spread = {c: np.asarray(v, dtype=np.uint32) for part in parts for c, v in part.items()}
        same = bool(all(np.array_equal(spread[c], loop[c]) and np.array_equal(batch_idx[c], loop[c])
                        for c in range(chains)))
    dist.barrier()
    return {'ms_per_chains': round(ms, 3), 'one_gpu_batch_ms': round(one_ms, 3) if one_ms else None,
            'speedup_vs_one_gpu': round(one_ms / ms, 3) if one_ms else None, 'chains': chains,
            'chains_per_rank': [len([c for c in range(chains) if c % world == r]) for r in range(world)],
            'n_per_chain': n, 'm': m, 'near_tie_guard': guard, 'same_indices_as_loop': same,
            'note': 'the reference\'s fan-out (one chain per worker, code/src/utils/parallel.py:48-52): chain c on '
                    'rank c % world, each GPU thinning its chains with the drop-in path (run starts, near-tie guard, '
                    'one batch launch); ms = barrier to barrier, max over ranks; one_gpu_batch_ms = all chains in '
                    'one batch launch on rank 0\'s GPU; indices of both against the per-chain loop' +
                    (' -- ranks SHARE one GPU here (rehearsal)' if SHARE_DEVICE else '')}


# Rehearsal mode (ST_BENCH_SHARE_DEVICE=1, never used by the driver): every rank on cuda:0 and a
# gloo group, so the N > 1 flow (mailbox setup, device exchange, timing reductions) can run on a
# one-GPU box with several processes sharing the device.
SHARE_DEVICE = os.environ.get('ST_BENCH_SHARE_DEVICE') == '1'


def _setup_ranks():
    import torch
    rank = int(os.environ.get('RANK', 0))
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = 0 if SHARE_DEVICE else int(os.environ.get('LOCAL_RANK', 0))
    torch.cuda.set_device(local)
    return rank, world, torch.device('cuda', local)


def _init_group(dev):
    import torch.distributed as dist
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29531')
    os.environ.setdefault('RANK', os.environ.get('RANK', '0'))
    os.environ.setdefault('WORLD_SIZE', os.environ.get('WORLD_SIZE', '1'))
    if SHARE_DEVICE:
        dist.init_process_group('gloo')
    else:
        dist.init_process_group('nccl', device_id=dev)


def _max_over_ranks(values, dev):
    """Element-wise max over ranks of a list of floats (RCCL, or gloo on host tensors)."""
    import torch
    import torch.distributed as dist
    on = dev if dist.get_backend() == 'nccl' else torch.device('cpu')
    t = torch.tensor(values, dtype=torch.float64, device=on)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def pmc_traffic(key: str):
    """HBM bytes per launch of a workload's dominant kernel from the committed PMC summary
    (profiles/pmc_traffic.json, written by tools/summarize_pmc.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes with the gfx950 corrections), or None when no pass was recorded."""
    path = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    rec = (json.load(open(path)) if os.path.exists(path) else {}).get(key)
    return round(rec['hbm_bytes_per_launch']) if rec else None


def algorithmic_flop_per_pair(d: int, gf: bool) -> int:
    """Algorithmic fp64 work of one Stein-kernel pair, SURVEY.md section 8(d): 12 d + 40 flop
    (isotropic Gamma^-1; the per-coordinate products and sums of vfk0_imq,
    JAX_Stein_Thinning.ipynb:354-361, plus the constant tail of 2 pow, 1 sqrt, 3 divisions); the
    gradient-free weights w_i w_j add 2 multiplies.  88 at d = 4, 640 at d = 50.  This is the
    figure `roofline.frac` is priced on; the kernels' ISA count (correctly rounded powers in
    double-double, Newton steps of the divisions) is reported beside it as `issue`."""
    return 12 * d + 40 + (2 if gf else 0)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _launch_ranks(argv) -> int:
    """`--gpus N` without a launcher: run N ranks under torch.distributed.run as a child process
    (this process never touches the GPU) and return its exit code; rank 0 prints the JSON line."""
    import re
    m = re.search(r'--gpus[ =](\d+)', ' '.join(argv))
    n = int(m.group(1)) if m else 1
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={n}',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


def main():
    faulthandler.enable()   # a crash (e.g. under rocprofv3) leaves the Python stack in the log
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5, help='timed thins')
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--config', default='c4', choices=sorted(CONFIGS))
    ap.add_argument('--cpu-steps', type=int, default=100, help='greedy steps of the NumPy one-core sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-kernel-timing', action='store_true')
    ap.add_argument('--no-e2e', action='store_true', help='skip the end_to_end legs (drop-in thin on host arrays)')
    ap.add_argument('--no-graph', action='store_true', help='N > 1: eager per-step launches instead of a HIP graph')
    ap.add_argument('--sharded', action='store_true', help='use the sharded (RCCL) path even at N = 1')
    ap.add_argument('--no-config5', action='store_true',
                    help='thin workload at N > 1: skip the config5_sharded object (config 5 row-sharded)')
    ap.add_argument('--no-chains', action='store_true',
                    help='thin workload at N > 1: skip the chains_over_gpus object (the 5 LV chains over the ranks)')
    ap.add_argument('--ksd-full', action='store_true', help='ksd workload on config 4 (n = 2e6) instead of config 2')
    ap.add_argument('--proxy-kind', default='gauss', choices=['gauss', 't'], help='proxy workload: Gaussian or Student-t')
    ap.add_argument('--lv-mode', type=int, default=0, help='lv workload: 0 two-phase (default), 1 single-phase')
    ap.add_argument('--lv-global-obs', type=int, default=0,
                    help='lv workload: 1 = phase B reads the observations from global memory (st_tune key 17)')
    ap.add_argument('--lv-pieces', type=int, default=-1,
                    help='lv workload: phase-B observation pieces per lane (st_tune key 18; -1 = auto)')
    ap.add_argument('--proxy-mode', type=int, default=0, help='proxy kernel (st_tune key 7; 0 = auto)')
    ap.add_argument('--energy-variant', type=int, default=0, help='energy kernel (st_tune key 13; 0 = auto)')
    ap.add_argument('--energy-units', type=int, default=-1,
                    help='energy kernel work units per launch (st_tune key 14; -1 = auto)')
    ap.add_argument('--headline-guard', action='store_true',
                    help='thin workload: time the headline thin with the near-tie guard on (default off: the guard is '
                         'timed beside it, "near_tie_guard")')
    ap.add_argument('--arith', default='compact', choices=['compact', 'exact'],
                    help='arithmetic of the d <= 8 greedy kernels (stein_thinning.set_arithmetic)')
    ap.add_argument('--chains', type=int, default=5,
                    help='chains workload: independent chains thinned (5 = lotka_volterra.n_chains, code/src/lotka_volterra.py:67-75)')
    ap.add_argument('--batch', type=int, default=-1,
                    help='chains workload: problems per st_greedy_batch launch (1 = streams only; -1 = device.BATCH)')
    ap.add_argument('--in-flight', type=int, default=-1,
                    help='chains workload: thins in flight at once (-1 = stein_thinning.device.IN_FLIGHT)')
    ap.add_argument('--workload', default='thin', choices=['thin', 'ksd', 'proxy', 'lv', 'energy', 'ranks', 'chains'],
                    help='thin: the headline greedy thin (default); ksd: full-sample cumulative KSD '
                         '(row-sharded, RCCL all-reduce of the n-length column-sum vector); ranks: launcher '
                         'check only (gloo, no GPU)')
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error('--gpus must be >= 1')
    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and args.gpus > 1:
        return _launch_ranks(sys.argv[1:])
    if env_world is not None and int(env_world) != args.gpus:
        print(f'bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}', file=sys.stderr)
        return 2
    if args.workload == 'ranks':
        return main_ranks(args)
    if args.workload == 'energy':
        return main_energy(args)
    if args.workload == 'ksd':
        return main_ksd(args)
    if args.workload == 'proxy':
        return main_proxy(args)
    if args.workload == 'lv':
        return main_lv(args)
    if args.workload == 'chains':
        return main_chains(args)

    import torch
    import torch.distributed as dist
    rank, world, dev = _setup_ranks()
    sharded = world > 1 or args.sharded
    if sharded and not dist.is_initialized():
        _init_group(dev)
    if SHARE_DEVICE and world > 1:
        from stein_thinning import _native as nat
        nat.lib().st_tune(5, 256 // world)   # the ranks' persistent grids must co-reside on one GPU

    cfg = CONFIGS[args.config]
    n, m = cfg['n'], cfg['m']
    if os.environ.get('ST_TUNE'):   # measurement sweeps: "key=value,key=value" st_tune settings
        from stein_thinning import _native as nat
        for kv in os.environ['ST_TUNE'].split(','):
            k, v = kv.split('=')
            nat.check(nat.lib().st_tune(int(k), int(v)), 'ST_TUNE')
    integrand, host_x, host_g = make_integrand(cfg)
    d = integrand.sample.shape[1]
    import stein_thinning
    stein_thinning.set_arithmetic(args.arith)
    arithmetic = args.arith
    from stein_thinning import _native as nat
    # the headline leg: st_greedy over all n rows as the kernel computes them (compact arithmetic: no
    # near-tie flag, unless --headline-guard).  The drop-in thin's default (guard on) is timed beside it:
    # "near_tie_guard" (all rows) and "dedup" (the run starts, the drop-in's path on repeated rows).
    _set_guard(bool(args.headline_guard))

    if not sharded:
        prob = integrand.device_problem()
        idx, a, ws = prob.greedy_buffers(m)

        def run_once():
            prob.greedy_launch(m, idx, a, ws)
    else:
        from stein_thinning import distributed as sd
        # collective; completes one (untimed) validation run of the chosen exchange engine
        runner = sd.sharded_runner(integrand, m, use_graph=not args.no_graph)

        def run_once():
            runner.launch()

    for _ in range(args.warmup):
        run_once()
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()   # st_greedy / graph replays are enqueued on it
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        run_once()
        e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    launch_s = [e0.elapsed_time(e1) * 1e-3 for e0, e1 in evs]
    if sharded:
        dist.barrier()
        elapsed = _max_over_ranks([elapsed], dev)[0]

    if not sharded:
        result_idx = idx.cpu().numpy().view(np.uint32)
    else:
        result_idx = runner.indices() if hasattr(runner, 'indices') else runner.backend.indices()
    # N > 1: the measured rank level of this run and config 5 sharded (nulls at N = 1)
    hop, c5 = None, config5_sharded(rank, 1, dev)
    if sharded and world > 1 and runner.mode == 'device-exchange':
        hop = rank_hop(elapsed / args.steps * 1e3, integrand, m, rank, world, dev)
    if sharded and world > 1 and not args.no_config5 and args.config == 'c4':
        c5 = config5_sharded(rank, world, dev)
    cog = chains_over_gpus(rank, 1, dev)
    if sharded and world > 1 and not args.no_chains and args.config == 'c4':
        _set_guard(None)   # the drop-in default (guard on unless ST_NEAR_TIE=0), as the reference's call gets it
        cog = chains_over_gpus(rank, world, dev)
        _set_guard(bool(args.headline_guard))

    roofline = None
    cpu = None
    persistent = (d in (2, 4) and not sharded) or (sharded and runner.mode == 'device-exchange')
    if rank == 0 or sharded:
        gf = integrand.weights is not None
        bytes_per_pair = 16 * d + (24 if gf else 16)
        # algorithmic work per pair: what `frac` is priced on
        flop_per_pair = algorithmic_flop_per_pair(d, gf)
        # what the persistent kernel's hot loop actually issues, counted in its ISA.  Compact
        # arithmetic (the default, stein_math.hpp pair_compact_ct): 8 v_mul_f64 + 9 v_add_f64 + 25
        # v_fma/v_fmac_f64 (running-sum update included) + 1 v_rsq_f64 + 1 v_cmp_f64 = 44 fp64 VALU
        # instructions, 67 flop (fma = 2); each further coordinate adds 5 (2 sub + 3 fma, 8 flop).
        # Exact arithmetic (ST_ARITH=exact): 40 mul + 28 add + 31 fma + 1 rsq + 1 cmp = 101, 130 flop;
        # each further coordinate adds 13.  The gradient-free weights add 2 mul.
        if arithmetic == 'compact' and d <= 8:
            instr_per_pair = 44 + 5 * (d - 4) + (2 if gf else 0)
            issue_flop_per_pair = 67 + 8 * (d - 4) + (2 if gf else 0)
        else:
            instr_per_pair = 101 + 13 * (d - 4) + (2 if gf else 0)
            issue_flop_per_pair = 130 + 13 * (d - 4) + (2 if gf else 0)
        pmc = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
        pmc_rec = json.load(open(pmc)) if os.path.exists(pmc) else {}
        if persistent:
            # dominant kernel = the single persistent launch that runs the whole thin (per rank);
            # its duration = HIP events on the launch stream around each timed thin (includes the
            # ~2 us workspace memset enqueued just before it); max over ranks
            avg = float(np.mean(launch_s))
            med = float(np.median(launch_s))
            if sharded:
                avg, med = _max_over_ranks([avg, med], dev)
            pairs_launch = n * m / world          # per rank
            tflops = pairs_launch * flop_per_pair / med / 1e12
            gins = pairs_launch * instr_per_pair / med / 1e12
            issue_peak = 256 * 4 * 16 * 2.4e9 / 1e12   # fp64 lane-instructions/s (T), 4 cycles per wave-instr
            alg_bytes = int(pairs_launch * bytes_per_pair)
            rec = pmc_rec.get(f'{args.config}_persistent') if world == 1 else None
            traffic = round(rec['hbm_bytes_per_launch']) if rec else None
            traffic_src = (f"profiles/pmc_traffic.json['{args.config}_persistent']: {rec.get('source', 'rocprofv3 --pmc pass')}"
                           f" of {rec['kernel']} (FETCH_SIZE / WRITE_SIZE, gfx950 corrections) -- a committed "
                           f"measurement of this workload, not taken in this run") if rec else None
            roofline = {
                'bound': 'valu', 'achieved': round(tflops, 2), 'peak': FP64_VALU_PEAK_TFS, 'unit': 'TFLOP/s',
                'frac': round(tflops / FP64_VALU_PEAK_TFS, 4), 'traffic': traffic, 'traffic_source': traffic_src,
                'kernel': _persistent_label(n // world, d, gf, arithmetic, world)
                          + (f' x{world} ranks' if sharded else ''),
                'kernel_median_us': round(med * 1e6, 1), 'kernel_avg_us': round(avg * 1e6, 1),
                'timing': f'median of HIP events on the launch stream around each of the {args.steps} timed '
                          'thins (the persistent launch(es) of one thin)' + (', max over ranks' if sharded else ''),
                'flop_per_pair': flop_per_pair,
                'flop_per_pair_source': 'SURVEY.md 8(d): 12 d + 40 (+2 gradient-free), algorithmic',
                'issue': {'fp64_instr_per_pair': instr_per_pair, 'isa_flop_per_pair': issue_flop_per_pair,
                          'achieved_TFs': round(pairs_launch * issue_flop_per_pair / med / 1e12, 2),
                          'achieved_Tinstr_s': round(gins, 2), 'peak_Tinstr_s': round(issue_peak, 2),
                          'frac': round(gins / issue_peak, 4)},
                'note': ('compute-bound: the persistent kernel keeps the rows in VGPR/AGPR/LDS across the m steps '
                         '(PMC traffic per launch = "traffic", far below the streaming figure), so the roofline is '
                         'fp64 VALU (MI355X fp64 vector peak 78.6 TF = fp64 matrix peak; no MFMA shape fits '
                         'the per-pair scalar work); part of each step is the in-launch winner exchange'),
                'hbm_view': {'measured_bytes_per_launch': traffic,
                             'measured_GBs': round(traffic / med / 1e9, 1) if traffic else None,
                             'peak_GBs': HBM_PEAK_GBS,
                             'measured_frac': round(traffic / med / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                             'streaming_design_bytes_per_launch': alg_bytes, 'bytes_per_pair': bytes_per_pair,
                             'note': 'HBM is not the bound: the rows stay on chip, so the kernel moves the measured '
                                     'bytes, not the streaming design\'s n m (16 d + 16) B (SURVEY 8(d)), which '
                                     'would exceed HBM peak at this kernel time'},
            }
        if not sharded and not args.no_kernel_timing:
            s_avg, s_med = kernel_timing(prob, min(m, 200))
            step = {
                'kernel': f'greedy_step_ct<{d}> (launch-per-step path, st_greedy_steps)' if d <= 8 else
                          'greedy_step_rt (launch-per-step path, st_greedy_steps)',
                'avg_us': round(s_avg * 1e6, 2), 'median_us': round(s_med * 1e6, 2),
                'achieved_GBs': round(n * bytes_per_pair / s_avg / 1e9, 1),
                'frac_hbm': round(n * bytes_per_pair / s_avg / 1e9 / HBM_PEAK_GBS, 4),
                'algorithmic_bytes_per_launch': n * bytes_per_pair}
            if persistent:
                roofline['step_kernel'] = step
            else:
                rec = pmc_rec.get(args.config)
                roofline = {'bound': 'hbm', 'achieved': step['achieved_GBs'], 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                            'frac': step['frac_hbm'], 'traffic': round(rec['hbm_bytes_per_launch']) if rec else None,
                            'kernel': step['kernel'], 'kernel_avg_us': step['avg_us'],
                            'kernel_median_us': step['median_us'],
                            'algorithmic_bytes_per_launch': step['algorithmic_bytes_per_launch'],
                            'bytes_per_pair': bytes_per_pair,
                            'timing': 'HIP events around back-to-back single-step launches'}
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(cfg, integrand, args.cpu_steps, result_idx, arithmetic)
        exact = None
        if world == 1 and not sharded and d <= 8 and arithmetic == 'compact':
            # the same thin with the exact arithmetic (NumPy's evaluation order; not `value`): its
            # time and whether it selects the same indices as the timed compact run
            import stein_thinning
            stein_thinning.set_arithmetic('exact')
            try:
                run_once()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
                for e0, e1 in ev:
                    e0.record(stream)
                    run_once()
                    e1.record(stream)
                torch.cuda.synchronize()
                exact_idx = idx.cpu().numpy().view(np.uint32)
                exact = {'ms_per_thin': round(float(np.median([a.elapsed_time(b) for a, b in ev])), 4),
                         'same_indices_as_timed_run': bool(np.array_equal(exact_idx, result_idx))}
            finally:
                stein_thinning.set_arithmetic('compact')
                run_once()   # leave the buffers as the timed (compact) run left them
                torch.cuda.synchronize()
        guarded = None
        guard_lib = _set_guard(None)   # the drop-in default from here on (ST_NEAR_TIE, on unless '0')
        if world == 1 and not sharded and d in (2, 4) and arithmetic == 'compact' and nat.near_tie_guard() \
                and guard_lib:
            # the same thin of all n rows with the near-tie guard (not `value`): its time and first
            # flagged step (-1 none; rows that repeat their predecessor tie exactly, so a raw MCMC sample
            # is flagged at once -- the drop-in thins its run starts instead, "dedup")
            run_once()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
            for e0, e1 in ev:
                e0.record(stream)
                run_once()
                e1.record(stream)
            torch.cuda.synchronize()
            try:
                tie = nat.near_tie_step(ws)
            except nat.HipExtensionError:   # an older A/B build (ST_HIP_LIB) without the guard
                tie = None
            guarded = {'ms_per_thin': round(float(np.median([a.elapsed_time(b) for a, b in ev])), 4),
                       'first_flagged_step': tie,
                       'same_indices_as_timed_run': bool(np.array_equal(idx.cpu().numpy().view(np.uint32),
                                                                        result_idx)),
                       'note': 'st_greedy of all n rows with the near-tie guard (DESIGN.md section 1); a flagged '
                               'drop-in thin is re-run in the exact arithmetic ("exact_arithmetic")'}
        dedup = None
        if world == 1 and not sharded:
            dedup = dedup_timing(prob, m, result_idx, stream)
        e2e = None
        if world == 1 and not cfg['gf'] and not cfg.get('d50') and not args.no_e2e:
            # the drop-in call on host arrays (not `value`): standardisation + 'med' + H2D upload +
            # SoA layout + the persistent launch + D2H of the indices
            from stein_thinning import thinning as st
            st.thin(host_x, host_g, m, preconditioner='med')
            dts = []
            for _ in range(3):
                t_e = time.perf_counter()
                e2e_idx = st.thin(host_x, host_g, m, preconditioner='med')
                dts.append(time.perf_counter() - t_e)
            dt_e = float(np.median(dts))
            e2e = {'thin_host_arrays_s': round(dt_e, 4), 'runs_s': [round(v, 4) for v in dts],
                   'pair_evals_per_s': n * m / dt_e,
                   'same_indices_as_timed_run': bool(np.array_equal(e2e_idx, result_idx))}
            # the same call on ROCm tensors already on the GPU (the raw sample and gradient, row-major):
            # x comes down for its statistics and the 'med' subsample, g stays (thinning._download_standardized)
            xd = torch.from_numpy(np.ascontiguousarray(host_x)).to(dev)
            gd = torch.from_numpy(np.ascontiguousarray(host_g)).to(dev)
            torch.cuda.synchronize()
            try:
                st.thin(xd, gd, m, preconditioner='med')
                dts = []
                for _ in range(3):
                    t_e = time.perf_counter()
                    dev_idx = st.thin(xd, gd, m, preconditioner='med')
                    dts.append(time.perf_counter() - t_e)
                e2e['thin_device_tensors_s'] = round(float(np.median(dts)), 4)
                e2e['device_tensors_runs_s'] = [round(v, 4) for v in dts]
                e2e['device_tensors_same_indices'] = bool(np.array_equal(dev_idx, result_idx))
            except nat.HipExtensionError:   # an A/B build (ST_HIP_LIB) older than the device-tensor path
                e2e['thin_device_tensors_s'] = None
            del xd, gd

    exchange, degraded = None, False
    if sharded:
        # the engine the run was meant to use vs the one it ended on (a fallback after a failed
        # mailbox setup or an expired bounded wait is reported, never silent)
        engine = runner.engine
        want = {'persistent': 'device-exchange', 'steps': 'device-exchange-steps-graph',
                'replicated': 'replicated',
                'rccl': 'rccl-graph' if dist.get_backend() == 'nccl' else 'records-all-gather'}[engine]
        exchange = {'engine': engine, 'mode': runner.mode}
        degraded = runner.mode != want
        if degraded and rank == 0:
            print(f'bench.py: DEGRADED exchange: wanted {want}, ran {runner.mode}', file=sys.stderr)
    if rank == 0:
        pairs = float(n) * m * args.steps
        line = {
            'metric': BASELINE['metric'],
            'value': pairs / elapsed,
            'unit': 'pair-evals/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'f64',
            'data': 'synthetic (seeded RW-MH LV-surrogate chains; see bench.py docstring)',
            'config': {'workload': (f"config {args.config[1]}: {cfg['desc']}" if args.config in ('c2', 'c3', 'c4', 'c5') else cfg['desc']),
                       'n': n, 'd': d, 'm': m,
                       'preconditioner': 'med', 'kernel': 'gradient-free' if integrand.weights is not None else 'langevin',
                       'parallelism': (f'rows-sharded x{world}, per-step exchange: {runner.mode}'
                                       if sharded else 'single-gpu'),
                       'arithmetic': arithmetic if d <= 8 else 'exact',
                       'near_tie_guard': bool(args.headline_guard and d in (2, 4) and arithmetic == 'compact'
                                              and not sharded),
                       'wallclock_thin_s': {
                           'device_resident': elapsed / args.steps,
                           'device_resident_dedup': (round(dedup['s_per_thin_incl_detect'], 6)
                                                     if rank == 0 and dedup and dedup.get('used') else None),
                           'thin_host_arrays': e2e['thin_host_arrays_s'] if rank == 0 and e2e else None,
                           'note': 'device_resident = ms_per_step: the timed thin of the standardised sample '
                                   'already in HBM, every one of the n m pairs evaluated (value); '
                                   'device_resident_dedup = the same thin with repeated rows dropped first '
                                   '(run detection + compaction + the thin of the run starts: the drop-in '
                                   'thin\'s default, same indices; "dedup" below); thin_host_arrays = the drop-in '
                                   'thin(sample, gradient, m) on host NumPy arrays (validation, standardisation, '
                                   'med, H2D, dedup, launch, D2H), the median of three calls after the timed region'},
                       'first_indices': result_idx[:8].tolist()},
            'exchange': exchange,
            'degraded': degraded,
            'rank_hop': hop,
            'config5_sharded': c5,
            'chains_over_gpus': cog,
            'roofline': roofline,
            'cpu_baseline': cpu,
            'end_to_end': e2e if rank == 0 and not sharded else None,
            'exact_arithmetic': exact if rank == 0 and not sharded else None,
            'near_tie_guard': guarded if rank == 0 and not sharded else None,
            'dedup': dedup if rank == 0 and not sharded else None,
        }
        print(json.dumps(line), flush=True)
    if sharded:
        dist.destroy_process_group()


def thinned_sizes(n_points_calculate: int = 1000) -> np.ndarray:
    """Comparison.ipynb cell 21: 50 sizes on [5, 100] and 200 on [100, n_points_calculate]."""
    return np.concatenate([np.linspace(5, 100, 50).astype(int),
                           np.linspace(100, n_points_calculate, 200).astype(int)])


def main_chains(args):
    """The reference's per-chain LV thinning (Stein_thinning.ipynb cell 12: every RW-MH chain of
    n ~ 5e5 thinned on its own to m = 10 000 with 'med'; the fan-out is code/src/utils/parallel.py:48-52)
    for `--chains` seeded surrogate chains (default 5, the reference's n_chains; lv_call_shape 'exp'),
    standardised arrays resident on the
    GPU.  A step = all the chains' thins: one after the other (the loop the notebook runs) and side by
    side (stein_thinning.device.greedy_concurrent, each latency-bound thin on a share of the CUs);
    both drop repeated rows first (the drop-in thin's default), and the indices must agree.  `value`
    = chains thinned per second by greedy_concurrent; N > 1: the chains are dealt to the ranks."""
    import torch
    import torch.distributed as dist
    from stein_thinning import device as sdev
    from stein_thinning import thinning as st
    rank, world, dev = _setup_ranks()
    if world > 1:
        _init_group(dev)
    n, m = 500_000, 10_000
    mine = list(range(rank, args.chains, world))
    host = [lv_call_shape(n, 20_000 + k, 'exp') for k in mine]
    probs = [st._make_stein_integrand(x, g, preconditioner='med').device_problem() for x, g in host]
    in_flight = args.in_flight if args.in_flight > 0 else sdev.IN_FLIGHT
    batch = args.batch if args.batch > 0 else sdev.BATCH

    def run(c, b=batch):
        for p in probs:
            p._dedup = False   # run detection inside the timed region
        return sdev.greedy_concurrent(probs, m, in_flight=c, batch=b)
    seq = run(1)
    for _ in range(args.warmup):
        run(in_flight)
    times, seq_times = [], []
    for _ in range(args.steps):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got = run(in_flight)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    streams_times = []
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(1)
        torch.cuda.synchronize()
        seq_times.append(time.perf_counter() - t0)
        if batch > 1:   # the same on streams only (no batch launch), for comparison
            t0 = time.perf_counter()
            st_only = run(in_flight, 1)
            torch.cuda.synchronize()
            streams_times.append(time.perf_counter() - t0)
    # end to end from host arrays (standardisation, upload, preconditioner, thin): the drop-in loop of
    # thin() calls against thin_chains
    import stein_thinning
    e2e_loop, e2e_chains = [], []
    for _ in range(2):
        t0 = time.perf_counter()
        loop_idx = [stein_thinning.thin(x, g, m, preconditioner='med') for x, g in host]
        e2e_loop.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        ch_idx = stein_thinning.thin_chains([x for x, _ in host], [g for _, g in host], m, preconditioner='med')
        e2e_chains.append(time.perf_counter() - t0)
    same_e2e = all(np.array_equal(a, b) for a, b in zip(loop_idx, ch_idx)) and \
        all(np.array_equal(a, b) for a, b in zip(loop_idx, seq))
    same = all(np.array_equal(a, b) for a, b in zip(got, seq))
    if streams_times:
        same = same and all(np.array_equal(a, b) for a, b in zip(st_only, seq))
    elapsed = float(np.median(times))
    if world > 1:
        elapsed = _max_over_ranks([elapsed], dev)[0]
    if rank == 0:
        line = {'metric': 'independent chain thins per second (the reference LV call shape: n=5e5, m=1e4 per chain)',
                'value': args.chains / elapsed, 'unit': 'chains/s', 'n_gpus': world, 'steps': args.steps,
                'warmup': args.warmup, 'ms_per_step': elapsed * 1e3, 'higher_is_better': True, 'scaling': 'strong',
                'vs_baseline': None, 'dtype': 'f64',
                'data': 'synthetic (seeded RW-MH LV-surrogate chains, one per seed; see bench.py lv_call_shape)',
                'config': {'workload': f"{args.chains} chains x thin(np.exp(s), grads, 10_000, 'med')",
                           'n_per_chain': n, 'm': m, 'in_flight': in_flight, 'batch': batch,
                           'run_starts': [p.dedup_view().n_unique if p.dedup_view() is not None else p.n for p in probs],
                           'parallelism': f'chains dealt to {world} ranks' if world > 1 else 'single-gpu'},
                'one_after_the_other_ms': round(float(np.median(seq_times)) * 1e3, 2),
                'side_by_side_ms': round(elapsed * 1e3, 2),
                'streams_only_ms': round(float(np.median(streams_times)) * 1e3, 2) if streams_times else None,
                'e2e_from_host_arrays_ms': {'loop_of_thin': round(min(e2e_loop) * 1e3, 2),
                                            'thin_chains': round(min(e2e_chains) * 1e3, 2),
                                            'same_indices': bool(same_e2e)},
                'same_indices_as_one_after_the_other': bool(same)}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_energy(args):
    """The reference's fit_quality curve (Comparison.ipynb cells 19-23): sqrt(dcor.energy_distance(
    validation[::10], sample[idx[:k]])) for the 250 thinned sizes k of cell 21, on the config-4 scale:
    validation = a second seeded LV-surrogate pool of 2e6 points (the reference's validation HMC chains
    live in S3) taken [::10] -> 2e5 points; sample / idx = config 4's sample and its m = 1000 Stein
    thinning.  A step = one whole curve, inputs resident on the GPU (stein_thinning.energy.EnergyCurve:
    the validation set's triangle once, the cross block, the selection's triangle).  N > 1: replicas
    (each rank evaluates the whole curve; the reference evaluates one curve per chain and method)."""
    import torch
    import torch.distributed as dist
    from stein_thinning import energy as se
    from stein_thinning import thinning as st
    rank, world, dev = _setup_ranks()
    if world > 1:
        _init_group(dev)
    cfg = CONFIGS['c4']
    x, g, _, _ = lv_surrogate(cfg['n'], cfg['seed'])
    validation = lv_surrogate(cfg['n'], cfg['seed'] + 100)[0][::10]
    idx = st.thin(x, g, cfg['m'], preconditioner='med')
    sizes = thinned_sizes(cfg['m'])
    # headline: the whole curve per step, the validation triangle included (cache_reference=False);
    # `cached` below: the reference's loop over methods x chains, where that triangle is computed
    # once per validation sample (stein_thinning.energy.PointSet) and a curve is the cross block and
    # the selection's triangle
    from stein_thinning import _native as nat
    nat.check(nat.lib().st_tune(13, args.energy_variant), 'st_tune')
    nat.check(nat.lib().st_tune(14, args.energy_units), 'st_tune')
    curve = se.EnergyCurve(validation, x[idx], cache_reference=False)
    pairs = curve.pair_count()
    curve_c = se.EnergyCurve(validation, x[idx])
    pairs_c = curve_c.pair_count(include_reference=False)
    out_c = curve_c.launch(sizes)   # first use computes and keeps the validation triangle
    for _ in range(args.warmup):
        curve_c.launch(sizes)
    torch.cuda.synchronize()
    evs_c = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for e0, e1 in evs_c:
        e0.record(torch.cuda.current_stream())
        out_c = curve_c.launch(sizes)
        e1.record(torch.cuda.current_stream())
    torch.cuda.synchronize()
    step_c = float(np.median([e0.elapsed_time(e1) * 1e-3 for e0, e1 in evs_c]))
    for _ in range(args.warmup):
        curve.launch(sizes)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        out = curve.launch(sizes)
        e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step_s = float(np.median([e0.elapsed_time(e1) * 1e-3 for e0, e1 in evs]))
    got = out.cpu().numpy()
    if world > 1:
        dist.barrier()
        elapsed, step_s = _max_over_ranks([elapsed, step_s], dev)
    if rank == 0:
        d = x.shape[1]
        flop_pair = 3 * d + 1   # d sub, d mul, d - 1 add, 1 sqrt, 1 accumulate
        tflops = pairs * flop_pair / step_s / 1e12
        line = {
            'metric': 'energy-distance curve: pair-distance evals/s (fit_quality over 250 prefixes)',
            'value': pairs * args.steps * world / elapsed, 'unit': 'pair-distance evals/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic (seeded RW-MH LV-surrogate pools; validation = a second pool [::10])',
            'config': {'workload': 'fit_quality curve: validation 2e5 x 4 against prefixes of config 4\'s m = 1000 '
                                   'Stein selection, 250 sizes (Comparison.ipynb cells 19-23)',
                       'n_validation': int(validation.shape[0]), 'm': int(cfg['m']), 'sizes': int(sizes.size),
                       'pairs_per_step': int(pairs), 'ed_at_1000': float(got[-1]),
                       'cached': {'what': 'the same curve with the validation triangle cached across curves '
                                          '(one validation sample for every method x chain, Comparison.ipynb '
                                          'cells 19-23)',
                                  'step_median_us': round(step_c * 1e6, 1), 'pairs_per_step': int(pairs_c),
                                  'same_curve': bool(np.allclose(out_c.cpu().numpy(), got, rtol=1e-12, atol=0))},
                       'parallelism': f'replicas x{world}' if world > 1 else 'single-gpu'},
            'roofline': {'bound': 'valu', 'achieved': round(tflops, 2), 'peak': FP64_VALU_PEAK_TFS, 'unit': 'TFLOP/s',
                         'frac': round(tflops / FP64_VALU_PEAK_TFS, 4),
                         'traffic': pmc_traffic('energy') if world == 1 else None,
                         'kernel': f'dist_colsum_kernel<{d},U,MINB> variant {args.energy_variant} units {args.energy_units} (+ reduce / cumsum)', 'step_median_us': round(step_s * 1e6, 1),
                         'flop_per_pair': flop_pair,
                         'note': 'per pair: d differences, squares and sums, one correctly rounded sqrt (the '
                                 'range-guarded ~10-instruction sequence, one quarter-rate v_rsq_f64) and the '
                                 'accumulate; O(n d) bytes -- fp64 VALU-bound'},
        }
        if not args.no_cpu_baseline:
            from oracle import stein_numpy as ref
            xs = validation[:10_000]
            ys = x[idx]
            c0 = time.perf_counter()
            ref.energy_distance(xs, ys)
            dt = time.perf_counter() - c0
            cpu_pairs = xs.shape[0] ** 2 + xs.shape[0] * ys.shape[0] + ys.shape[0] ** 2
            ref_pairs = sizes.size * validation.shape[0] ** 2 + int(np.sum(validation.shape[0] * sizes + sizes ** 2))
            line['cpu_baseline'] = {
                'value': cpu_pairs / dt, 'unit': 'pair-distance evals/s', 'cores': 1, 'kind': 'port',
                'sample': (f'oracle.stein_numpy.energy_distance (the reference\'s dcor.energy_distance restated as '
                           f'scipy cdist means) for validation[:10000] vs the 1000 selected points: {cpu_pairs:.3g} '
                           f'distances in {dt:.2f} s; the reference\'s curve (one full energy distance per size, '
                           f'{ref_pairs:.3g} distances) extrapolates to {ref_pairs * dt / cpu_pairs:.0f} s')}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_ranks(args):
    """Launcher check without a GPU: every rank joins a gloo group and contributes its rank; rank 0
    prints the group size and the rank sum (tests/test_bench_launch.py)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', 1))
    rank = int(os.environ.get('RANK', 0))
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        dist.init_process_group('gloo')
    t = torch.tensor([rank], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({'workload': 'ranks', 'n_gpus': world, 'rank_sum': int(t.item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_ksd(args):
    """Full-sample cumulative KSD of the config's sample (stein_thinning.stein.ksd over all n rows):
    n(n-1)/2 off-diagonal pair-evaluations per step.  N > 1: the triangle's rows are split into
    pair-balanced blocks, every rank sums its rows into the n-length column-sum vector, one RCCL
    all-reduce, every rank finishes the prefix scan (stein_thinning/distributed.py run_ksd_sharded)."""
    import torch
    import torch.distributed as dist
    from stein_thinning import distributed as sd
    rank, world, dev = _setup_ranks()
    if world > 1:
        _init_group(dev)
    cfg = CONFIGS[args.config if args.config != 'c4' or args.ksd_full else 'c2']
    integrand, _, _ = make_integrand(cfg)
    n, d = cfg['n'], integrand.sample.shape[1]
    import stein_thinning
    stein_thinning.set_arithmetic(args.arith)
    be = sd.HipKsdBackend(integrand, n)
    a0, a1 = sd.triangle_row_bounds(n, rank, world)
    ks = torch.empty(n, dtype=torch.float64, device=dev)
    from stein_thinning import _native as nat
    L = nat.lib()
    p = be.prob
    stream = torch.cuda.current_stream()

    def run_once():
        c = be.colsum(a0, a1)
        if world > 1:
            sd._all_reduce_sum(c)
        nat.check(L.st_ksd_finish(nat.ptr(p.x), nat.ptr(p.g), nat.ptr(p.w), n, p.ld, p.d, p.l, p.tr,
                                  nat.ptr(c), nat.ptr(ks), nat.stream_handle()), 'st_ksd_finish')
    for _ in range(args.warmup):
        run_once()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ce = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    e0.record(stream)
    for c0, c1 in ce:
        c0.record(stream)
        be.colsum(a0, a1)
        c1.record(stream)
    e1.record(stream)
    torch.cuda.synchronize()
    colsum_s = float(np.median([c0.elapsed_time(c1) * 1e-3 for c0, c1 in ce]))
    # full steps (column sums + all-reduce + finish)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_once()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed, colsum_s = _max_over_ranks([elapsed, colsum_s], dev)
    gf = integrand.weights is not None
    pairs = n * (n - 1) / 2
    rank_pairs = sum(n - 1 - a for a in range(a0, a1)) if n < 10 ** 4 else \
        (a1 - a0) * (n - 1) - (a1 * (a1 - 1) - a0 * (a0 - 1)) // 2
    flop_per_pair = algorithmic_flop_per_pair(d, gf) + 1     # + the column accumulate
    # the column-sum kernel's ISA flop per pair: compact arithmetic (default, d <= 8) 67 - 2 (the
    # running-sum fma is the plain accumulate here) + 8 per further coordinate; exact 134 + 13 per
    # coordinate; + the weights' 2 mul, + the accumulate
    if args.arith == 'compact' and d <= 8:
        isa_flop_per_pair = 65 + 8 * (d - 4) + (2 if gf else 0) + 1
    else:
        isa_flop_per_pair = 134 + 13 * (d - 4) + (2 if gf else 0) + 1
    if rank == 0:
        tflops = rank_pairs * flop_per_pair / colsum_s / 1e12
        line = {
            'metric': 'Stein-kernel pair-evals/s, full-sample cumulative KSD (stein.ksd over all n rows)',
            'value': pairs * args.steps / elapsed, 'unit': 'pair-evals/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': elapsed / args.steps * 1e3,
            'higher_is_better': True, 'scaling': 'strong', 'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic (seeded RW-MH LV-surrogate chains; see bench.py docstring)',
            'config': {'workload': f"full-sample KSD of config {cfg['desc']}", 'n': n, 'd': d,
                       'kernel': 'gradient-free' if gf else 'langevin',
                       'arithmetic': args.arith if d <= 8 else 'exact',
                       'parallelism': f'triangle rows x{world}, RCCL all-reduce of the n-vector' if world > 1
                       else 'single-gpu'},
            'roofline': {'bound': 'valu', 'achieved': round(tflops, 2), 'peak': FP64_VALU_PEAK_TFS,
                         'unit': 'TFLOP/s', 'frac': round(tflops / FP64_VALU_PEAK_TFS, 4),
                         'traffic': pmc_traffic('ksd_' + ('c4' if args.ksd_full else 'c2')) if world == 1 else None,
                         'kernel': f'ksd_colsum_kernel<{d},{str(gf).lower()}>', 'kernel_avg_us': round(colsum_s * 1e6, 1),
                         'flop_per_pair': flop_per_pair,
                         'flop_per_pair_source': 'SURVEY.md 8(d): 12 d + 40 (+2 gradient-free) + 1 accumulate',
                         'issue': {'isa_flop_per_pair': isa_flop_per_pair,
                                   'achieved_TFs': round(rank_pairs * isa_flop_per_pair / colsum_s / 1e12, 2)}},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_proxy(args):
    """Proxy producers (stein_thinning.proxy; csrc/proxy.hip): log q and grad log q of config 5's
    Gaussian proxy N(sample mean, 1.2 sample cov) -- or a Student-t proxy with the same shape,
    df = 4 (--proxy-kind t) -- at every row of the n = 5e5, d = 50 sample, inputs resident in HBM.
    N > 1: each rank evaluates its contiguous row block (no exchange)."""
    import torch
    import torch.distributed as dist
    from stein_thinning import _native as nat
    from stein_thinning import proxy
    from stein_thinning.distributed import shard_bounds
    rank, world, dev = _setup_ranks()
    if world > 1:
        _init_group(dev)
    cfg = CONFIGS['c5']
    x, _, _, _ = gaussian_d50(cfg['n'], cfg['seed'])
    n, d = x.shape
    mean = np.mean(x, axis=0)
    cov = 1.2 * np.cov(x, rowvar=False)
    t_kind = args.proxy_kind == 't'
    df = 4.0 if t_kind else 0.0
    psd = proxy._psd(cov, allow_singular=t_kind)
    if t_kind:
        from scipy.special import gammaln
        c_log = float(gammaln(0.5 * (df + d)) - gammaln(0.5 * df) - d / 2. * np.log(df * np.pi) - 0.5 * psd.log_pdet)
    else:
        c_log = psd.rank * proxy._LOG_2PI + psd.log_pdet
    r0, r1 = shard_bounds(n, rank, world)
    rows = r1 - r0
    nat.check(nat.lib().st_tune(7, args.proxy_mode), 'st_tune')
    xd = torch.from_numpy(np.ascontiguousarray(x[r0:r1])).to(dev)
    loc = torch.from_numpy(mean).to(dev)
    U = torch.from_numpy(np.ascontiguousarray(psd.U)).to(dev)
    P = torch.from_numpy(np.ascontiguousarray(np.linalg.inv(cov))).to(dev)
    lq = torch.empty(rows, dtype=torch.float64, device=dev)
    gq = torch.empty((rows, d), dtype=torch.float64, device=dev)
    L = nat.lib()

    def run_once():
        nat.check(L.st_proxy_logpdf_grad(nat.ptr(xd), rows, d, nat.ptr(loc), nat.ptr(U), nat.ptr(P), df, c_log,
                                         nat.ptr(lq), nat.ptr(gq), nat.stream_handle()), 'st_proxy_logpdf_grad')
    for _ in range(args.warmup):
        run_once()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        run_once()
        e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_s = float(np.median([e0.elapsed_time(e1) * 1e-3 for e0, e1 in evs]))
    if world > 1:
        dist.barrier()
        elapsed, kern_s = _max_over_ranks([elapsed, kern_s], dev)
    if rank == 0:
        # algorithmic work of the kernel that runs: 16 < d <= 64 -> the matrix-core kernel (one
        # product y = P dev per row, Mahalanobis term dev . y: 2d^2 + 2d flop + the epilogue);
        # otherwise the VALU kernel (z = dev U and y: 4d^2 + 2d)
        mfma = 16 < d <= 64 and args.proxy_mode != 1
        flop_row = (2 * d * d + 2 * d if mfma else 4 * d * d + 2 * d) + (2 * d + 12 if t_kind else 2)
        bytes_row = 16 * d + 8
        tflops = rows * flop_row / kern_s / 1e12
        gbs = rows * bytes_row / kern_s / 1e9
        hbm_bound = bytes_row / (HBM_PEAK_GBS * 1e9) >= flop_row / (FP64_VALU_PEAK_TFS * 1e12)
        line = {
            'metric': 'proxy rows/s (log q + grad log q per sample row)', 'value': n * args.steps / elapsed,
            'unit': 'rows/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'strong',
            'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic (config 5: iid N(0, AR(1) 0.5), d = 50)',
            'config': {'workload': f"config 5 proxy: {'Student-t df=4' if t_kind else 'Gaussian'} "
                                   'N(mean, 1.2 cov), n=5e5 d=50', 'n': n, 'd': d,
                       'parallelism': f'row blocks x{world}' if world > 1 else 'single-gpu'},
            'roofline': dict(
                ({'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                  'frac': round(gbs / HBM_PEAK_GBS, 4)} if hbm_bound else
                 {'bound': 'mfma' if mfma else 'valu', 'achieved': round(tflops, 2), 'peak': FP64_VALU_PEAK_TFS,
                  'unit': 'TFLOP/s', 'frac': round(tflops / FP64_VALU_PEAK_TFS, 4)}),
                traffic=pmc_traffic('proxy_' + args.proxy_kind) if world == 1 and args.proxy_mode == 0 else None,
                kernel=(('proxy_mfma_buf_kernel<4,14>' if args.proxy_mode in (0, 4) and d % 2 == 0
                                       else 'proxy_mfma_stream_kernel<4,14>' if args.proxy_mode in (0, 3, 4)
                                       else 'proxy_mfma_kernel (LDS-tiled)') if mfma else 'proxy_kernel'),
                kernel_avg_us=round(kern_s * 1e6, 1), flop_per_row=flop_row, bytes_per_row=bytes_row,
                fp64_view={'achieved_TFs': round(tflops, 2), 'peak_TFs': FP64_VALU_PEAK_TFS,
                           'frac': round(tflops / FP64_VALU_PEAK_TFS, 4)},
                hbm_view={'achieved_GBs': round(gbs, 1), 'peak_GBs': HBM_PEAK_GBS,
                          'frac': round(gbs / HBM_PEAK_GBS, 4)}),
        }
        if world == 1 and not args.no_cpu_baseline:
            from oracle import proxy_numpy as op
            m = 100_000
            c0 = time.perf_counter()
            if t_kind:
                op.student_t_proxy(x[:m], mean, cov, df)
            else:
                op.gaussian_proxy(x[:m], mean, cov)
            dt = time.perf_counter() - c0
            line['cpu_baseline'] = {'value': m / dt, 'unit': 'rows/s', 'kind': 'reference',
                                    'cores': int(os.environ.get('OMP_NUM_THREADS', os.cpu_count())),
                                    'sample': f'scipy {"multivariate_t" if t_kind else "multivariate_normal"}.logpdf + '
                                              f'the reference\'s einsum gradient on the first {m} rows ({dt:.2f} s; '
                                              'BLAS threads as configured on the host)'}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_lv(args):
    """Lotka-Volterra gradients (stein_thinning.lotka_volterra; csrc/lv.hip): grad log posterior
    from the forward sensitivity equations (RK45, scipy's algorithm) at 113 143 parameter points --
    the unique-sample count of the reference's Dask/AWS gradient run -- drawn around the
    data-generating theta.  N > 1: each rank evaluates a contiguous block of points."""
    import torch
    import torch.distributed as dist
    from stein_thinning import _native as nat
    from stein_thinning import lotka_volterra as lv
    from stein_thinning.distributed import shard_bounds
    rank, world, dev = _setup_ranks()
    if world > 1:
        _init_group(dev)
    n = 113_143
    rng = np.random.default_rng(12350)
    theta = np.exp(np.log(lv.THETA) + 0.05 * rng.normal(size=(n, 4)))
    data = lv.reference_data()
    t, y, s = lv._settings(data, lv.RTOL, lv.ATOL)
    cinv = np.ascontiguousarray(np.linalg.inv(data.cov))
    r0, r1 = shard_bounds(n, rank, world)
    m = r1 - r0
    thd = torch.from_numpy(np.ascontiguousarray(theta[r0:r1])).to(dev)
    td, yd = torch.from_numpy(t).to(dev), torch.from_numpy(y).to(dev)
    out = torch.empty((m, 4), dtype=torch.float64, device=dev)
    status = torch.zeros(m, dtype=torch.int32, device=dev)
    L = nat.lib()
    two_phase = args.lv_mode == 0
    nat.check(L.st_tune(17, args.lv_global_obs), 'st_tune')
    nat.check(L.st_tune(18, args.lv_pieces), 'st_tune')
    wb = int(L.st_lv_grad_workspace_bytes(m, t.size))
    work = torch.empty((wb + 7) // 8, dtype=torch.float64, device=dev) if two_phase else None

    def run_once():
        if two_phase:
            nat.check(L.st_lv_grad_log_posterior_ws(nat.ptr(thd), m, nat.ptr(td), t.size, nat.ptr(yd), s.ctypes.data,
                                                    cinv.ctypes.data, lv.MAX_STEPS, nat.ptr(out), nat.ptr(status),
                                                    nat.ptr(work), wb, nat.stream_handle()),
                      'st_lv_grad_log_posterior_ws')
            return
        nat.check(L.st_lv_grad_log_posterior(nat.ptr(thd), m, nat.ptr(td), t.size, nat.ptr(yd), s.ctypes.data,
                                             cinv.ctypes.data, lv.MAX_STEPS, nat.ptr(out), nat.ptr(status),
                                             nat.stream_handle()), 'st_lv_grad_log_posterior')
    for _ in range(args.warmup):
        run_once()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(stream)
        run_once()
        e1.record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_s = float(np.mean([e0.elapsed_time(e1) * 1e-3 for e0, e1 in evs]))
    failed = int((status != 0).sum().item())
    lv_flops = float(m) * t.size * LV_FLOP_PER_OBS
    if world > 1:
        dist.barrier()
        elapsed, kern_s = _max_over_ranks([elapsed, kern_s], dev)
    if rank == 0:
        line = {
            'metric': 'LV grad-log-posterior points/s (forward sensitivities, RK45)', 'value': n * args.steps / elapsed,
            'unit': 'points/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': elapsed / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'strong',
            'vs_baseline': None, 'dtype': 'f64',
            'data': 'synthetic parameter points exp(N(log theta*, 0.05^2)); observations = the reference module\'s data',
            'config': {'workload': 'LV gradients at 113 143 points (Dask_AWS unique-sample count), t_n = 2400, '
                                   'rtol 1e-3 / atol 1e-6', 'n': n,
                       'parallelism': f'point blocks x{world}' if world > 1 else 'single-gpu'},
            'roofline': ({'bound': 'valu', 'achieved': round(lv_flops / kern_s / 1e12, 2), 'peak': FP64_VALU_PEAK_TFS,
                          'unit': 'TFLOP/s', 'frac': round(lv_flops / kern_s / 1e12 / FP64_VALU_PEAK_TFS, 4),
                          'traffic': pmc_traffic('lv2') if world == 1 else None,
                          'kernel': 'lv_kernel<10,record> + lv_dense_kernel<' +
                                    ('4,global-obs' if args.lv_global_obs == 1 else '8,lds-obs') + '> (+ overflow pass)',
                          'kernel_avg_us': round(kern_s * 1e6, 1), 'flop_per_observation': LV_FLOP_PER_OBS,
                          'note': 'priced on the dense-output work only (n x t_n observation points x '
                                  f'{LV_FLOP_PER_OBS} flop: the quartic for 10 states, residual, C^-1 and the '
                                  'sensitivity products); the RK45 integration (~32 accepted steps per point, '
                                  'one thread each) is the serial part'} if two_phase else
                         {'bound': 'latency', 'achieved': None, 'peak': None, 'unit': None, 'frac': None,
                          'traffic': pmc_traffic('lv') if world == 1 else None, 'kernel': 'lv_kernel<10>',
                          'kernel_avg_us': round(kern_s * 1e6, 1),
                          'note': 'single-phase: one thread per point integrates and evaluates its 2400 '
                                  'observation points; 354 VGPRs -> one wave per SIMD; 113 143 points fill 1 768 '
                                  'waves = 1.7 waves per SIMD'}),
            'failed_points': failed,
        }
        if world == 1 and not args.no_cpu_baseline:
            from oracle import lv_numpy as ol
            k = 200
            c0 = time.perf_counter()
            for row in theta[:k]:
                ol.grad_log_posterior(row, data.t, data.y, data.cov)
            dt = time.perf_counter() - c0
            line['cpu_baseline'] = {'value': k / dt, 'unit': 'points/s', 'cores': 1, 'kind': 'port',
                                    'sample': f'oracle.lv_numpy.grad_log_posterior (the notebook function on '
                                              f'scipy solve_ivp) for the first {k} points, {dt:.2f} s, one process'}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _dump_maps():
    """ST_BENCH_DUMP_MAPS=<file>: the process's memory map at the end of main (resolves the
    addresses of a crash in exit-time destructors)."""
    path = os.environ.get('ST_BENCH_DUMP_MAPS')
    if path:
        with open('/proc/self/maps') as src, open(path, 'w') as dst:
            dst.write(src.read())


if __name__ == '__main__':
    rc = main() or 0
    _dump_maps()
    sys.exit(rc)
