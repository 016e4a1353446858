"""Persistent-kernel variant sweep on one GPU: time st_greedy for the bench configs under several
st_tune settings and check that every variant selects the same indices.

    python tools/tune_sweep.py [c4|c2|c3|c4@<n>][+dedup] "8=1" "8=2" "8=2,3=4" ...
(+dedup: the thin of the run starts, DeviceProblem.dedup_view, as the drop-in thin runs it)
Each argument is a comma-separated list of key=value st_tune settings (reset to -1 between)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gradient-free-mcmc-postprocessing_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from stein_thinning import _native as nat  # noqa: E402

cfg_name = sys.argv[1] if len(sys.argv) > 1 and not '=' in sys.argv[1] else 'c4'
settings = [a for a in sys.argv[1:] if '=' in a] or ['8=1', '8=2']
# "c4@1000000": config 4's data and m at another n (crossover sweeps)
cfg_name, plus, mode = cfg_name.partition('+')
base, _, n_over = cfg_name.partition('@')
cfg = dict(bench.CONFIGS[base])
if n_over:
    cfg['n'] = int(float(n_over))
integrand, _, _ = bench.make_integrand(cfg)
prob = integrand.device_problem()
if mode == 'dedup':
    prob = prob.dedup_view().problem
    print(f'{cfg_name}+dedup: {prob.n} run starts of {cfg["n"]} rows', flush=True)
m = cfg['m']
L = nat.lib()
ref = None
for st in settings:
    for k in (3, 4, 5, 8, 9, 10, 15, 16, 19):
        L.st_tune(k, -1)
    for kv in st.split(','):
        k, v = (int(x) for x in kv.split('='))
        assert L.st_tune(k, v) == 0, kv
    idx, a, ws = prob.greedy_buffers(m)
    prob.greedy_launch(m, idx, a, ws)
    torch.cuda.synchronize()
    times = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        prob.greedy_launch(m, idx, a, ws)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    got = idx.cpu().numpy().view(np.uint32).copy()
    if ref is None:
        ref = got
    same = bool(np.array_equal(got, ref))
    print(f'{cfg_name} {st:>14}: {np.median(times):8.3f} ms/thin (min {min(times):.3f}), '
          f'{np.median(times) / m * 1e3:6.2f} us/step, same indices: {same}', flush=True)
