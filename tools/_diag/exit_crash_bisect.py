"""Exit-crash bisection under rocprofv3 (diagnostic): one GPU feature per mode, then a normal exit.
modes: pinned | persistent | steps | thin | thin_nopin"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd'))
mode = sys.argv[1]
x = torch.ones(1 << 20, device='cuda')
print(float(x.sum().item()), flush=True)
rng = np.random.default_rng(0)
s = rng.normal(size=(50_000, 4))
if mode == 'pinned':
    h = torch.empty((1 << 20,), dtype=torch.float64, pin_memory=True)
    h.numpy()[:] = 1.0
    print(float(h.cuda().sum().item()), flush=True)
elif mode in ('persistent', 'steps'):
    from stein_thinning.device import DeviceProblem
    from stein_thinning import _native as nat
    if mode == 'steps':
        nat.lib().st_tune(3, 0)
    p = DeviceProblem(s, -s, None, 0.5, 2.0)
    print(p.greedy(50)[:5], flush=True)
elif mode in ('thin', 'thin_nopin'):
    if mode == 'thin_nopin':
        from stein_thinning import thinning
        thinning._host_buffer = lambda shape: np.empty(shape, dtype=np.float64)
    from stein_thinning import thinning as st
    print(st.thin(s, -s, 50)[:5], flush=True)
torch.cuda.synchronize()
print('exit', mode, flush=True)
