"""Config-5 shapes at shard sizes (d = 50, gradient-free, m = 500) on one GPU: the wide persistent
kernel (shards of at most 256 rows per CU) against the launch-per-step path (st_tune key 3 = 0)."""
import os
import sys
import warnings

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'gradient-free-mcmc-postprocessing_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from stein_thinning import _native as nat  # noqa: E402
from stein_thinning import thinning as st  # noqa: E402

L = nat.lib()
for n in (int(a) for a in (sys.argv[1:] or ['62500', '31250', '125000'])):
    x, log_p, log_q, gq = bench.gaussian_d50(n, 12349)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        integ = st._make_stein_gf_integrand(x, log_p, log_q, gq, preconditioner='med')
    prob = integ.device_problem()
    m = 500
    ref = None
    for label, rt in (('persistent (auto)', -1), ('launch per step', 0)):
        L.st_tune(3, rt)
        idx, a, ws = prob.greedy_buffers(m)
        prob.greedy_launch(m, idx, a, ws)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            prob.greedy_launch(m, idx, a, ws)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        got = idx.cpu().numpy().view(np.uint32).copy()
        ref = got if ref is None else ref
        print(f'n={n:7d} d=50 gf m={m} {label:>18}: {np.median(ts):7.2f} ms/thin, {np.median(ts) / m * 1e3:6.2f} '
              f'us/step, same indices: {bool(np.array_equal(got, ref))}', flush=True)
    L.st_tune(3, -1)
