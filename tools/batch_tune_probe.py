"""Measurement probe (not product code): the chains batch launch (the reference's 5 LV-shape chains,
run starts only) under st_tune settings, e.g. poll delay (key 16), record replicas (key 10), LDS
chunk chains (key 19).  Indices must agree with the default.

    python tools/batch_tune_probe.py [chains] key=value[,value...] ...
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    from stein_thinning import _native as nat
    from stein_thinning import device
    from stein_thinning import thinning as st
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    specs = []
    for a in sys.argv[2:]:
        k, vs = a.split('=')
        specs += [(int(k), int(v)) for v in vs.split(',')]
    n, m = 500_000, 10_000
    probs = []
    for k in range(K):
        prob = st._make_stein_integrand(*bench.lv_call_shape(n, 20_000 + k, 'exp'), preconditioner='med').device_problem()
        view = prob.dedup_view()
        probs.append(view.problem if view is not None else prob)
    print(f'{K} chains, run starts {[p.n for p in probs]}', flush=True)
    L = nat.lib()
    ref = None
    for key, val in [(None, None)] + specs + [(None, None)]:
        if key is not None:
            assert L.st_tune(key, val) == 0, (key, val)
        try:
            ts = []
            for rep in range(3):
                bufs = [p.greedy_buffers(m) for p in probs]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                assert device._launch_batch(probs, m, bufs)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                got = [b[0].cpu().numpy().view(np.uint32).copy() for b in bufs]
                if ref is None:
                    ref = got
                same = all(np.array_equal(a, b) for a, b in zip(got, ref))
            label = 'default' if key is None else f'key {key} = {val}'
            print(f'{label:>16}: {" ".join(f"{1e3 * t:7.2f}" for t in ts)} ms, same indices {same}', flush=True)
        finally:
            if key is not None:
                L.st_tune(key, -1)


if __name__ == '__main__':
    main()
