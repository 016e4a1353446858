"""Where the near-tie guard's time goes on small shards: one launch's fixed part (staging, bounds) against
the per-step part.  Times st_greedy on a BASELINE config's standardised sample (all rows, compact
arithmetic) for several m with the guard off and on, HIP events on the launch stream, median of `reps`;
prints ms per thin and the least-squares split  t(m) = fixed + m * per_step  for each setting.

  python tools/guard_fixed_cost.py [config ...]      (default: c2 c4r8)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd'))


def main():
    import torch
    import bench
    from stein_thinning import _native as nat
    cfgs = sys.argv[1:] or ['c2', 'c4r8']
    ms_list = [2, 10, 50, 100, 300, 1000]
    reps = 9
    out = {}
    for name in cfgs:
        integrand, _, _ = bench.make_integrand(bench.CONFIGS[name])
        prob = integrand.device_problem()
        stream = torch.cuda.current_stream()
        rec = {}
        for guard in (False, True):
            nat.set_near_tie_guard(guard)
            ts = []
            for m in ms_list:
                idx, a, ws = prob.greedy_buffers(m)
                prob.greedy_launch(m, idx, a, ws)   # warm-up (plan, LDS attribute)
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
                for e0, e1 in evs:
                    e0.record(stream)
                    prob.greedy_launch(m, idx, a, ws)
                    e1.record(stream)
                torch.cuda.synchronize()
                ts.append(float(np.median([e0.elapsed_time(e1) for e0, e1 in evs])))
            A = np.vstack([np.ones(len(ms_list)), np.array(ms_list, dtype=float)]).T
            fixed, per = np.linalg.lstsq(A, np.array(ts), rcond=None)[0]
            key = 'guard' if guard else 'plain'
            rec[key] = {'ms': dict(zip(ms_list, [round(t, 4) for t in ts])), 'fixed_us': round(fixed * 1e3, 1),
                        'per_step_us': round(per * 1e3, 3)}
            print(name, key, json.dumps(rec[key]), flush=True)
        out[name] = rec
    nat.set_near_tie_guard(None)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
