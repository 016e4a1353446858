"""Measurement probe (not product code): where the wall time of stein_thinning.thin() on host
arrays goes at config 4 (n = 2e6, d = 4, m = 1000): host preprocessing, preconditioner, upload,
the persistent launch, index read-back (the breakdown runs the stages one after another; thin()
overlaps the upload with the preconditioner and thins the run starts, DeviceProblem.dedup_view)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd')]


def main():
    import torch
    import bench
    from stein_thinning import thinning as st
    from stein_thinning.kernel import make_precon
    x, g, _, _ = bench.lv_surrogate(2_000_000, 12345)
    st.thin(x, g, 1000, preconditioner='med')      # warm-up (module load, allocator)
    for _ in range(3):
        t0 = time.perf_counter()
        xs, gs = st._validate_and_standardize(x, g, True)
        t1 = time.perf_counter()
        linv = make_precon(xs, 'med', on_device=True)
        t2 = time.perf_counter()
        integ = st.SteinIntegrand(xs, gs, linv)
        prob = integ.device_problem()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        idx, a, ws = prob.greedy_buffers(1000)
        prob.greedy_launch(1000, idx, a, ws)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        out = idx.cpu().numpy()
        t5 = time.perf_counter()
        print(f'standardize {1e3 * (t1 - t0):.1f} ms  precon {1e3 * (t2 - t1):.1f}  upload+layout {1e3 * (t3 - t2):.1f}  '
              f'greedy {1e3 * (t4 - t3):.1f}  readback {1e3 * (t5 - t4):.2f}  total {1e3 * (t5 - t0):.1f} ms', flush=True)
    ts = []
    for _ in range(9):
        t0 = time.perf_counter()
        st.thin(x, g, 1000, preconditioner='med')
        ts.append(time.perf_counter() - t0)
    print(f'thin() end to end: median {1e3 * np.median(ts):.1f} ms, min {1e3 * min(ts):.1f}, '
          f'runs {" ".join(f"{1e3 * v:.1f}" for v in ts)}', flush=True)
    t0 = time.perf_counter()
    make_precon(xs, 'med')
    t1 = time.perf_counter()
    make_precon(xs, 'med', on_device=True)
    t2 = time.perf_counter()
    print(f'med preconditioner: host {1e3 * (t1 - t0):.2f} ms, device {1e3 * (t2 - t1):.2f} ms', flush=True)


if __name__ == '__main__':
    main()
