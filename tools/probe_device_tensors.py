"""Phase times of the drop-in thin on host arrays vs ROCm tensors (config 4 shape): where the
device-tensor call spends its time.  Prints one line per phase (median of 5)."""
import time

import numpy as np
import torch

import bench
from stein_thinning import thinning as st


def main():
    cfg = dict(bench.CONFIGS['c4'])
    _, hx, hg = bench.make_integrand(cfg)
    m = cfg['m']
    xd = torch.from_numpy(np.ascontiguousarray(hx)).cuda()
    gd = torch.from_numpy(np.ascontiguousarray(hg)).cuda()
    torch.cuda.synchronize()

    def clock(f):
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = f()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3, r
    t, up = clock(lambda: st._download_standardized(xd, gd))
    print(f'download_standardized   {t:8.2f} ms')
    t, integ = clock(lambda: st._device_integrand(st._download_standardized(xd, gd), 'med', None))
    print(f'+ device_integrand(med)  {t:8.2f} ms')
    t, _ = clock(lambda: st._greedy_search(m, st._device_integrand(st._download_standardized(xd, gd), 'med', None)))
    print(f'+ greedy_search          {t:8.2f} ms')
    t, _ = clock(lambda: st.thin(xd, gd, m, preconditioner='med'))
    print(f'thin(device tensors)     {t:8.2f} ms')
    t, _ = clock(lambda: st._upload_standardized(hx, hg, True))
    print(f'upload_standardized      {t:8.2f} ms')
    t, _ = clock(lambda: st._make_stein_integrand(hx, hg, True, 'med'))
    print(f'+ integrand(med)         {t:8.2f} ms')
    t, _ = clock(lambda: st.thin(hx, hg, m, preconditioner='med'))
    print(f'thin(host arrays)        {t:8.2f} ms')
    stage = torch.empty((xd.shape[0], xd.shape[1]), dtype=torch.float64, pin_memory=True)
    t, _ = clock(lambda: stage.copy_(xd))
    print(f'D2H x alone              {t:8.2f} ms')
    t, _ = clock(lambda: torch.stack([torch.isnan(gd).any(), torch.isinf(gd).any()]).tolist())
    print(f'g flags                  {t:8.2f} ms')


if __name__ == '__main__':
    main()
