import time, torch, numpy as np
n=2_000_000*4
a=np.random.default_rng(0).normal(size=n)
p=torch.empty(n, dtype=torch.float64, pin_memory=True); pn=p.numpy(); pn[:]=a
dev=torch.device('cuda',0)
for name, arr in [('pageable', a), ('pinned-view', pn)]:
    for _ in range(3):
        torch.cuda.synchronize(); t=time.perf_counter()
        d=torch.from_numpy(arr).to(dev); torch.cuda.synchronize()
        print(name, f'{(time.perf_counter()-t)*1e3:.2f} ms', flush=True)
for _ in range(3):
    torch.cuda.synchronize(); t=time.perf_counter()
    d=p.to(dev, non_blocking=True); torch.cuda.synchronize()
    print('pinned-tensor', f'{(time.perf_counter()-t)*1e3:.2f} ms', flush=True)
t=time.perf_counter(); q=torch.empty(n, dtype=torch.float64, pin_memory=True); print('pin alloc 64MB', (time.perf_counter()-t)*1e3)
del q
t=time.perf_counter(); q=torch.empty(n, dtype=torch.float64, pin_memory=True); print('pin alloc again', (time.perf_counter()-t)*1e3)
