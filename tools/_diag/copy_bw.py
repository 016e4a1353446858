"""HBM read+write reference points on the box: torch copy_ / fill_ / sum over 200 MB fp64 buffers (the
config-5 proxy moves 200 MB in + 204 MB out)."""
import torch

n = 25_000_000
a = torch.randn(n, dtype=torch.float64, device='cuda')
b = torch.empty_like(a)


def t(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    return ms[len(ms) // 2] * 1e3


us = t(lambda: b.copy_(a))
print(f'copy 200 MB -> 200 MB: {us:.1f} us  {400e6 / us / 1e3:.0f} GB/s (read+write)')
us = t(lambda: b.fill_(1.0))
print(f'fill 200 MB: {us:.1f} us  {200e6 / us / 1e3:.0f} GB/s (write)')
s = torch.empty(1, dtype=torch.float64, device='cuda')
us = t(lambda: torch.sum(a, out=s))
print(f'sum 200 MB: {us:.1f} us  {200e6 / us / 1e3:.0f} GB/s (read)')
