"""Exit-crash probe: a torch-only GPU process (no stein library), to run under rocprofv3."""
import sys

import torch

x = torch.ones(1 << 20, device='cuda')
print(float((x * 2).sum().item()), flush=True)
if len(sys.argv) > 1 and sys.argv[1] == 'ctypes':
    import ctypes
    import os
    ctypes.CDLL(os.path.join(os.path.dirname(__file__), '..', '..', 'gradient-free-mcmc-postprocessing_amd',
                             'stein_thinning', '_lib', 'libstein_hip.so'))
    print('loaded libstein_hip.so', flush=True)
