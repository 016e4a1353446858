"""Digest of the synthetic bench / golden inputs and of NumPy's pow on this host's CPU.

Run here and on the GPU box: equal digests mean the golden index fixtures made in the build
container (tests/golden/make_config_golden.py) apply to the inputs the box regenerates.
"""
import hashlib
import os
import platform
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import gaussian_d50, lv_surrogate  # noqa: E402


def digest(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()[:16]


def main():
    cpu = 'unknown'
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    cpu = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    print('cpu', cpu, platform.machine())
    x, g, log_p, (log_q, gq) = lv_surrogate(2_000_000, 12345)
    print('c4 x,g', digest(x, g))
    x, g, log_p, (log_q, gq) = lv_surrogate(200_000, 12348)
    print('c3 x,lp,lq,gq', digest(x, log_p, log_q, gq))
    x, log_p, log_q, gq = gaussian_d50(500_000, 12349)
    print('c5 x', digest(x), 'lp', digest(log_p), 'lq', digest(log_q), 'gq', digest(gq))
    v = np.random.default_rng(1).uniform(1.0, 50.0, 1 << 20)
    print('pow2.5', digest(v ** 2.5), 'pow1.5', digest(v ** 1.5), 'sqrt', digest(v ** 0.5))


if __name__ == '__main__':
    main()
