"""Freeze the reference NumPy path's selections at BASELINE configs 4 and 5 as golden fixtures.

Runs in the build container (CPU only, ~3 + ~6 minutes):

    python tests/golden/make_config_golden.py [c4] [c5]

For each config it regenerates the seeded synthetic input (``bench.lv_surrogate`` /
``bench.gaussian_d50``), runs the oracle's restatement of the reference greedy loop
(``oracle/stein_numpy.py``: ``JAX_Stein_Thinning.ipynb:281-295`` with the kernel of ``:354-361``)
over the FULL length (m = 1000 / 500) and writes ``tests/golden/config{4,5}_numpy_indices.json``:

* ``indices``      -- the selected index sequence (what ``oracle.thin`` / ``thin_gf`` return);
* ``margin_ulps``  -- per step, (second-smallest distinct running sum - smallest) in ulps of the
                      smallest: how far each argmin is from flipping under a 1-ulp perturbation;
* ``ties``         -- per step, how many rows share the smallest value (duplicated rows of the
                      RW-MH chains; np.argmin resolves them to the lowest index);
* ``input_sha256`` -- digest of the arrays fed to the oracle, so a GPU test can tell "different
                      input" from "different selection" (tools/input_digest.py showed the build
                      container and the MI355X box generate bit-identical inputs and NumPy pow).

The loop below is ``oracle.stein_numpy._greedy_search`` with the margin bookkeeping added; it calls
the oracle's own integrand, so the indices are those of ``oracle.stein_numpy.thin`` (checked on the
first 50 steps before writing).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from bench import gaussian_d50, lv_surrogate  # noqa: E402
from oracle import stein_numpy as o  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def digest(*arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def greedy_with_margins(m: int, integrand):
    idx = np.empty(m, dtype=np.int64)
    margin = np.empty(m)
    ties = np.empty(m, dtype=np.int64)

    def pick(k0, t):
        i = int(np.argmin(k0))
        best = k0[i]
        eq = k0 == best
        ties[t] = int(np.count_nonzero(eq))
        rest = k0[~eq]
        margin[t] = (float(np.min(rest)) - best) / np.spacing(abs(best)) if rest.size else np.inf
        idx[t] = i

    t0 = time.time()
    k0 = integrand(slice(None), slice(None))
    pick(k0, 0)
    for t in range(1, m):
        k0 += 2 * integrand(slice(None), [idx[t - 1]])
        pick(k0, t)
        if t % 100 == 0:
            print(f'  step {t}/{m}  {time.time() - t0:.0f} s', flush=True)
    return idx, margin, ties


def write(name, cfg_desc, idx, margin, ties, sha, seconds):
    out = dict(
        config=cfg_desc,
        generator='tests/golden/make_config_golden.py (oracle/stein_numpy.py, NumPy %s)' % np.__version__,
        reference='JAX_Stein_Thinning.ipynb:281-295 (greedy loop), :354-361 (vfk0_imq)',
        input_sha256=sha,
        seconds=round(seconds, 1),
        indices=[int(i) for i in idx],
        margin_ulps=[None if not np.isfinite(v) else float('%.4g' % v) for v in margin],
        ties=[int(t) for t in ties],
        min_margin_ulps=float('%.4g' % np.min(margin)),
    )
    path = os.path.join(HERE, name)
    with open(path, 'w') as f:
        json.dump(out, f, separators=(',', ':'))
    print('wrote', path, 'min margin', out['min_margin_ulps'], 'ulps; max ties', int(np.max(ties)))


def config4():
    n, m = 2_000_000, 1000
    x, g, _, _ = lv_surrogate(n, 12345)
    integ = o._make_stein_integrand(x, g, True, 'med')
    t0 = time.time()
    idx, margin, ties = greedy_with_margins(m, integ)
    secs = time.time() - t0
    np.testing.assert_array_equal(idx[:50], o.thin(x, g, 50, preconditioner='med'))
    write('config4_numpy_indices.json', 'config 4: lv_surrogate(2e6, seed 12345), thin m=1000, med',
          idx, margin, ties, digest(x, g), secs)


def config5():
    n, m = 500_000, 500
    x, log_p, log_q, gq = gaussian_d50(n, 12349)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        integ = o._make_stein_gf_integrand(x, log_p, log_q, gq, True, None, 'med')
        t0 = time.time()
        idx, margin, ties = greedy_with_margins(m, integ)
        secs = time.time() - t0
        np.testing.assert_array_equal(idx[:10], o.thin_gf(x, log_p, log_q, gq, 10, preconditioner='med'))
    write('config5_numpy_indices.json', 'config 5: gaussian_d50(5e5, seed 12349), thin_gf m=500, med',
          idx, margin, ties, digest(x, log_p, log_q, gq), secs)


if __name__ == '__main__':
    which = sys.argv[1:] or ['c4', 'c5']
    if 'c4' in which:
        config4()
    if 'c5' in which:
        config5()
