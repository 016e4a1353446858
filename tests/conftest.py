import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_ROOT = os.path.join(ROOT, 'gradient-free-mcmc-postprocessing_amd')
for p in (ROOT, PKG_ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a HIP device (MI355X); runs the HIP path')
    config.addinivalue_line('markers', 'slow: longer CPU oracle runs')


@pytest.fixture(scope='session')
def golden():
    import json
    with open(os.path.join(ROOT, 'tests', 'golden', 'reference_outputs.json')) as f:
        return json.load(f)


@pytest.fixture(scope='session')
def curves():
    import json
    with open(os.path.join(ROOT, 'tests', 'golden', 'gm_comparison_curves.json')) as f:
        return json.load(f)['curves']


@pytest.fixture(scope='session')
def gm():
    from oracle import models
    return models.gm_reference_sample()


@pytest.fixture(scope='session')
def config4():
    """BASELINE config 4 (n = 2e6, d = 4, Langevin, 'med', m = 1000): raw LV-surrogate arrays, the
    oracle's standardised inputs and the threaded C bit model's full 1000-step run on them
    (oracle/stein_ref.c sr_greedy_mt: ~10 s on 16 host threads)."""
    import numpy as np
    from bench import lv_surrogate
    from oracle import stein_numpy as o
    from tests import oracle_c
    n, m = 2_000_000, 1000
    x, g, _, _ = lv_surrogate(n, 12345)
    s, gs = o._validate_and_standardize(x, g, True)
    linv = o.make_precon(s, 'med')
    l, tr = float(linv[0, 0]), float(np.trace(linv))
    cidx, cA = oracle_c.greedy_mt(s, gs, None, l, tr, m)
    return dict(x=x, g=g, s=s, gs=gs, l=l, tr=tr, m=m, idx=cidx, A=cA)
