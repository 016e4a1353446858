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
