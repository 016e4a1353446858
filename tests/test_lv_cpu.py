"""LV oracle pinned to the reference module's own outputs (tests/golden/lv_reference.json) and the
host-side checks of stein_thinning.lotka_volterra (no device)."""
import json
import os

import numpy as np
import pytest

from oracle import lv_numpy as ol

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), 'golden', 'lv_reference.json')))


def test_reference_data_is_the_modules_data():
    from stein_thinning import lotka_volterra as lv
    d = lv.reference_data()
    assert d.t.shape == (GOLDEN['t_n'],) and float(np.sum(d.t)) == GOLDEN['t_sum']
    assert np.sum(d.y, axis=0).tolist() == GOLDEN['y_sum']
    assert d.y[:5].tolist() == GOLDEN['y_head'] and d.y[-5:].tolist() == GOLDEN['y_tail']


def test_oracle_log_target_density_is_bit_identical_to_the_module():
    from stein_thinning import lotka_volterra as lv
    d = lv.reference_data()
    for lt, want in zip(GOLDEN['log_theta'], GOLDEN['log_target_density']):
        assert ol.log_target_density(np.array(lt), d.t, d.y, d.cov) == want


def test_host_argument_checks():
    from stein_thinning import lotka_volterra as lv
    d = lv.LvData(t=np.linspace(0, 25, 10), y=np.zeros((10, 2)))
    with pytest.raises(ValueError, match=r'\(n, 4\)'):
        lv.grad_log_posterior(np.zeros((3, 3)), d)
    with pytest.raises(ValueError, match='t_n'):
        lv.grad_log_posterior(np.ones(4), lv.LvData(t=np.zeros(10), y=np.zeros((9, 2))))
    with pytest.raises(ValueError, match='ascending'):
        lv.grad_log_posterior(np.ones(4), lv.LvData(t=np.linspace(25, 0, 10), y=np.zeros((10, 2))))
