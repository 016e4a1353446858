"""BASELINE configs 4 and 5 at full size and full length against the reference NumPy path's own
selections.

``tests/golden/config{4,5}_numpy_indices.json`` hold every index the NumPy restatement of the
reference loop (``JAX_Stein_Thinning.ipynb:281-295``, kernel ``:354-361``; ``oracle/stein_numpy.py``)
selects on the seeded inputs, made in the build container by ``tests/golden/make_config_golden.py``
(with the per-step argmin margin in ulps).  The GPU box regenerates the same inputs bit for bit
(``input_sha256`` is checked first; tools/input_digest.py showed identical inputs and NumPy pow on
the build container's Xeon and the MI355X box's EPYC).  Bar: all 1000 / 500 indices identical
through the drop-in ``thin`` / ``thin_gf``.
"""
import hashlib
import json
import os
import warnings

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip('torch')
if not torch.cuda.is_available():
    pytest.skip('no HIP device', allow_module_level=True)

from stein_thinning import thinning as st  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def _fixture(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def _digest(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _compare(got, fx):
    want = np.asarray(fx['indices'], dtype=np.int64)
    got = np.asarray(got, dtype=np.int64)
    assert got.shape == want.shape
    bad = np.flatnonzero(got != want)
    if bad.size:
        t = int(bad[0])
        pytest.fail(f'{bad.size} of {want.size} indices differ; first at step {t}: GPU {got[t]} vs NumPy '
                    f'{want[t]} (NumPy argmin margin at that step: {fx["margin_ulps"][t]} ulps, '
                    f'{fx["ties"][t]} tied rows)')


def test_config4_all_1000_indices_equal_numpy_reference_path():
    from bench import lv_surrogate
    fx = _fixture('config4_numpy_indices.json')
    x, g, _, _ = lv_surrogate(2_000_000, 12345)
    assert _digest(x, g) == fx['input_sha256'], 'regenerated config-4 input differs from the fixture input'
    _compare(st.thin(x, g, 1000, preconditioner='med'), fx)


def test_config5_all_500_indices_equal_numpy_reference_path():
    from bench import gaussian_d50
    fx = _fixture('config5_numpy_indices.json')
    x, log_p, log_q, gq = gaussian_d50(500_000, 12349)
    assert _digest(x, log_p, log_q, gq) == fx['input_sha256'], 'regenerated config-5 input differs'
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        _compare(st.thin_gf(x, log_p, log_q, gq, 500, preconditioner='med'), fx)
