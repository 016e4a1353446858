"""Generate tests/golden/lv_reference.json from the reference's own LV module
(/root/reference/code/src/lotka_volterra.py, importable in the build container: scipy only).
Run by hand in the build container; the GPU box never reads /root/reference.  The fixture pins
  * the observation data the module builds at import (t, y: checksums + a few values), and
  * log_target_density(log_theta) of the module itself at the chain initial points of the module
    and a few perturbed points,
so that stein_thinning.lotka_volterra.reference_data() and oracle.lv_numpy are checked against the
reference rather than against a restatement."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, '/root/reference/code/src')
import lotka_volterra as ref  # noqa: E402

rng = np.random.default_rng(7)
log_thetas = [np.log(np.asarray(ref.theta))] + [np.log(t) for t in ref.theta_inits] + \
    [np.log(np.asarray(ref.theta)) + 0.05 * rng.normal(size=4) for _ in range(4)]
out = {
    'source': 'code/src/lotka_volterra.py (module-level data and log_target_density)',
    't_n': int(ref.t_n), 't_span': list(ref.t_span), 'theta': list(ref.theta), 'u_init': list(ref.u_init),
    'C': np.asarray(ref.C).tolist(),
    't_sum': float(np.sum(ref.t)), 'y_sum': np.sum(ref.y, axis=0).tolist(),
    'y_head': ref.y[:5].tolist(), 'y_tail': ref.y[-5:].tolist(),
    'log_theta': [lt.tolist() for lt in log_thetas],
    'log_target_density': [float(ref.log_target_density(lt)) for lt in log_thetas],
}
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'lv_reference.json')
with open(path, 'w') as f:
    json.dump(out, f, indent=1)
print('wrote', path)
