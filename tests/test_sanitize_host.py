"""Host-code sanitizers: the native input preparation under ASan + UBSan
(scripts/sanitize_host.sh asan).  The TSan and C-ABI argument-validation builds of the same script
take minutes and are run per round (log: profiles/r02_sanitize_host.log)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('g++') is None, reason='needs g++')
def test_host_prep_asan_ubsan():
    out = subprocess.run(['bash', 'scripts/sanitize_host.sh', 'asan'], cwd=ROOT, capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert 'ok: 0 failure(s)' in out.stdout
