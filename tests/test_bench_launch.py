"""bench.py's launcher contract on CPU: `--gpus N` without torchrun spawns N ranks (one process
each) instead of silently running one; a WORLD_SIZE that disagrees with --gpus is an error."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    env.update(kw)
    return env


def test_gpus_flag_spawns_ranks():
    out = subprocess.run([sys.executable, 'bench.py', '--gpus', '3', '--workload', 'ranks'], cwd=ROOT,
                         env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith('{')]
    assert lines == [{'workload': 'ranks', 'n_gpus': 3, 'rank_sum': 3}]


def test_world_size_mismatch_is_an_error():
    out = subprocess.run([sys.executable, 'bench.py', '--gpus', '2', '--workload', 'ranks'], cwd=ROOT,
                         env=_env(WORLD_SIZE='1', RANK='0'), capture_output=True, text=True, timeout=120)
    assert out.returncode == 2
    assert 'WORLD_SIZE=1 but --gpus 2' in out.stderr


def test_single_gpu_default_runs_in_process():
    out = subprocess.run([sys.executable, 'bench.py', '--workload', 'ranks'], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])['n_gpus'] == 1
