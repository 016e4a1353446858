"""Device policy of a process (stein_thinning._native.select_device_index): the
reference thins its chains in joblib worker processes (code/src/utils/parallel.py:48-52) and torchrun
starts one process per GPU; both must spread over the node's GPUs instead of piling onto cuda:0.
CPU-only: the device count is passed in."""
import pytest

from stein_thinning import _native as nat


def test_explicit_device_wins():
    assert nat.select_device_index(8, {'ST_DEVICE': '3', 'LOCAL_RANK': '5'}, worker=True, pid=7) == 3
    with pytest.raises(ValueError, match='only 2'):
        nat.select_device_index(2, {'ST_DEVICE': '2'})
    with pytest.raises(ValueError, match='device index'):
        nat.select_device_index(2, {'ST_DEVICE': 'gpu1'})


def test_local_rank_one_process_per_gpu():
    assert [nat.select_device_index(8, {'LOCAL_RANK': str(r)}) for r in range(8)] == list(range(8))
    assert nat.select_device_index(4, {'LOCAL_RANK': '6'}) == 2
    assert nat.select_device_index(1, {'LOCAL_RANK': '3'}) == 0


def test_pool_workers_spread_round_robin():
    # five joblib workers (the reference's five chains): the pool's own worker ordinals (loky /
    # multiprocessing / concurrent.futures names) give an exact round-robin
    names = [f'LokyProcess-{k}' for k in range(1, 6)]
    assert [nat.select_device_index(8, {}, worker=True, pid=9, worker_name=nm) for nm in names] == [0, 1, 2, 3, 4]
    assert nat.select_device_index(4, {}, worker=True, pid=9, worker_name='ForkPoolWorker-6') == 1
    assert nat.select_device_index(4, {}, worker=True, pid=9, worker_name='SpawnProcess-3') == 2
    # Dask's nanny workers carry no ordinal: their pids spread them
    got = [nat.select_device_index(8, {}, worker=True, pid=4000 + k, worker_name='Dask Worker process (from Nanny)')
           for k in range(5)]
    assert len(set(got)) == 5
    assert nat.select_device_index(1, {}, worker=True, pid=4001, worker_name='LokyProcess-2') is None   # one device
    assert nat.select_device_index(8, {}, worker=False, pid=4001) is None  # the main process: current device


def test_other_child_processes_get_no_policy():
    """a user's own multiprocessing.Process or a DataLoader worker is not a pool worker -- its
    device stays the caller's choice (require_device also keeps any non-default device already set)."""
    for nm in ['Process-3', 'MainProcess', '', 'Dask-like worker 2']:
        assert nat.select_device_index(8, {}, worker=True, pid=4003, worker_name=nm) is None


def test_no_hip_initialisation_at_import():
    """The policy is applied on first use (require_device), never at import: importing the package in a
    pool worker must not touch HIP (fork / spawn safety)."""
    import subprocess
    import sys
    code = ('import sys; sys.path.insert(0, "gradient-free-mcmc-postprocessing_amd"); import torch; '
            'import stein_thinning, stein_thinning.thinning, stein_thinning.device; '
            'print(torch.cuda.is_initialized())')
    out = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, check=True)
    assert out.stdout.strip() == 'False'
