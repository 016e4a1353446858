"""Host-side controls of the native library that need no GPU (the library loads on any host): the
per-thread arithmetic override and grid cap (st_tune keys 22 / 23)."""
import pytest

from stein_thinning import _native as nat


@pytest.fixture(autouse=True)
def _lib():
    try:
        nat.lib()
    except nat.HipExtensionError as e:   # not built here
        pytest.skip(str(e))


def test_arithmetic_override_is_per_thread():
    """arithmetic_override holds for the calling host thread only (st_tune key 22): a thread
    inside an 'exact' block and one outside launch with their own arithmetic at the same time."""
    import threading
    barrier = threading.Barrier(2)
    seen = {}

    def worker(name, exact):
        if exact:
            with nat.arithmetic_override('exact'):
                barrier.wait()
                seen[name] = (nat.arithmetic(), int(nat.lib().st_tune_get(22)))
                barrier.wait()
        else:
            barrier.wait()
            seen[name] = (nat.arithmetic(), int(nat.lib().st_tune_get(22)))
            barrier.wait()
    ts = [threading.Thread(target=worker, args=('e', True)), threading.Thread(target=worker, args=('c', False))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert seen == {'e': ('exact', 0), 'c': ('compact', -1)}
    assert nat.arithmetic() == 'compact' and int(nat.lib().st_tune_get(22)) == -1


def test_grid_cap_is_per_thread_and_nests():
    L = nat.lib()
    base = int(L.st_tune_get(5))
    with nat.grid_cap(64):
        assert int(L.st_tune_get(23)) == 64
        with nat.grid_cap(0):
            assert int(L.st_tune_get(23)) == -1
        assert int(L.st_tune_get(23)) == 64
        assert int(L.st_tune_get(5)) == base   # the process-wide key is untouched
    assert int(L.st_tune_get(23)) == -1


def test_arithmetic_override_nests():
    with nat.arithmetic_override('exact'):
        with nat.arithmetic_override('compact'):
            assert nat.arithmetic() == 'compact' and int(nat.lib().st_tune_get(22)) == 1
        assert nat.arithmetic() == 'exact' and int(nat.lib().st_tune_get(22)) == 0
    assert int(nat.lib().st_tune_get(22)) == -1
