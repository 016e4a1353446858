"""ctypes binding of the HIP C-ABI (include/stein_thinning_hip.h).

The shared library ``_lib/libstein_hip.so`` is built in-tree by ``__graft_entry__.build()``
(hipcc --offload-arch=gfx950).  Nothing here touches HIP at import time (the reference calls the
library from joblib / Dask worker processes, ``code/src/utils/parallel.py:18-52``); the library is
loaded on first use, after ``torch`` so that exactly one HIP runtime (torch's
``libamdhip64.so.7``) is mapped into the process.  There is no CPU fallback: every entry point
raises if the extension or a HIP device is missing.
"""
from __future__ import annotations

import ctypes
import os
import threading

_LIB = None
_LOCK = threading.Lock()

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), '_lib', 'libstein_hip.so')

ST_OK = 0
ST_ERR_INVALID = -1
ST_ERR_UNSUPPORTED = -2
ST_ERR_HIP = -3

_c_dp = ctypes.c_void_p  # device pointers / stream handles
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_f64 = ctypes.c_double

# symbol -> (restype, argtypes); mirrors include/stein_thinning_hip.h
SIGNATURES = {
    'st_abi_version': (ctypes.c_int, []),
    'st_last_error': (ctypes.c_char_p, []),
    'st_greedy_workspace_bytes': (_i64, [_i64, _i32, _i32]),
    'st_candidate_stride': (_i64, [_i32]),
    'st_tune': (ctypes.c_int, [_i32, _i32]),
    'st_tune_get': (_i32, [_i32]),
    'st_greedy': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _f64, _f64, _i64,
                                 _c_dp, _c_dp, _c_dp, _i64, _c_dp]),
    # arrays of per-problem pointers / sizes (host arrays, see st_greedy_batch)
    'st_greedy_batch': (ctypes.c_int, [_i32, _c_dp, _c_dp, _c_dp, _c_dp, _i32, _c_dp, _c_dp, _c_dp, _i64,
                                       _c_dp, _c_dp, _c_dp, _c_dp, _c_dp]),
    'st_greedy_near_tie': (ctypes.c_int, [_c_dp, _i64, ctypes.POINTER(_i64), _c_dp]),
    'st_greedy_steps': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _f64, _f64, _i64,
                                       _i64, _i64, _c_dp, _c_dp, _c_dp, _i64, _c_dp]),
    'st_greedy_step': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _f64, _f64,
                                      _i64, _i64, _i32, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp,
                                      _i64, _c_dp]),
    'st_greedy_finalize': (ctypes.c_int, [_c_dp, _i32, _i32, _c_dp, _i64, _c_dp]),
    'st_kernel_pairs': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _f64, _f64, _c_dp,
                                       _c_dp, _i64, _c_dp, _c_dp]),
    'st_ksd_workspace_bytes': (_i64, [_i64, _i64]),
    'st_ksd_cumulative': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i64, _i32, _f64, _f64,
                                         _c_dp, _c_dp, _i64, _c_dp]),
    'st_kmat': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i64, _i32, _f64, _f64, _c_dp,
                               _c_dp]),
    'st_layout_soa': (ctypes.c_int, [_c_dp, _i64, _i32, _i64, _c_dp, _c_dp]),
    'st_pdist': (ctypes.c_int, [_c_dp, _i64, _i32, _c_dp, _c_dp]),
    'st_layout_soa_scaled': (ctypes.c_int, [_c_dp, _i64, _i32, _i64, _c_dp, _i32, _c_dp, _c_dp]),
    'st_standardize_download': (ctypes.c_int, [_c_dp, _i64, _i32, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp]),
    'st_standardize_upload': (ctypes.c_int, [_c_dp, _c_dp, _i64, _i32, _c_dp, _c_dp, _c_dp, _c_dp,
                                             _c_dp, _c_dp, _c_dp, _c_dp]),
    'st_run_workspace_bytes': (_i64, [_i64]),
    'st_run_starts': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _c_dp, _c_dp, _i64, _c_dp]),
    'st_run_compact': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _c_dp, _c_dp, _i64, _i64,
                                      _c_dp, _c_dp, _c_dp, _c_dp, _c_dp]),
    'st_ksd_colsum': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i64, _i32, _f64, _f64, _i64, _i64,
                                     _c_dp, _c_dp]),
    'st_ksd_finish': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i64, _i32, _f64, _f64, _c_dp,
                                     _c_dp, _c_dp]),
    'st_distance_colsum': (ctypes.c_int, [_c_dp, _i64, _i64, _c_dp, _i64, _i64, _i32, _i64, _i64,
                                          _i32, _c_dp, _c_dp]),
    'st_distance_workspace_bytes': (_i64, [_i64, _i64, _i64]),
    'st_distance_colsum_ws': (ctypes.c_int, [_c_dp, _i64, _i64, _c_dp, _i64, _i64, _i32, _i64, _i64,
                                             _i32, _c_dp, _c_dp, _i64, _c_dp]),
    'st_standardize_host': (ctypes.c_int, [_c_dp, _c_dp, _i64, _i32, _i32, _c_dp, _c_dp, _c_dp, _c_dp,
                                           ctypes.POINTER(ctypes.c_int32)]),
    'st_mailbox_bytes': (_i64, [_i32]),
    'st_mailbox_alloc': (ctypes.c_int, [_i64, ctypes.POINTER(ctypes.c_void_p)]),
    'st_mailbox_free': (ctypes.c_int, [_c_dp]),
    'st_ipc_handle_bytes': (ctypes.c_int, []),
    'st_ipc_get_handle': (ctypes.c_int, [_c_dp, _c_dp]),
    'st_ipc_open_handle': (ctypes.c_int, [_c_dp, ctypes.POINTER(ctypes.c_void_p)]),
    'st_ipc_close_handle': (ctypes.c_int, [_c_dp]),
    'st_mailbox_handshake': (ctypes.c_int, [_c_dp, _i32, _i32, ctypes.c_uint64, _c_dp, _c_dp]),
    'st_greedy_sharded': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _f64, _f64,
                                         _i64, _i64, _i32, _i32, _c_dp, ctypes.c_uint64, _i64,
                                         _c_dp, _c_dp, _c_dp, _i64, _c_dp]),
    'st_greedy_sharded_supported': (ctypes.c_int, [_i64, _i32, _i32, _i64, _i64, _i32, _i32, _i64]),
    'st_greedy_step_exchange': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _f64, _f64,
                                               _i64, _i64, _i32, _i32, _c_dp, _c_dp, _c_dp, _c_dp,
                                               _c_dp, _i64, _c_dp, _c_dp]),
    'st_lv_grad_log_posterior': (ctypes.c_int, [_c_dp, _i64, _c_dp, _i32, _c_dp, _c_dp, _c_dp, _i64, _c_dp,
                                                _c_dp, _c_dp]),
    'st_lv_grad_workspace_bytes': (_i64, [_i64, _i32]),
    'st_lv_grad_log_posterior_ws': (ctypes.c_int, [_c_dp, _i64, _c_dp, _i32, _c_dp, _c_dp, _c_dp, _i64, _c_dp,
                                                   _c_dp, _c_dp, _i64, _c_dp]),
    'st_lv_log_density_workspace_bytes': (_i64, [_i64, _i32]),
    'st_lv_log_target_density': (ctypes.c_int, [_c_dp, _c_dp, _i64, _c_dp, _i32, _c_dp, _c_dp, _c_dp, _f64,
                                                _f64, _i64, _c_dp, _c_dp, _c_dp, _i64, _c_dp]),
    'st_kde_workspace_bytes': (_i64, [_i64, _i32]),
    'st_kde_logpdf_grad': (ctypes.c_int, [_c_dp, _i64, _i64, _c_dp, _f64, _c_dp, _i64, _i64, _i32, _f64, _c_dp,
                                          _c_dp, _c_dp, _c_dp, _i64, _c_dp]),
    'st_proxy_logpdf_grad': (ctypes.c_int, [_c_dp, _i64, _i32, _c_dp, _c_dp, _c_dp, _f64, _f64, _c_dp,
                                            _c_dp, _c_dp]),
}
ABI_VERSION = 1


class HipExtensionError(RuntimeError):
    """The HIP extension is missing, failed to load, or reported an error."""


def load_library(path: str = LIB_PATH, partial: bool = False) -> ctypes.CDLL:
    """Load and type the C-ABI library (no GPU access: usable for symbol checks on CPU hosts).
    ``partial``: an older build of the same ABI (ST_HIP_LIB, same-box A/B timing) may lack newer entry
    points; they raise when called."""
    if not os.path.exists(path):
        raise HipExtensionError(
            f'HIP extension not built: {path} is missing. Run `python -c "import __graft_entry__ as g; '
            f'g.build()"` from the repository root (hipcc --offload-arch=gfx950).')
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if not partial:
                raise

            def missing(*_a, _name=name):
                raise HipExtensionError(f'{_name}: not in {path} (an older build)')
            setattr(lib, name, missing)
            continue
        fn.restype = res
        fn.argtypes = args
    if lib.st_abi_version() != ABI_VERSION:
        raise HipExtensionError(f'ABI mismatch: library {lib.st_abi_version()} != {ABI_VERSION}')
    return lib


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        with _LOCK:
            if _LIB is None:
                import torch  # noqa: F401  -- map torch's HIP runtime before ours resolves against it
                # ST_HIP_LIB: another build of the same ABI (same-box A/B timing of a kernel change,
                # scripts/ab_run.sh); the in-tree library otherwise
                alt = os.environ.get('ST_HIP_LIB')
                L = load_library(alt or LIB_PATH, partial=bool(alt))
                mode = os.environ.get('ST_ARITH')
                if mode:
                    if mode not in ARITHMETIC:
                        raise ValueError(f'ST_ARITH={mode!r}: expected one of {sorted(ARITHMETIC)}')
                    L.st_tune(11, ARITHMETIC[mode])
                    global _ARITH
                    _ARITH = mode
                L.st_tune(20, 1 if near_tie_guard() else 0)   # (an older A/B build rejects the key: harmless)
                _LIB = L
    return _LIB


# greedy-kernel arithmetic (st_tune key 11; include/stein_thinning_hip.h)
ARITHMETIC = {'exact': 0, 'compact': 1}
_ARITH = 'compact'   # what the loaded library was last told (its default until then)


_TL = threading.local()   # this host thread's arithmetic_override (st_tune key 22), None: the process mode


def arithmetic() -> str:
    """The arithmetic the greedy kernels launched from this thread use now ('compact' or 'exact'):
    an enclosing arithmetic_override, else the process-wide mode (set_arithmetic / ST_ARITH)."""
    lib()
    mode = getattr(_TL, 'mode', None)
    return _ARITH if mode is None else mode


def set_arithmetic(mode: str) -> None:
    """Arithmetic of the d <= 8 greedy kernels (thin / thin_gf / _greedy_search on a Stein integrand).

    'compact' (default): the IMQ Stein-kernel value regrouped around one correctly rounded reciprocal
    square root -- a few ulps from NumPy's evaluation of vfk0_imq, ~2.3x fewer fp64 instructions per
    pair; selections equal the reference's on every fixture it holds (tests/test_oracle_compact.py).
    'exact': NumPy's evaluation order, rounding for rounding (correctly rounded powers).  Pairs with a
    coordinate outside [2^-60, 2^60] always take the exact arithmetic.  Process-wide; every rank of a
    sharded run must use the same mode (ST_ARITH in the environment sets it at library load)."""
    if mode not in ARITHMETIC:
        raise ValueError(f'arithmetic {mode!r}: expected one of {sorted(ARITHMETIC)}')
    check(lib().st_tune(11, ARITHMETIC[mode]), 'set_arithmetic')
    global _ARITH
    _ARITH = mode


_GUARD = None   # set_near_tie_guard(); None: the ST_NEAR_TIE environment variable ('0' = off; on by default)


def set_near_tie_guard(enabled) -> None:
    """Near-tie guard of the compact arithmetic (st_tune key 20), on by default: a compact-arithmetic thin
    whose selection at some step rests on sums closer than the arithmetic's error band is re-run with the
    exact arithmetic, so the drop-in thin selects the reference NumPy path's rows.
    True / False, or None to return to the ST_NEAR_TIE environment variable."""
    global _GUARD
    _GUARD = None if enabled is None else bool(enabled)
    check(lib().st_tune(20, 1 if near_tie_guard() else 0), 'set_near_tie_guard')


def near_tie_guard() -> bool:
    if _GUARD is not None:
        return _GUARD
    return os.environ.get('ST_NEAR_TIE', '1') != '0'


class arithmetic_override:
    """``with arithmetic_override('exact'): ...`` -- the greedy kernels' arithmetic for the launches this
    host thread enqueues inside the block.  Thread-local (st_tune key 22: the library keeps the override
    per host thread), so concurrent threads -- thin_chains runs one per GPU -- never see each other's
    mode; blocks nest (the previous override is restored on exit)."""

    def __init__(self, mode: str):
        if mode not in ARITHMETIC:
            raise ValueError(f'arithmetic {mode!r}: expected one of {sorted(ARITHMETIC)}')
        self.mode = mode

    def __enter__(self):
        L = lib()
        self.prev = getattr(_TL, 'mode', None)
        check(L.st_tune(22, ARITHMETIC[self.mode]), 'arithmetic_override')
        _TL.mode = self.mode
        return self

    def __exit__(self, *exc):
        check(lib().st_tune(22, -1 if self.prev is None else ARITHMETIC[self.prev]), 'arithmetic_override')
        _TL.mode = self.prev
        return False


class grid_cap:
    """``with grid_cap(k): ...`` -- at most k blocks per persistent-kernel grid for the launches this host
    thread enqueues inside the block (st_tune key 23, per host thread; st_tune key 5 is the process-wide
    cap); k <= 0: no cap of this thread's own."""

    def __init__(self, blocks: int):
        self.blocks = int(blocks)

    def __enter__(self):
        L = lib()
        self.prev = int(L.st_tune_get(23))
        check(L.st_tune(23, self.blocks if self.blocks > 0 else -1), 'grid_cap')
        return self

    def __exit__(self, *exc):
        check(lib().st_tune(23, self.prev), 'grid_cap')
        return False


def near_tie_step(ws) -> int:
    """First flagged step of the completed greedy run whose workspace is ``ws`` (a device tensor), -1 when
    none, -2 when the run was not guarded (st_greedy_near_tie; synchronises the current stream)."""
    out = ctypes.c_int64(0)
    check(lib().st_greedy_near_tie(ptr(ws), ws.numel() * ws.element_size(), ctypes.byref(out), stream_handle()),
          'st_greedy_near_tie')
    return int(out.value)


def check_host(rc: int, what: str = '') -> None:
    if rc != ST_OK:
        raise ValueError(f'{what}: invalid arguments ({rc})')


def check(rc: int, what: str = '') -> None:
    if rc != ST_OK:
        msg = lib().st_last_error().decode(errors='replace')
        if rc == ST_ERR_UNSUPPORTED:
            raise NotImplementedError(f'{what}: {msg}')
        if rc == ST_ERR_INVALID:
            raise ValueError(f'{what}: {msg}')
        raise HipExtensionError(f'{what}: HIP error ({rc}): {msg}')


# worker processes of the pools the reference fans thin() out with (joblib's loky / multiprocessing backends,
# concurrent.futures): "LokyProcess-3", "ForkPoolWorker-3", "SpawnPoolWorker-3", "ForkServerPoolWorker-3",
# "SpawnProcess-3" / "ForkProcess-3" / "ForkServerProcess-3" (ProcessPoolExecutor).  A user's own
# multiprocessing.Process ("Process-3") or a DataLoader worker is not a pool worker: no policy there.
POOL_WORKER_NAMES = r'^(?:LokyProcess|ForkPoolWorker|SpawnPoolWorker|ForkServerPoolWorker|SpawnProcess|ForkProcess|' \
                    r'ForkServerProcess)-(\d+)$'


def select_device_index(count: int, env=None, worker: bool = False, pid: int = 0, worker_name: str = ''):
    """The device policy of a process (pure: tests call it with a mocked device count):
    * ``ST_DEVICE`` in the environment: that device (an index < count);
    * else ``LOCAL_RANK`` (torchrun / torch.distributed.run: one process per GPU): LOCAL_RANK % count;
    * else, in a worker process of a pool (joblib's loky / multiprocessing backends, concurrent.futures --
      the reference fans ``thin`` out over chains in such workers, ``code/src/utils/parallel.py:48-52``;
      POOL_WORKER_NAMES) with several devices: the worker's ordinal from its process name
      ("LokyProcess-3", "ForkPoolWorker-3", "SpawnProcess-3": (3 - 1) % count -- the pool's workers
      round-robin over the GPUs), a Dask nanny worker ("Dask Worker process ...") its pid % count; any other
      child process (a user's own multiprocessing.Process, a DataLoader worker) gets no policy;
    * else None: the current torch device (cuda:0 unless the caller chose another).
    Returns the device index or None."""
    env = os.environ if env is None else env
    v = env.get('ST_DEVICE')
    if v is not None and v != '':
        try:
            idx = int(v)
        except ValueError:
            raise ValueError(f'ST_DEVICE={v!r}: expected a device index') from None
        if not 0 <= idx < count:
            raise ValueError(f'ST_DEVICE={idx}: only {count} HIP device(s) visible')
        return idx
    v = env.get('LOCAL_RANK')
    if v is not None and v != '' and count > 0:
        return int(v) % count
    if worker and count > 1:
        import re
        k = re.match(POOL_WORKER_NAMES, worker_name or '')
        if k:
            return (int(k.group(1)) - 1) % count
        if (worker_name or '').startswith('Dask Worker'):   # Dask's nanny workers carry no ordinal: the pid
            return pid % count
    return None


_DEVICE_POLICY_DONE = False


def _pool_worker() -> bool:
    import multiprocessing
    return multiprocessing.parent_process() is not None


def require_device():
    """Return the torch device the engine runs on; raise if no HIP device is visible.  On first use the
    process applies ``select_device_index`` (ST_DEVICE, LOCAL_RANK, or a pool worker's share of the GPUs)
    with torch.cuda.set_device; without a policy it uses the current device, so ``with
    torch.cuda.device(k)`` blocks are honoured."""
    import torch
    if not torch.cuda.is_available():
        raise HipExtensionError(
            'stein_thinning (MI355X engine) needs a HIP device: torch.cuda.is_available() is False. '
            'There is no CPU fallback.')
    global _DEVICE_POLICY_DONE
    if not _DEVICE_POLICY_DONE:
        _DEVICE_POLICY_DONE = True
        idx = _policy_index()
        # a device the caller already chose (torch.cuda.set_device / with torch.cuda.device(k): not the
        # default 0) is kept; the policy only moves a process that is still on the default device
        if idx is not None and idx != torch.cuda.current_device() and torch.cuda.current_device() == 0:
            torch.cuda.set_device(idx)
    return torch.device('cuda', torch.cuda.current_device())


def _policy_index():
    import multiprocessing
    import torch
    return select_device_index(torch.cuda.device_count(), os.environ, _pool_worker(), os.getpid(),
                               multiprocessing.current_process().name)


def policy_pinned() -> bool:
    """True when the process's device comes from the policy (ST_DEVICE, LOCAL_RANK, a pool worker):
    thin_chains then keeps every chain on that device instead of spreading them over all GPUs."""
    return _policy_index() is not None


def stream_handle():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
