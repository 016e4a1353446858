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
    'st_greedy': (ctypes.c_int, [_c_dp, _c_dp, _c_dp, _i64, _i32, _i64, _f64, _f64, _i64,
                                 _c_dp, _c_dp, _c_dp, _i64, _c_dp]),
    # arrays of per-problem pointers / sizes (host arrays, see st_greedy_batch)
    'st_greedy_batch': (ctypes.c_int, [_i32, _c_dp, _c_dp, _c_dp, _c_dp, _i32, _c_dp, _c_dp, _c_dp, _i64,
                                       _c_dp, _c_dp, _c_dp, _c_dp, _c_dp]),
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


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load and type the C-ABI library (no GPU access: usable for symbol checks on CPU hosts)."""
    if not os.path.exists(path):
        raise HipExtensionError(
            f'HIP extension not built: {path} is missing. Run `python -c "import __graft_entry__ as g; '
            f'g.build()"` from the repository root (hipcc --offload-arch=gfx950).')
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
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
                L = load_library(os.environ.get('ST_HIP_LIB') or LIB_PATH)
                mode = os.environ.get('ST_ARITH')
                if mode:
                    if mode not in ARITHMETIC:
                        raise ValueError(f'ST_ARITH={mode!r}: expected one of {sorted(ARITHMETIC)}')
                    L.st_tune(11, ARITHMETIC[mode])
                    global _ARITH
                    _ARITH = mode
                _LIB = L
    return _LIB


# greedy-kernel arithmetic (st_tune key 11; include/stein_thinning_hip.h)
ARITHMETIC = {'exact': 0, 'compact': 1}
_ARITH = 'compact'   # what the loaded library was last told (its default until then)


def arithmetic() -> str:
    """The arithmetic the greedy kernels use now ('compact' or 'exact'; set_arithmetic / ST_ARITH)."""
    lib()
    return _ARITH


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


def require_device():
    """Return the torch device the engine runs on; raise if no HIP device is visible."""
    import torch
    if not torch.cuda.is_available():
        raise HipExtensionError(
            'stein_thinning (MI355X engine) needs a HIP device: torch.cuda.is_available() is False. '
            'There is no CPU fallback.')
    return torch.device('cuda', torch.cuda.current_device())


def stream_handle():
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)
