"""The C-ABI library loads (no GPU needed) and exports every function include/*.h declares."""
import glob
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in glob.glob(os.path.join(ROOT, 'include', '*.h')):
        src = open(h).read()
        src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
        names |= set(re.findall(r'^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*(st_[a-z0-9_]+)\s*\(', src, flags=re.M))
    return names


@pytest.fixture(scope='module')
def libpath():
    import __graft_entry__ as ge
    ge.build()
    return ge.HIP_LIB


def test_header_declares_api():
    names = _declared()
    for must in ['st_greedy', 'st_greedy_step', 'st_greedy_finalize', 'st_kernel_pairs', 'st_ksd_cumulative',
                 'st_kmat', 'st_last_error', 'st_abi_version', 'st_layout_soa']:
        assert must in names


def test_library_exports_every_declared_symbol(libpath):
    out = subprocess.run(['nm', '-D', '--defined-only', libpath], capture_output=True, text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = _declared() - exported
    assert not missing, missing


def test_library_loads_and_types_without_gpu(libpath):
    from stein_thinning import _native
    lib = _native.load_library(libpath)
    assert lib.st_abi_version() == _native.ABI_VERSION
    assert set(_native.SIGNATURES) == _declared()
    # host-only entry points: sizes and argument validation (no device memory touched)
    assert lib.st_candidate_stride(4) == 12
    assert lib.st_greedy_workspace_bytes(10, 4, 1) > 0
    assert lib.st_greedy_workspace_bytes(10, 129, 1) == -1
    assert lib.st_greedy(None, None, None, 10, 4, 10, 1.0, 4.0, 5, None, None, None, 0, None) == _native.ST_ERR_INVALID
    assert b'NULL' in lib.st_last_error()
    assert lib.st_kernel_pairs(None, None, None, 8, 200, 1.0, 1.0, None, None, 1, None, None) == _native.ST_ERR_INVALID


def test_host_side_validation_of_the_newer_entry_points(libpath):
    """Argument checks that fail before any HIP call (no device needed): multi-GPU greedy, mailbox
    sizing, KSD column sums, energy-distance column sums, host standardisation."""
    import ctypes
    from stein_thinning import _native
    lib = _native.load_library(libpath)
    inv = _native.ST_ERR_INVALID
    assert lib.st_mailbox_bytes(1) > 0 and lib.st_mailbox_bytes(8) >= lib.st_mailbox_bytes(1)
    assert lib.st_mailbox_bytes(0) == -1 and lib.st_mailbox_bytes(9) == -1
    assert lib.st_ipc_handle_bytes() == 64
    # st_greedy_sharded: NULL arrays, then nranks / rank / peer table / row range checks
    args = [None, None, None, 10, 4, 16, 1.0, 4.0, 0, 10, 0, 2, None, 0, 5, None, None, None, 0, None]
    assert lib.st_greedy_sharded(*args) == inv
    buf = (ctypes.c_double * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    base = [p, p, None, 10, 4, 16, 1.0, 4.0, 0, 10, 0, 2, None, 0, 5, p, p, p, 1 << 20, None]
    assert lib.st_greedy_sharded(*base) == inv                    # no peer table
    assert b'peer' in lib.st_last_error()
    table = (ctypes.c_void_p * 8)(p.value, p.value)
    tp = ctypes.cast(table, ctypes.c_void_p)
    for k, bad in [(11, 1), (11, 9), (10, 2), (8, 10), (9, 11)]:   # nranks 1 / 9, rank 2, row range
        a = list(base)
        a[12] = tp
        a[k] = bad
        assert lib.st_greedy_sharded(*a) == inv, (k, bad)
    # st_greedy_step_exchange: peer table / status checks
    step = [p, p, None, 10, 9, 16, 1.0, 4.0, 0, 0, 0, 2, None, p, p, p, p, 1 << 20, p, None]
    assert lib.st_greedy_step_exchange(*step) == inv               # no peer table
    step[12] = tp
    step[18] = None
    assert lib.st_greedy_step_exchange(*step) == inv               # no status word
    step[18] = p
    step[16] = None
    assert lib.st_greedy_step_exchange(*step) == inv               # no workspace
    assert lib.st_mailbox_handshake(tp, 1, 0, 1, p, None) == inv
    assert lib.st_mailbox_handshake(tp, 2, 0, 1 << 63, p, None) == inv
    # KSD column sums / finish
    assert lib.st_ksd_colsum(p, p, None, 10, 16, 4, 1.0, 4.0, 3, 2, p, None) == inv   # row_end < row_begin
    assert lib.st_ksd_colsum(p, p, None, 10, 16, 4, 1.0, 4.0, 0, 11, p, None) == inv  # row_end > n
    assert lib.st_ksd_finish(p, p, None, 10, 16, 4, 1.0, 4.0, None, p, None) == inv
    # energy-distance column sums
    assert lib.st_distance_colsum(p, 16, 10, p, 16, 10, 4, 0, 10, 0, None, None) == inv
    assert lib.st_distance_colsum(p, 12, 10, p, 16, 10, 4, 0, 10, 0, p, None) == inv   # ld % 8
    assert lib.st_distance_colsum(p, 16, 10, p, 16, 10, 4, 0, 11, 0, p, None) == inv   # range
    assert lib.st_distance_colsum(p, 16, 10, None, 16, 10, 4, 0, 10, 1, p, None) == inv
    assert lib.st_distance_colsum(p, 16, 10, p, 16, 10, 200, 0, 10, 0, p, None) == _native.ST_ERR_UNSUPPORTED
    # host standardisation: bad arguments
    status = ctypes.c_int32(0)
    assert lib.st_standardize_host(None, None, 10, 4, 1, None, None, None, None, ctypes.byref(status)) == inv
    # standardisation with the upload underneath: NULLs, unaligned staging, and the cases it leaves to
    # st_standardize_host (d outside 2 .. 8, n < 65536) -- all before any HIP call
    st = [p, p, 100_000, 4, p, p, p, p, p, p, ctypes.byref(status), None]
    assert lib.st_standardize_upload(None, *st[1:]) == inv
    odd = ctypes.c_void_p(p.value + 8)
    assert lib.st_standardize_upload(*(st[:4] + [odd] + st[5:])) == inv
    assert lib.st_standardize_upload(*(st[:3] + [9] + st[4:])) == _native.ST_ERR_UNSUPPORTED
    assert lib.st_standardize_upload(*(st[:2] + [1000] + st[3:])) == _native.ST_ERR_UNSUPPORTED
    # the device-tensor counterpart: NULLs and empty inputs
    assert lib.st_standardize_download(None, 100, 4, p, p, p, ctypes.byref(status), None) == inv
    assert lib.st_standardize_download(p, 0, 4, p, p, p, ctypes.byref(status), None) == inv
    assert lib.st_standardize_download(p, 100, 0, p, p, p, ctypes.byref(status), None) == inv
    # near-tie guard: the flag read-back's checks, the switch and its read-back (host-only state)
    step = ctypes.c_int64(0)
    assert lib.st_greedy_near_tie(None, 4096, ctypes.byref(step), None) == inv
    assert lib.st_greedy_near_tie(p, 64, ctypes.byref(step), None) == inv
    assert lib.st_tune_get(20) in (0, 1)
    assert lib.st_tune_get(999) == -2 ** 31   # INT32_MIN: no such key
    # repeated-row compaction, scaled layout, 'med' distances
    assert lib.st_run_workspace_bytes(1) > 0 and lib.st_run_workspace_bytes(1 << 20) >= 8 + 8 * 1024
    assert lib.st_run_starts(p, p, None, 10, 4, 16, None, p, 1 << 10, None) == inv          # no output
    assert lib.st_run_starts(p, p, None, 10, 4, 16, p, p, 8, None) == inv                   # workspace too small
    assert lib.st_run_starts(p, p, None, 10, 4, 12, p, p, 1 << 10, None) == inv             # ld % 8
    assert lib.st_run_compact(p, p, None, 10, 4, 16, p, p, 11, 16, p, p, None, p, None) == inv   # count > n
    assert lib.st_run_compact(p, p, None, 10, 4, 16, p, p, 5, 4, p, p, None, p, None) == inv     # ld_out < count
    assert lib.st_run_compact(p, p, p, 10, 4, 16, p, p, 5, 8, p, p, None, p, None) == inv        # weights, no w_out
    assert lib.st_layout_soa_scaled(p, 10, 4, 8, p, 1, p, None) == inv                     # ld < n
    assert lib.st_layout_soa_scaled(p, 10, 4, 16, None, 1, p, None) == inv                 # no scale
    assert lib.st_pdist(p, 1, 4, p, None) == inv and lib.st_pdist(p, 70_000, 4, p, None) == inv
    assert lib.st_pdist(p, 10, 0, p, None) == inv and lib.st_pdist(None, 10, 4, p, None) == inv
    # batch launch: count, NULL arrays, per-problem checks (weights for some problems only, ld % 8,
    # workspace size) -- all before any HIP call
    def arr(ctype, vals):
        return (ctype * len(vals))(*vals)
    P2 = arr(ctypes.c_void_p, [p.value, p.value])
    N2, LD2 = arr(ctypes.c_int64, [10, 10]), arr(ctypes.c_int64, [16, 16])
    F2 = arr(ctypes.c_double, [1.0, 1.0])
    WS2 = arr(ctypes.c_int64, [1 << 24, 1 << 24])
    batch = [2, P2, P2, None, N2, 4, LD2, F2, F2, 5, P2, P2, P2, WS2, None]
    for k, bad in [(0, 0), (0, 9), (1, None), (6, None), (13, None), (9, 0)]:
        a = list(batch)
        a[k] = bad
        assert lib.st_greedy_batch(*a) == inv, (k, bad)
    a = list(batch)
    a[3] = arr(ctypes.c_void_p, [p.value, None])                      # weights for one problem only
    assert lib.st_greedy_batch(*a) == inv and b'weights' in lib.st_last_error()
    a = list(batch)
    a[6] = arr(ctypes.c_int64, [16, 12])                              # ld % 8
    assert lib.st_greedy_batch(*a) == inv
    a = list(batch)
    a[13] = arr(ctypes.c_int64, [1 << 24, 8])                         # workspace too small
    assert lib.st_greedy_batch(*a) == inv and b'problem 1' in lib.st_last_error()


def test_library_is_gfx950_only(libpath):
    # the embedded code-object bundle names its target: amdgcn-amd-amdhsa--gfx950
    blob = open(libpath, 'rb').read()
    targets = set(re.findall(rb'amdgcn-amd-amdhsa--(gfx[0-9a-z]+)', blob))
    assert targets == {b'gfx950'}, targets


def test_tune_keys_validate_without_gpu(libpath):
    """st_tune only records host-side knobs: valid values are accepted and restored, invalid ones
    rejected (record replicas: powers of two 1..32; record pitch: powers of two 16..4096)."""
    from stein_thinning import _native
    lib = _native.load_library(libpath)
    for key, good, bad in [(10, [1, 2, 16, 32], [0, 3, 64]), (9, [16, 256, 4096], [8, 24, 8192]),
                           (4, [256, 512], [128, 1024]), (8, [1], [2, 3]), (11, [0, 1], [2, -2]),
                           (12, [0, 8, 9], [4, 6, 7, 10, 11]), (13, [0, 1, 2, 5, 6], [7, -2]),
                           (3, [0, 1, 2, 4, 8, 16], [3, 6, 32]), (22, [0, 1], [2, -2]), (23, [1, 64, 512], [0, 513]),
                           (17, [0, 1], [2, -2]), (18, [1, 2, 3], [0, 4]), (19, [0, 1], [2, -2])]:
        for v in good:
            assert lib.st_tune(key, v) == 0, (key, v)
        for v in bad:
            assert lib.st_tune(key, v) != 0, (key, v)
        assert lib.st_tune(key, -1) == 0
    assert lib.st_tune(99, 1) != 0


def test_set_arithmetic_is_host_only_and_validates(libpath):
    """stein_thinning.set_arithmetic (st_tune key 11) records a host-side knob: both modes are
    accepted without a GPU, anything else is rejected before reaching the library."""
    import stein_thinning
    with pytest.raises(ValueError):
        stein_thinning.set_arithmetic('fast')
    stein_thinning.set_arithmetic('exact')
    stein_thinning.set_arithmetic('compact')
