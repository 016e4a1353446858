"""HBM-resident problem: the standardised sample / score (SoA fp64) plus optional weights.

Data layout in HBM (DESIGN.md "Data layout"): element (i, k) of an (n, d) array lives at
``soa[k * ld + i]`` with ``ld`` = n rounded up to a multiple of 64, so that every candidate column
is a coalesced, 512-byte-aligned fp64 stream and a lane reads two adjacent candidates with one
16-byte load.  Weights and running sums are (ld,) vectors.  Padding rows are zero and never enter
an argmin.
"""
from __future__ import annotations

import contextlib
import warnings
from typing import Optional

import numpy as np

from . import _native as nat

PAD = 64
# thin the run starts instead of all rows when at most this fraction of the rows start a run ...
DEDUP_MAX_FRAC = 0.9
# ... and (greedy(dedup=True)) the pair work it saves is estimated at >= this many seconds
DEDUP_MIN_SAVING_S = 50e-6


def padded_ld(n: int) -> int:
    return max(PAD, ((n + PAD - 1) // PAD) * PAD)


class DedupView:
    """A problem's run starts as a compact DeviceProblem (DeviceProblem.dedup_view) and the maps
    between the two index spaces (the compaction keeps row order, so a lower index stays lower)."""

    def __init__(self, parent: 'DeviceProblem', starts, ws, count: int):
        import torch
        d, dev = parent.d, parent.device
        ld = padded_ld(count)
        x = torch.empty((d, ld), dtype=torch.float64, device=dev)
        g = torch.empty((d, ld), dtype=torch.float64, device=dev)
        w = torch.empty(ld, dtype=torch.float64, device=dev) if parent.w is not None else None
        self.rows = torch.empty(count, dtype=torch.int32, device=dev)   # compact row -> source row
        nat.check(nat.lib().st_run_compact(
            nat.ptr(parent.x), nat.ptr(parent.g), nat.ptr(parent.w), parent.n, d, parent.ld, nat.ptr(starts),
            nat.ptr(ws), count, ld, nat.ptr(x), nat.ptr(g), nat.ptr(w), nat.ptr(self.rows),
            nat.stream_handle()), 'st_run_compact')
        self.starts = starts                                   # (n,) uint8: row starts a run
        self.problem = DeviceProblem.from_soa(x, g, w, count, parent.l, parent.tr)

    @property
    def n_unique(self) -> int:
        return self.problem.n

    @property
    def rows_host(self) -> np.ndarray:
        return self.rows.cpu().numpy().astype(np.uint32)

    def to_rows(self, compact_idx: np.ndarray) -> np.ndarray:
        import torch
        t = torch.from_numpy(np.asarray(compact_idx, dtype=np.int64)).to(self.rows.device)
        return self.rows.index_select(0, t).cpu().numpy().astype(np.uint32)

    def expand_sums(self, a_compact) -> np.ndarray:
        """Running sums of all parent rows: every row takes its run start's."""
        import torch
        group = torch.cumsum(self.starts, 0, dtype=torch.int64) - 1
        return a_compact.index_select(0, group).cpu().numpy()


_SIDE_STREAMS = {}   # device -> the side stream of pdist_median (one per process)


def pdist_median(sub: np.ndarray, device=None) -> np.float64:
    """np.median(scipy.spatial.distance.pdist(sub)) with the distances computed and sorted on the
    GPU (st_pdist: bit-identical to scipy's) on a side stream, so it runs while a large upload is in
    flight on the current one; the middle value(s) come back and are averaged by np.mean exactly as
    np.median averages them.  ``sub``: (k, d) host rows, 2 <= k <= 65535."""
    import torch
    dev = device if device is not None else nat.require_device()
    sub = np.ascontiguousarray(sub, dtype=np.float64)
    k, d = sub.shape
    cnt = k * (k - 1) // 2
    side = _SIDE_STREAMS.get(dev)
    if side is None:
        side = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(side):
        rows = torch.from_numpy(sub).to(dev)
        dist = torch.empty(cnt, dtype=torch.float64, device=dev)
        nat.check(nat.lib().st_pdist(nat.ptr(rows), k, d, nat.ptr(dist), nat.stream_handle()), 'st_pdist')
        mid = torch.sort(dist).values[(cnt - 1) // 2:cnt // 2 + 1].cpu().numpy()
    return np.mean(mid)


def isotropic_scale(linv: np.ndarray):
    """(l, trace) if linv == l * I exactly, else None (dense preconditioners: not on the HIP path)."""
    linv = np.asarray(linv, dtype=np.float64)
    d = linv.shape[0]
    diag = np.diag(linv)
    off = linv - np.diag(diag)
    if np.any(off != 0) or np.any(diag != diag[0]):
        return None
    # np.trace(linv) exactly as the reference evaluates it (pairwise for d >= 8)
    return float(diag[0]), float(np.trace(linv))


class DeviceProblem:
    """Standardised (n, d) sample + score resident on the GPU in SoA layout."""

    def __init__(self, sample: np.ndarray, gradient: np.ndarray, weights: Optional[np.ndarray],
                 linv_scale: float, linv_trace: float, device=None):
        import torch
        self.device = device if device is not None else nat.require_device()
        sample = np.ascontiguousarray(sample, dtype=np.float64)
        gradient = np.ascontiguousarray(gradient, dtype=np.float64)
        self.n, self.d = sample.shape
        if self.d > 128:
            raise NotImplementedError(f'd = {self.d} > 128 is not supported by the HIP engine')
        self.ld = padded_ld(self.n)
        self.l = float(linv_scale)
        self.tr = float(linv_trace)
        self.x = self._soa(torch, sample)
        self.g = self._soa(torch, gradient)
        self.w = None
        if weights is not None:
            w = torch.zeros(self.ld, dtype=torch.float64, device=self.device)
            w[:self.n] = torch.from_numpy(np.ascontiguousarray(weights, dtype=np.float64)).to(self.device)
            self.w = w
        # asynchronous uploads (page-locked sources): an event after the layout kernels, so the owner
        # can make sure they finished before the arrays are used on another stream (wait_upload)
        self._upload_event = None
        if self._async:
            self._upload_event = torch.cuda.Event()
            self._upload_event.record()

    def wait_upload(self) -> None:
        """Block until an asynchronous upload has landed (no-op for synchronous ones)."""
        ev = getattr(self, '_upload_event', None)
        if ev is not None:
            ev.synchronize()
            self._upload_event = None
            self._raw = None

    def _soa(self, torch, rowmajor: np.ndarray):
        # page-locked host arrays (thinning._host_buffer) go up asynchronously on the current stream:
        # the caller keeps them alive (SteinIntegrand holds them) and the layout kernel is queued
        # behind the copy, so host work after this call (the 'med' preconditioner) overlaps the DMA
        src = torch.from_numpy(rowmajor)
        pinned = bool(src.is_pinned())
        self._async = getattr(self, '_async', False) or pinned
        rm = src.to(self.device, non_blocking=pinned)
        soa = torch.zeros((self.d, self.ld), dtype=torch.float64, device=self.device)
        nat.check(nat.lib().st_layout_soa(nat.ptr(rm), self.n, self.d, self.ld, nat.ptr(soa),
                                          nat.stream_handle()), 'st_layout_soa')
        return soa

    @classmethod
    def from_raw_device(cls, x_raw, g_raw, weights: Optional[np.ndarray], scl: np.ndarray,
                        linv_scale: float, linv_trace: float) -> 'DeviceProblem':
        """Problem from RAW row-major (n, d) device arrays (thinning._upload_standardized), laid out
        to SoA with the standardisation applied on the device: x / scl, g * scl (st_layout_soa_scaled).
        Everything is queued on the current stream without a host wait (small inputs go up from
        page-locked copies); the upload event marks the end, as for page-locked uploads."""
        import torch
        self = cls.__new__(cls)
        self.device = x_raw.device
        self.n, self.d = x_raw.shape
        self.ld = padded_ld(self.n)
        self.l, self.tr = float(linv_scale), float(linv_trace)

        def up(a):
            return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).pin_memory().to(
                self.device, non_blocking=True)
        sc = up(scl)
        L = nat.lib()
        self.x = torch.zeros((self.d, self.ld), dtype=torch.float64, device=self.device)
        self.g = torch.zeros((self.d, self.ld), dtype=torch.float64, device=self.device)
        for raw, soa, divide in ((x_raw, self.x, 1), (g_raw, self.g, 0)):
            nat.check(L.st_layout_soa_scaled(nat.ptr(raw), self.n, self.d, self.ld, nat.ptr(sc), divide,
                                             nat.ptr(soa), nat.stream_handle()), 'st_layout_soa_scaled')
        self.w = None
        if weights is not None:
            self.w = torch.zeros(self.ld, dtype=torch.float64, device=self.device)
            self.w[:self.n] = up(weights)
        self._raw = (x_raw, g_raw, sc)   # in use by the queued kernels until the upload event
        self._async = True
        self._upload_event = torch.cuda.Event()
        self._upload_event.record()
        return self

    @classmethod
    def from_soa(cls, x_soa, g_soa, w, n: int, linv_scale: float, linv_trace: float):
        """Wrap already-resident SoA tensors (d, ld) without copies (bench / sharded paths)."""
        self = cls.__new__(cls)
        self.device = x_soa.device
        self.d, self.ld = x_soa.shape
        self.n = int(n)
        self.l, self.tr = float(linv_scale), float(linv_trace)
        self.x, self.g, self.w = x_soa, g_soa, w
        return self

    # -- greedy ------------------------------------------------------------------------------
    def greedy_buffers(self, n_points: int):
        import torch
        ws_bytes = int(nat.lib().st_greedy_workspace_bytes(self.n, self.d, 1))
        ws = torch.empty((ws_bytes + 15) // 16 * 2, dtype=torch.float64, device=self.device)
        a = torch.empty(self.ld, dtype=torch.float64, device=self.device)
        idx = torch.empty(n_points, dtype=torch.int32, device=self.device)
        return idx, a, ws

    def greedy_launch(self, n_points: int, idx, a, ws) -> None:
        """Enqueue the whole greedy run on the current stream (no sync)."""
        nat.check(nat.lib().st_greedy(
            nat.ptr(self.x), nat.ptr(self.g), nat.ptr(self.w), self.n, self.d, self.ld,
            self.l, self.tr, int(n_points), nat.ptr(idx), nat.ptr(a), nat.ptr(ws),
            ws.numel() * 8, nat.stream_handle()), 'st_greedy')

    def greedy_steps_launch(self, n_points: int, idx, a, ws) -> None:
        """Enqueue the whole greedy run on the launch-per-step kernels (st_greedy_steps: no
        co-residency requirement, the same bits as the persistent kernel)."""
        nat.check(nat.lib().st_greedy_steps(
            nat.ptr(self.x), nat.ptr(self.g), nat.ptr(self.w), self.n, self.d, self.ld,
            self.l, self.tr, 0, int(n_points), int(n_points), nat.ptr(idx), nat.ptr(a), nat.ptr(ws),
            ws.numel() * 8, nat.stream_handle()), 'st_greedy_steps')

    def guard_mode(self, guard: bool = True) -> Optional[str]:
        """How ``greedy(guard=True)`` -- the drop-in thin's call -- keeps the reference's selection under
        the compact arithmetic (near-tie guard, on by default: nat.set_near_tie_guard / ST_NEAR_TIE): None
        when nothing is needed (``guard`` False, the exact arithmetic, d > 8, or the guard is off); 'kernel'
        for d = 2, 4 -- the persistent kernel flags a
        step whose argmin rests on sums closer than the arithmetic's error band (st_greedy_near_tie) and
        a flagged thin is re-run with the exact arithmetic; 'exact' for the other d <= 8, whose
        launch-per-step kernels carry no flag: the thin runs with the exact arithmetic."""
        if not guard or not nat.near_tie_guard() or self.d > 8 or nat.arithmetic() != 'compact':
            return None
        return 'kernel' if self.d in (2, 4) else 'exact'

    def greedy(self, n_points: int, return_sums: bool = False, margins: bool = False, dedup=False,
               guard: bool = False):
        """The reference's _greedy_search on the device.  ``self.fallback`` is None when the
        persistent launch completed, else why the run was repeated on the launch-per-step path
        (its bounded waits expired: the grid was not co-resident next to other work).
        ``margins=True``: (indices, diagnostics.GreedyMargins) -- the same selection with each step's
        argmin margin against the arithmetic's error band (launch-per-step kernels, one step at a time).
        ``dedup=True``: thin the run starts only (``dedup_view``) when repeated rows make that
        worthwhile (``dedup_pays``); ``dedup='always'``: whenever dedup_view has a view.  Either way the
        same indices and running sums bit for bit.  (The near-tie guard does not count a tie between rows
        equal bit for bit, so repeated rows -- adjacent or not -- never flag a step.)
        ``guard=True`` (the drop-in thin): the near-tie guard (``guard_mode``); the indices are then the
        reference NumPy path's even where the compact arithmetic alone would select another row, and
        the sums those of whichever arithmetic ran.  ``self.near_tie``: the guard's verdict -- None (no
        guard), -1 (no step flagged), t >= 0 (step t was flagged and the thin re-ran with the exact
        arithmetic), -2 (the run carried no flag: it re-ran with the exact arithmetic)."""
        if margins:
            from .diagnostics import greedy_margins
            gm = greedy_margins(self, n_points)
            return gm.indices, gm
        mode = self.guard_mode(guard)
        view = None
        if dedup == 'always' or (dedup and self.dedup_pays(n_points)):
            view = self.dedup_view()
            if view is not None and dedup != 'always' and not self.dedup_pays(n_points, view.n_unique):
                view = None
        self.dedup_used = view is not None
        if view is not None:
            out, a = view.problem._greedy_run(n_points, mode)
            self.fallback = view.problem.fallback
            self.near_tie = view.problem.near_tie
            out = view.to_rows(out)
            return (out, view.expand_sums(a)) if return_sums else out
        out, a = self._greedy_run(n_points, mode)
        return (out, a[:self.n].cpu().numpy()) if return_sums else out

    def _greedy_run(self, n_points: int, mode: Optional[str] = None):
        """(uint32 indices on the host, running sums on the device).  ``mode``: guard_mode()'s value --
        'exact' runs the exact arithmetic; 'kernel' reads the near-tie verdict of the compact run and
        re-runs a flagged (or unflagged-capable: fallback) thin with the exact arithmetic."""
        idx, a, ws = self.greedy_buffers(n_points)

        def run(exact: bool):
            with nat.arithmetic_override('exact') if exact else contextlib.nullcontext():
                self.greedy_launch(n_points, idx, a, ws)
                out = idx.cpu().numpy().view(np.uint32).copy()
                if out.size and int(out.max()) >= self.n:
                    self.fallback = ('persistent greedy kernel timed out (grid not co-resident?); '
                                     're-ran on the launch-per-step kernels')
                    warnings.warn(self.fallback, RuntimeWarning, stacklevel=4)
                    self.greedy_steps_launch(n_points, idx, a, ws)
                    out = idx.cpu().numpy().view(np.uint32).copy()
                    if out.size and int(out.max()) >= self.n:
                        raise nat.HipExtensionError('greedy step kernels returned out-of-range indices')
            return out

        self.fallback = None
        self.near_tie = None
        out = run(mode == 'exact')
        if mode == 'kernel':
            self.near_tie = nat.near_tie_step(ws)
            if self.near_tie != -1:   # flagged, or the run carried no flag (the step kernels' fallback)
                out = run(True)
        return out, a

    def dedup_view(self, any_repeat: bool = False) -> Optional['DedupView']:
        """The run starts of this problem as a compact problem, or None when fewer than
        ``1 - DEDUP_MAX_FRAC`` of the rows repeat their predecessor (``any_repeat``: when no row does);
        computed once, then cached.

        A row that repeats the row before it bit for bit (x, g and w: a rejected MCMC proposal;
        about 77 % of the rows of a random-walk chain at the usual acceptance rate) has every pair
        value, hence every running sum, equal to the run's first row, so it can only tie with that
        row and lose the tie to its lower index (np.argmin order): it is never selected.  Thinning
        the run starts and mapping the winners back gives the same indices, and the dropped rows'
        sums are their run start's."""
        import torch
        cached = getattr(self, '_dedup', False)
        if cached is False:   # run detection, once
            det = None
            if self.n > 1:
                L = nat.lib()
                starts = torch.empty(self.n, dtype=torch.uint8, device=self.device)
                ws = torch.empty((int(L.st_run_workspace_bytes(self.n)) + 7) // 8, dtype=torch.int64,
                                 device=self.device)
                nat.check(L.st_run_starts(nat.ptr(self.x), nat.ptr(self.g), nat.ptr(self.w), self.n, self.d,
                                          self.ld, nat.ptr(starts), nat.ptr(ws), ws.numel() * 8,
                                          nat.stream_handle()), 'st_run_starts')
                det = [starts, ws, int(ws[0].item()), None]   # count sizes the compact arrays; the view
            self._dedup = cached = det
        if cached is None:
            return None
        starts, ws, count, view = cached
        if count >= self.n or (not any_repeat and count > DEDUP_MAX_FRAC * self.n):
            return None
        if view is None:
            view = cached[3] = DedupView(self, starts, ws, count)
        return view

    def dedup_pays(self, n_points: int, n_unique: Optional[int] = None) -> bool:
        """Cost gate of ``greedy(dedup=True)`` (a heuristic: either answer gives the same indices).
        Before detection (n_unique None): is the whole thin's pair work worth a detection pass
        (>= 4 x DEDUP_MIN_SAVING_S)?  After: do the dropped rows save >= DEDUP_MIN_SAVING_S?  Per-pair
        costs measured on MI355X: ~1.8 ps per Langevin d = 4 pair on the
        persistent kernel above its per-step exchange floor, scaled by the flop count for d <= 8;
        the launch-per-step kernels of d > 8 stream (16 d + 24) B per pair at ~5 TB/s."""
        d = self.d
        if d <= 8:
            per_pair = 1.8e-12 * (12 * d + 40 + (2 if self.w is not None else 0)) / 88.0
        else:
            per_pair = (16 * d + 24) / 5e12
        if n_unique is None:
            return self.n * n_points * per_pair >= 4 * DEDUP_MIN_SAVING_S
        return (self.n - n_unique) * n_points * per_pair >= DEDUP_MIN_SAVING_S

    # -- integrand protocol --------------------------------------------------------------------
    def pairs(self, i1: np.ndarray, i2: np.ndarray) -> np.ndarray:
        import torch
        L = int(i1.shape[0])
        if L == 0:
            return np.empty(0, dtype=np.float64)
        t1 = torch.from_numpy(np.ascontiguousarray(i1, dtype=np.int64)).to(self.device)
        t2 = torch.from_numpy(np.ascontiguousarray(i2, dtype=np.int64)).to(self.device)
        return self.pairs_device(t1, t2)

    def pairs_device(self, t1, t2) -> np.ndarray:
        """k(row t1[q], row t2[q]) for index vectors already on the device (int64, rows < ld)."""
        import torch
        L = int(t1.shape[0])
        out = torch.empty(L, dtype=torch.float64, device=self.device)
        if L:
            nat.check(nat.lib().st_kernel_pairs(
                nat.ptr(self.x), nat.ptr(self.g), nat.ptr(self.w), self.ld, self.d, self.l, self.tr,
                nat.ptr(t1), nat.ptr(t2), L, nat.ptr(out), nat.stream_handle()), 'st_kernel_pairs')
        return out.cpu().numpy()

    def subset(self, rows: np.ndarray) -> 'DeviceProblem':
        """Compact problem of the given rows (gather on device; used by ksd / kmat)."""
        import torch
        if isinstance(rows, torch.Tensor):
            ti = rows.to(device=self.device, dtype=torch.int64).reshape(-1)
        else:
            ti = torch.from_numpy(np.asarray(rows, dtype=np.int64).reshape(-1)).to(self.device)
        m = int(ti.shape[0])
        ld = padded_ld(m)
        x = torch.zeros((self.d, ld), dtype=torch.float64, device=self.device)
        g = torch.zeros((self.d, ld), dtype=torch.float64, device=self.device)
        x[:, :m] = self.x.index_select(1, ti)
        g[:, :m] = self.g.index_select(1, ti)
        w = None
        if self.w is not None:
            w = torch.zeros(ld, dtype=torch.float64, device=self.device)
            w[:m] = self.w.index_select(0, ti)
        return DeviceProblem.from_soa(x, g, w, m, self.l, self.tr)

    def ksd(self, m: int) -> np.ndarray:
        """Cumulative KSD over rows 0..m-1 of this problem."""
        import torch
        if m == 0:
            return np.empty(0)
        ws_bytes = int(nat.lib().st_ksd_workspace_bytes(m, self.ld))
        ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.float64, device=self.device)
        ks = torch.empty(m, dtype=torch.float64, device=self.device)
        nat.check(nat.lib().st_ksd_cumulative(
            nat.ptr(self.x), nat.ptr(self.g), nat.ptr(self.w), m, self.ld, self.d, self.l, self.tr,
            nat.ptr(ks), nat.ptr(ws), ws.numel() * 8, nat.stream_handle()), 'st_ksd_cumulative')
        return ks.cpu().numpy()

    def kmat(self, k: int) -> np.ndarray:
        import torch
        if k == 0:
            return np.zeros((0, 0))
        out = torch.empty((k, k), dtype=torch.float64, device=self.device)
        nat.check(nat.lib().st_kmat(
            nat.ptr(self.x), nat.ptr(self.g), nat.ptr(self.w), k, self.ld, self.d, self.l, self.tr,
            nat.ptr(out), nat.stream_handle()), 'st_kmat')
        return out.cpu().numpy()


# thins in flight at once in greedy_concurrent: 8 chains of the reference's LV call shape (5e5 rows,
# m = 10 000, repeated rows dropped, run detection included) took 83 ms with 4 in flight (64-block
# grids) and 156 ms with 2, against 258-264 ms one after the other (profiles/r04_chains_probe.log)
IN_FLIGHT = 4
# problems per st_greedy_batch launch (at most 8): ONE launch runs them side by side on #CU / k
# blocks each, whatever hardware queues streams would map to
BATCH = 8


def _launch_batch(runs, n_points: int, bufs) -> bool:
    """st_greedy_batch over ``runs`` (same d, all weighted or none) on the current stream; False when
    the batch kernel does not apply to them (nothing enqueued)."""
    import ctypes
    L = nat.lib()
    k = len(runs)

    def arr(ctype, vals):
        return (ctype * k)(*vals)
    vp = ctypes.c_void_p
    weighted = runs[0].w is not None
    rc = L.st_greedy_batch(
        k, arr(vp, [p.x.data_ptr() for p in runs]), arr(vp, [p.g.data_ptr() for p in runs]),
        arr(vp, [p.w.data_ptr() for p in runs]) if weighted else None,
        arr(ctypes.c_int64, [p.n for p in runs]), runs[0].d, arr(ctypes.c_int64, [p.ld for p in runs]),
        arr(ctypes.c_double, [p.l for p in runs]), arr(ctypes.c_double, [p.tr for p in runs]), int(n_points),
        arr(vp, [b[0].data_ptr() for b in bufs]), arr(vp, [b[1].data_ptr() for b in bufs]),
        arr(vp, [b[2].data_ptr() for b in bufs]), arr(ctypes.c_int64, [b[2].numel() * 8 for b in bufs]),
        nat.stream_handle())
    if rc == nat.ST_ERR_UNSUPPORTED:
        return False
    nat.check(rc, 'st_greedy_batch')
    return True


def greedy_concurrent(problems, n_points: int, in_flight: Optional[int] = None, dedup=True,
                      batch: Optional[int] = None, guard: bool = False) -> list:
    """Independent greedy thins on ONE GPU at the same time (the reference thins every MCMC chain on
    its own: Stein_thinning.ipynb, fan-out code/src/utils/parallel.py:48-52).  Each problem's launch
    runs on one of ``in_flight`` streams with a grid of #CU / in_flight blocks (st_tune key 5, restored
    afterwards), so that many latency-bound thins share the chip instead of queueing behind each
    other.  First, groups of up to ``batch`` (default BATCH) problems of one d go to the device as
    ONE launch each (st_greedy_batch); a group of 4 or more that the batch kernel declines (its
    problems plan onto different kernels) is split into its smaller and larger half, each tried
    again; what is left uses the streams.
    Every result equals
    ``problem.greedy(n_points, dedup=dedup, guard=guard)``; a launch whose bounded waits expired anyway (another
    process's kernels held CUs) is re-run alone.  Returns one uint32 index array per problem."""
    import torch
    problems = list(problems)
    if not problems:
        return []
    L = nat.lib()
    k = len(problems)
    c = max(1, min(k, in_flight if in_flight is not None else IN_FLIGHT))
    if c == 1:   # one at a time, full grid (the guard as the plain thin has it: ADVICE r05)
        return [p.greedy(n_points, dedup=dedup, guard=guard) for p in problems]
    cus = torch.cuda.get_device_properties(problems[0].device).multi_processor_count
    views, modes = [], []
    for p in problems:
        v = None
        mode = p.guard_mode(guard)
        if dedup == 'always' or (dedup and p.dedup_pays(n_points)):
            v = p.dedup_view()
            if v is not None and dedup != 'always' and not p.dedup_pays(n_points, v.n_unique):
                v = None
        views.append(v)
        modes.append(mode)
    runs = [v.problem if v is not None else p for p, v in zip(problems, views)]
    cur = torch.cuda.current_stream()
    bufs, streams = [None] * k, [None] * k
    kb = max(1, min(8, batch if batch is not None else BATCH))
    def try_batch(part):
        if len(part) < 2:
            return
        b = [runs[i].greedy_buffers(n_points) for i in part]
        if _launch_batch([runs[i] for i in part], n_points, b):
            for i, bi in zip(part, b):
                bufs[i], streams[i] = bi, cur
        elif len(part) >= 4:   # declined (plans differ): the smaller and the larger half on their own
            by_n = sorted(part, key=lambda i: runs[i].n)
            try_batch(by_n[:len(by_n) // 2])
            try_batch(by_n[len(by_n) // 2:])
    if kb > 1:   # batch launches over groups of one d (and weights or none), in order; the batch kernel
        groups = {}   # runs the compact arithmetic, so the problems the guard runs exactly go to the streams
        for i, p in enumerate(runs):
            if modes[i] != 'exact':
                groups.setdefault((p.d, p.w is not None), []).append(i)
        for ids in groups.values():
            for j in range(0, len(ids), kb):
                try_batch(ids[j:j + kb])
    rest = [i for i in range(k) if bufs[i] is None]
    c = max(1, min(len(rest), c))
    # c streams, problem i on stream i % c: at most c grids of #CU / c blocks are ever resident
    # together, so every grid fits beside the others
    pool = [torch.cuda.Stream(device=runs[0].device) for _ in range(c)] if rest else []
    for s in pool:
        s.wait_stream(cur)   # the problems' arrays were written on the current stream
    if rest:
        # this thread's grid cap (st_tune key 23) and, for the problems the guard runs exactly (d outside
        # {2, 4}: kernels without a flag), this thread's arithmetic -- neither touches other threads' launches
        with nat.grid_cap(max(1, cus // c) if c > 1 else 0):
            for j, i in enumerate(rest):
                s = pool[j % c]
                with torch.cuda.stream(s), (nat.arithmetic_override('exact') if modes[i] == 'exact'
                                            else contextlib.nullcontext()):
                    b = runs[i].greedy_buffers(n_points)
                    runs[i].greedy_launch(n_points, *b)
                bufs[i], streams[i] = b, s
    out = []
    for p, v, b, s, mode in zip(runs, views, bufs, streams, modes):
        s.synchronize()
        idx = b[0].cpu().numpy().view(np.uint32).copy()
        p.fallback, p.near_tie = None, None
        if idx.size and int(idx.max()) >= p.n:   # not co-resident next to the others: alone now
            p.fallback = 'the concurrent launch timed out (grid not co-resident?); re-ran alone'
            idx, _ = p._greedy_run(n_points, mode)
        elif mode == 'kernel':
            with torch.cuda.stream(s):
                p.near_tie = nat.near_tie_step(b[2])
            if p.near_tie != -1:   # flagged: the exact arithmetic decides (p.near_tie keeps the step)
                tie = p.near_tie
                idx, _ = p._greedy_run(n_points, 'exact')
                p.near_tie = tie
        out.append(v.to_rows(idx) if v is not None else idx)
    return out
