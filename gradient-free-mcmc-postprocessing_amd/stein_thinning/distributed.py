"""Row-sharded greedy Stein thinning across GPUs (one process per GPU of one node, over xGMI).

The reference has no multi-device path (its only parallelism is joblib / Dask fan-out over chains,
``code/src/utils/parallel.py:18-52``).  Here the candidate axis n of one greedy run is split into
contiguous row blocks, one per rank; every rank picks the same winner per step (lowest value, then
lowest global index, NaN first: np.argmin over the concatenated array).  Three exchange engines
(``exchange_engine``; ``sharded_runner`` picks, validates and falls back):

* ``PersistentShardedGreedy`` (d = 2, 4): every rank holds the full standardised arrays
  (replicated, read-only) and runs ONE persistent launch over its row block; per step the ranks
  exchange their local winners {A_min, global index} through IPC-mapped device mailboxes (xGMI
  stores, no host round trip, no collective launch).  Handles are exchanged once with
  ``torch.distributed`` and the round trip is verified by a handshake before first use.
* device-exchange steps (other d): per step a fused kernel over the shard, ONE candidate record
  {value, global index, x row, g row, w} per rank, exchanged by a one-block mailbox kernel
  (st_greedy_step_exchange); the m-step loop is captured once into a HIP graph.
* ``GraphedShardedGreedy`` with RCCL (any d; fallback, or ST_SHARDED_EXCHANGE=rccl): the same
  records, RCCL ``all_gather_into_tensor`` per step, also graph-captured.

No n-length vector crosses xGMI in either; the design choice vs. an all-reduce of the n-length
column-sum vector is recorded in DESIGN.md (that all-reduce is used by the full-sample KSD).

Each rank passes the FULL host arrays: standardisation and the 'med' preconditioner are computed
from all rows exactly as the single-process reference does (bit-identical).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

from . import _native as nat
from .thinning import _make_stein_gf_integrand, _make_stein_integrand, SteinIntegrand


def shard_bounds(n: int, rank: int, world: int):
    """Contiguous row block [r0, r1) of rank (balanced, lower ranks take the remainder)."""
    base, rem = divmod(n, world)
    r0 = rank * base + min(rank, rem)
    return r0, r0 + base + (1 if rank < rem else 0)


class HipShardBackend:
    """Device state of one rank's shard + the C-ABI step/finalize launches.  With ``mailboxes``
    (a verified PeerMailboxes set) each step also exchanges the rank records device-side
    (st_greedy_step_exchange) and no collective is issued."""

    def __init__(self, integrand: SteinIntegrand, r0: int, r1: int, nranks: int, n_points: int,
                 mailboxes: Optional['PeerMailboxes'] = None, rank: int = 0):
        import torch
        from .device import DeviceProblem
        self.device = nat.require_device()
        w = None if integrand.weights is None else integrand.weights[r0:r1]
        self.prob = DeviceProblem(integrand.sample[r0:r1], integrand.gradient[r0:r1], w,
                                  integrand.linv_scale, integrand.linv_trace, self.device)
        self.r0, self.nranks, self.d = r0, nranks, self.prob.d
        self.stride = int(nat.lib().st_candidate_stride(self.d))
        ws_bytes = int(nat.lib().st_greedy_workspace_bytes(self.prob.n, self.d, nranks))
        self.ws = torch.empty((ws_bytes + 15) // 16 * 2, dtype=torch.float64, device=self.device)
        self.a = torch.empty(self.prob.ld, dtype=torch.float64, device=self.device)
        self.idx = torch.zeros(n_points, dtype=torch.int32, device=self.device)
        self.send = torch.zeros(self.stride, dtype=torch.float64, device=self.device)
        self.recv = torch.zeros(self.stride * nranks, dtype=torch.float64, device=self.device)
        self.mb, self.rank = mailboxes, int(rank)
        self.device_exchange = mailboxes is not None
        self.status = torch.zeros(1, dtype=torch.int32, device=self.device)

    def step(self, t: int) -> None:
        p = self.prob
        if self.device_exchange:
            nat.check(nat.lib().st_greedy_step_exchange(
                nat.ptr(p.x), nat.ptr(p.g), nat.ptr(p.w), p.n, p.d, p.ld, p.l, p.tr, self.r0, t,
                self.rank, self.nranks, self.mb.table_ptr(), nat.ptr(self.recv), nat.ptr(self.idx),
                nat.ptr(self.a), nat.ptr(self.ws), self.ws.numel() * 8, nat.ptr(self.status),
                nat.stream_handle()), 'st_greedy_step_exchange')
            return
        nat.check(nat.lib().st_greedy_step(
            nat.ptr(p.x), nat.ptr(p.g), nat.ptr(p.w), p.n, p.d, p.ld, p.l, p.tr, self.r0, t,
            self.nranks, nat.ptr(self.recv), nat.ptr(self.send), nat.ptr(self.idx),
            nat.ptr(self.a), nat.ptr(self.ws), self.ws.numel() * 8, nat.stream_handle()),
            'st_greedy_step')

    def finalize(self, t: int) -> None:
        nat.check(nat.lib().st_greedy_finalize(nat.ptr(self.recv), self.nranks, self.d,
                                               nat.ptr(self.idx), t, nat.stream_handle()),
                  'st_greedy_finalize')

    def indices(self) -> np.ndarray:
        return self.idx.cpu().numpy().view(np.uint32).copy()

    def exchange_ok(self) -> bool:
        """No bounded wait of the device exchange expired (always True on the RCCL path)."""
        return int(self.status.item()) == 0


def _all_gather(recv, send, group=None) -> None:
    """recv <- concat over ranks of send.  RCCL (nccl backend): one all_gather_into_tensor on the
    device buffers.  gloo (CPU test rig): through host copies."""
    import torch
    import torch.distributed as dist
    if send.is_cuda and dist.get_backend(group) != 'nccl':
        parts = [torch.empty(send.shape, dtype=send.dtype) for _ in range(dist.get_world_size(group))]
        dist.all_gather(parts, send.cpu(), group=group)
        recv.copy_(torch.cat(parts))
    else:
        dist.all_gather_into_tensor(recv, send, group=group)


def _sharded_loop(backend, n_points: int, group=None) -> None:
    import torch.distributed as dist
    exchanged = getattr(backend, 'device_exchange', False)   # the step call exchanged already
    collective = dist.is_available() and dist.is_initialized()
    for t in range(n_points):
        backend.step(t)
        if exchanged:
            continue
        if collective:
            _all_gather(backend.recv, backend.send, group)
        else:
            backend.recv.copy_(backend.send)
    backend.finalize(n_points - 1)


def run_sharded(backend, n_points: int, group=None) -> np.ndarray:
    """Drive the per-step kernel / all-gather sequence.  ``backend`` exposes step(t), finalize(t),
    send, recv, nranks and indices(); the product backend is HipShardBackend, tests substitute a
    CPU backend with the same record format (gloo)."""
    _sharded_loop(backend, n_points, group)
    return backend.indices()


class GraphedShardedGreedy:
    """The m-step sharded loop (step kernel, publish kernel, RCCL all-gather per step) captured
    once into a HIP graph and replayed: removes the per-step host launch cost (~30 us of Python +
    ctypes + collective enqueue) that otherwise dominates the ~5 us of GPU work per step at 8 ranks.
    Falls back to eager launches if capture is not possible (reported in ``self.mode``)."""

    def __init__(self, backend: 'HipShardBackend', n_points: int, group=None, use_graph: bool = True):
        self.backend, self.n_points, self.group = backend, int(n_points), group
        self.graph = None
        self.mode = 'eager'
        if use_graph:
            try:
                self._capture()
                self.mode = 'graph'
            except Exception as e:   # capture unsupported here: keep eager launches
                self.graph = None
                self.mode = f'eager (graph capture failed: {type(e).__name__}: {e})'

    def _capture(self):
        import torch
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            _sharded_loop(self.backend, self.n_points, self.group)    # warm-up outside capture
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        eager_idx = self.backend.indices()
        g = torch.cuda.CUDAGraph()
        # thread_local: the process group's watchdog thread keeps querying events of earlier
        # collectives while this thread captures; global mode would turn those queries into
        # hipErrorStreamCaptureUnsupported
        with torch.cuda.graph(g, capture_error_mode='thread_local'):
            _sharded_loop(self.backend, self.n_points, self.group)
        self.graph = g
        g.replay()
        torch.cuda.synchronize()
        if not np.array_equal(self.backend.indices(), eager_idx):
            raise RuntimeError('graph replay disagrees with eager launches')

    def launch(self) -> None:
        """Enqueue one whole greedy run (no sync)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            _sharded_loop(self.backend, self.n_points, self.group)

    def indices(self) -> np.ndarray:
        return self.backend.indices()

    def run(self) -> np.ndarray:
        self.launch()
        return self.backend.indices()


MAX_PEER_RANKS = 8   # mailbox table size (include/stein_thinning_hip.h: one node)


class PeerMailboxes:
    """This rank's device mailbox plus its peers' mailboxes mapped into this process (IPC).

    Created collectively by every rank of ``group``; ``ok`` is the group-wide verdict (IPC setup
    and a device-side handshake succeeded on EVERY rank).  ``seq`` is the exchange sequence
    number the next persistent run starts at (identical on every rank: all ranks run the same
    sequence of collective thins)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.device = nat.require_device()
        self.seq = 0
        self.token = 0
        self.local = ctypes.c_void_p()
        self.opened = []
        self.table = (ctypes.c_void_p * MAX_PEER_RANKS)()
        L = nat.lib()
        err = ''
        handle = b''
        try:
            if self.world > MAX_PEER_RANKS:
                raise ValueError(f'{self.world} ranks > {MAX_PEER_RANKS}')
            nat.check(L.st_mailbox_alloc(L.st_mailbox_bytes(self.world), ctypes.byref(self.local)),
                      'st_mailbox_alloc')
            hb = L.st_ipc_handle_bytes()
            h = (ctypes.c_ubyte * hb)()
            nat.check(L.st_ipc_get_handle(self.local, h), 'st_ipc_get_handle')
            handle = bytes(h)
        except Exception as e:   # noqa: BLE001 -- reported through the group verdict
            err = f'{type(e).__name__}: {e}'
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        if not err and all(handles):
            try:
                for r in range(self.world):
                    if r == self.rank:
                        self.table[r] = self.local.value
                        continue
                    p = ctypes.c_void_p()
                    hr = (ctypes.c_ubyte * len(handles[r])).from_buffer_copy(handles[r])
                    nat.check(L.st_ipc_open_handle(hr, ctypes.byref(p)), f'st_ipc_open_handle(rank {r})')
                    self.opened.append(p)
                    self.table[r] = p.value
            except Exception as e:   # noqa: BLE001
                err = f'{type(e).__name__}: {e}'
        elif not err:
            err = 'a peer failed to export its mailbox'
        self.error = err
        self.ok = self._agree(not err) and self.handshake()

    def _agree(self, flag: bool) -> bool:
        """Group-wide AND of a per-rank flag."""
        return _group_all(flag, self.group)

    def handshake(self) -> bool:
        """Every rank stores a token into every peer's mailbox and polls its own (device side,
        bounded wait); True iff all ranks saw all tokens."""
        import torch
        self.token += 1
        ok = torch.zeros(1, dtype=torch.int32, device=self.device)
        good = False
        try:
            nat.check(nat.lib().st_mailbox_handshake(ctypes.cast(self.table, ctypes.c_void_p), self.world,
                                                     self.rank, self.token, nat.ptr(ok),
                                                     nat.stream_handle()), 'st_mailbox_handshake')
            torch.cuda.synchronize()
            good = int(ok.item()) == 1
            if not good:
                self.error = 'mailbox handshake timed out'
        except Exception as e:   # noqa: BLE001
            self.error = f'{type(e).__name__}: {e}'
        return self._agree(good)

    def table_ptr(self):
        return ctypes.cast(self.table, ctypes.c_void_p)

    def close(self) -> None:
        L = nat.lib()
        for p in self.opened:
            L.st_ipc_close_handle(p)
        self.opened = []
        if self.local.value:
            L.st_mailbox_free(self.local)
            self.local = ctypes.c_void_p()
        self.ok = False


def _group_all(flag: bool, group=None) -> bool:
    """Group-wide AND of a per-rank flag (RCCL on the device under nccl, host tensor under gloo)."""
    import torch
    import torch.distributed as dist
    dev = nat.require_device() if dist.get_backend(group) == 'nccl' else torch.device('cpu')
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _group_same(idx: np.ndarray, group=None) -> bool:
    """True iff every rank holds the same index vector (min and max of a 63-bit digest agree)."""
    import hashlib

    import torch
    import torch.distributed as dist
    h = int.from_bytes(hashlib.sha256(np.ascontiguousarray(idx).tobytes()).digest()[:8], 'little') >> 1
    dev = nat.require_device() if dist.get_backend(group) == 'nccl' else torch.device('cpu')
    lo = torch.tensor([h], dtype=torch.int64, device=dev)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    return int(lo.item()) == int(hi.item())


_MAILBOXES = {}


def peer_mailboxes(group=None) -> PeerMailboxes:
    """The process-wide mailbox set of ``group`` (collective on first use)."""
    import torch.distributed as dist
    key = (id(group), dist.get_world_size(group), dist.get_rank(group))
    mb = _MAILBOXES.get(key)
    if mb is None:
        mb = _MAILBOXES[key] = PeerMailboxes(group)
    return mb


WIDE_PERSISTENT_D = 50   # persistent kernel's wide instantiation (csrc/persistent.hip kWideD)


def _wide_fits(n: int, world: int) -> bool:
    """Every rank's shard fits the wide persistent kernel: at most 256 rows per CU (one register
    row per thread of one 256-thread block per CU)."""
    import torch
    cus = torch.cuda.get_device_properties(nat.require_device()).multi_processor_count
    return -(-n // world) <= 256 * cus


def exchange_engine(d: int, world: int, n: Optional[int] = None) -> str:
    """Engine of a ``world``-rank run at dimension d: 'persistent' (d = 2, 4: one persistent launch
    per rank, winners exchanged in-kernel), 'steps' (other d: launch-per-step kernels in a HIP graph,
    records exchanged by a mailbox kernel; also d = 50 -- the wide persistent kernel -- when a rank's
    shard exceeds 256 rows per CU), 'replicated' (d = 2, 4, ST_SHARDED_EXCHANGE=replicated:
    every GPU thins the whole sample; also the d = 2, 4 fallback) or 'rccl' (RCCL all-gather per
    step; forced by ST_SHARDED_EXCHANGE=rccl, and the fallback otherwise)."""
    choice = os.environ.get('ST_SHARDED_EXCHANGE', 'device')
    if choice == 'replicated' and d in (2, 4):
        return 'replicated'
    if not 2 <= world <= MAX_PEER_RANKS or choice == 'rccl':
        return 'rccl'
    if d in (2, 4) or (d == WIDE_PERSISTENT_D and n is not None and _wide_fits(n, world)):
        return 'persistent'
    return 'steps'


def persistent_supported(integrand: SteinIntegrand, rank: int, world: int, n_points: int,
                         group=None) -> bool:
    """Group-wide verdict of the C launcher's own eligibility check (st_greedy_sharded_supported:
    d, rows per block against the kernel's register / LDS budget, the grid cap) for every rank's
    block -- exchange_engine's choice is a cheap pre-filter, this is the launcher's decision."""
    r0, r1 = shard_bounds(integrand.n, rank, world)
    rc = nat.lib().st_greedy_sharded_supported(integrand.n, integrand.sample.shape[1],
                                               0 if integrand.weights is None else 1, r0, r1, rank, world,
                                               int(n_points))
    return _group_all(rc == 1, group)


def device_exchange_eligible(d: int, world: int) -> bool:
    """Whether a mailbox (device-side) exchange engine serves this run."""
    return exchange_engine(d, world) != 'rccl'


class PersistentShardedGreedy:
    """One rank of a multi-GPU greedy run on the persistent kernel with device-side exchange
    (C-ABI ``st_greedy_sharded``).  The full standardised problem is resident on every rank; this
    rank sweeps rows [r0, r1)."""

    mode = 'device-exchange'

    def __init__(self, integrand: SteinIntegrand, rank: int, world: int, n_points: int,
                 mailboxes: PeerMailboxes, problem=None):
        from .device import DeviceProblem
        self.device = nat.require_device()
        self.prob = problem if problem is not None else DeviceProblem(
            integrand.sample, integrand.gradient, integrand.weights, integrand.linv_scale,
            integrand.linv_trace, self.device)
        self.rank, self.world, self.n_points = rank, world, int(n_points)
        self.r0, self.r1 = shard_bounds(self.prob.n, rank, world)
        self.mb = mailboxes
        self.idx, self.a, self.ws = self.prob.greedy_buffers(self.n_points)

    def launch(self) -> None:
        """Enqueue one whole greedy run on the current stream (collective: every rank calls it)."""
        p = self.prob
        seq = self.mb.seq
        self.mb.seq += self.n_points
        nat.check(nat.lib().st_greedy_sharded(
            nat.ptr(p.x), nat.ptr(p.g), nat.ptr(p.w), p.n, p.d, p.ld, p.l, p.tr, self.r0, self.r1,
            self.rank, self.world, self.mb.table_ptr(), seq, self.n_points, nat.ptr(self.idx),
            nat.ptr(self.a), nat.ptr(self.ws), self.ws.numel() * 8, nat.stream_handle()),
            'st_greedy_sharded')

    def indices(self) -> np.ndarray:
        return self.idx.cpu().numpy().view(np.uint32).copy()

    def completed(self, idx: Optional[np.ndarray] = None) -> bool:
        idx = self.indices() if idx is None else idx
        return bool(idx.size == 0 or int(idx.max()) < self.prob.n)

    def near_tie_step(self) -> int:
        """This rank's near-tie word of the last run (st_greedy_near_tie: its own rows against the global
        winner): the first flagged step, -1 none, -2 the run carried no flag."""
        return nat.near_tie_step(self.ws)

    def run(self) -> np.ndarray:
        self.launch()
        return self.indices()


class ReplicatedGreedy:
    """Every rank runs the WHOLE greedy thin on its own GPU (the single-device persistent kernel
    over the replicated arrays): no exchange, and identical indices on every rank (same inputs,
    same deterministic kernel; checked on the first run).  The fallback for d = 2, 4 when the
    device exchange cannot be used: one GPU's time per thin, against ~25 us per step for an RCCL
    all-gather of per-step records at these sizes."""

    mode = 'replicated'

    def __init__(self, integrand: SteinIntegrand, n_points: int, problem=None):
        from .device import DeviceProblem
        self.device = nat.require_device()
        self.prob = problem if problem is not None else DeviceProblem(
            integrand.sample, integrand.gradient, integrand.weights, integrand.linv_scale,
            integrand.linv_trace, self.device)
        self.n_points = int(n_points)
        self.idx, self.a, self.ws = self.prob.greedy_buffers(self.n_points)

    def launch(self) -> None:
        self.prob.greedy_launch(self.n_points, self.idx, self.a, self.ws)

    def indices(self) -> np.ndarray:
        return self.idx.cpu().numpy().view(np.uint32).copy()

    def completed(self, idx: Optional[np.ndarray] = None) -> bool:
        idx = self.indices() if idx is None else idx
        return bool(idx.size == 0 or int(idx.max()) < self.prob.n)

    def near_tie_step(self) -> int:
        """The single-device kernel's near-tie word of the last run (all rows): see PersistentShardedGreedy."""
        return nat.near_tie_step(self.ws)

    def run(self) -> np.ndarray:
        self.launch()
        return self.indices()


_NO_TIE = 1 << 62


def combine_near_tie(step: int, group=None) -> int:
    """Collective: the near-tie verdict of a sharded run from every rank's own word (one all-reduce MIN per
    thin, none per step).  Each rank's kernel checks its own rows -- everything but the winner and its
    bitwise duplicates -- against the global winner and the same threshold (bounds over all n rows), so
    the union of the ranks' flags is the single-device rule (oracle/stein_ref.c sr_greedy_mt_ties).
    ``step``: this rank's first flagged step, -1 none, -2 no flag computed.  Returns the first flagged step
    over all ranks, -1 none, -2 if some rank computed no flag (its run must be re-run exactly)."""
    import torch
    import torch.distributed as dist
    v = _NO_TIE if step == -1 else (-1 if step < -1 else int(step))
    if _world(group)[1] > 1:
        dev = nat.require_device() if dist.get_backend(group) == 'nccl' else torch.device('cpu')
        t = torch.tensor([v], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        v = int(t.item())
    return -1 if v == _NO_TIE else (-2 if v < 0 else v)


# --------------------------------------------------------------------------------------------
# Full-sample KSD, row-sharded: every rank sums k(i, a) over its rows a < i for all columns i,
# the n-length column-sum vector is all-reduced (RCCL), every rank finishes the prefix scan.
# --------------------------------------------------------------------------------------------
def triangle_row_bounds(n: int, rank: int, world: int):
    """Row block [a0, a1) of rank such that the strictly-lower-triangle pair counts
    sum_{a in [a0, a1)} (n - 1 - a) are balanced across ranks."""
    total = n * (n - 1) // 2

    def first_row(target):   # smallest a0 with pairs(rows < a0) >= target
        if target <= 0:
            return 0
        # pairs(rows < a) = a (n - 1) - a (a - 1) / 2, increasing in a on [0, n]
        lo, hi = 0, n
        while lo < hi:
            mid = (lo + hi) // 2
            if mid * (n - 1) - mid * (mid - 1) // 2 >= target:
                hi = mid
            else:
                lo = mid + 1
        return lo
    a0 = first_row(total * rank // world) if rank > 0 else 0
    a1 = first_row(total * (rank + 1) // world) if rank + 1 < world else n
    return a0, a1


class HipKsdBackend:
    """Device side of the sharded KSD: the full problem resident on this rank's GPU."""

    def __init__(self, integrand: SteinIntegrand, n: int):
        import torch
        self.prob = integrand.device_problem()
        self.n = int(n)
        if not 0 <= self.n <= self.prob.n:
            raise ValueError(f'n = {n} outside [0, {self.prob.n}]')
        self.csum = torch.zeros(max(self.prob.ld, 1), dtype=torch.float64, device=self.prob.device)

    def colsum(self, a0: int, a1: int):
        p = self.prob
        nat.check(nat.lib().st_ksd_colsum(nat.ptr(p.x), nat.ptr(p.g), nat.ptr(p.w), self.n, p.ld, p.d,
                                          p.l, p.tr, a0, a1, nat.ptr(self.csum), nat.stream_handle()),
                  'st_ksd_colsum')
        return self.csum[:self.n]

    def finish(self, csum) -> np.ndarray:
        import torch
        p = self.prob
        ks = torch.empty(self.n, dtype=torch.float64, device=p.device)
        nat.check(nat.lib().st_ksd_finish(nat.ptr(p.x), nat.ptr(p.g), nat.ptr(p.w), self.n, p.ld, p.d,
                                          p.l, p.tr, nat.ptr(csum), nat.ptr(ks), nat.stream_handle()),
                  'st_ksd_finish')
        return ks.cpu().numpy()


def _all_reduce_sum(t, group=None) -> None:
    """In-place sum over ranks: RCCL on the device buffer (nccl), host round trip under gloo."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(group) != 'nccl':
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)


def run_ksd_sharded(backend, n: int, group=None) -> np.ndarray:
    """Drive colsum over this rank's triangle rows -> all-reduce of the n-vector -> finish.
    ``backend`` exposes colsum(a0, a1) -> tensor and finish(tensor) -> ndarray (HipKsdBackend;
    tests substitute a CPU backend)."""
    rank, world = _world(group)
    if n == 0:
        return np.empty(0)
    a0, a1 = triangle_row_bounds(n, rank, world)
    c = backend.colsum(a0, a1)
    if world > 1:
        _all_reduce_sum(c, group)
    return backend.finish(c)


def ksd_sharded(integrand: SteinIntegrand, n: int, group=None) -> np.ndarray:
    """Cumulative KSD of rows 0..n-1 of ``integrand`` (stein_thinning.stein.ksd semantics) with
    the O(n^2) pair work split over the ranks of ``group``."""
    return run_ksd_sharded(HipKsdBackend(integrand, n), int(n), group)


def _world(group):
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def thin_sharded(sample, gradient, n_points: int, standardize: bool = True, preconditioner='id',
                 group=None) -> np.ndarray:
    """``thin`` with the candidate rows sharded over the ranks of ``group`` (identical result)."""
    integrand = _make_stein_integrand(sample, gradient, standardize, preconditioner)
    return _thin_sharded_integrand(integrand, n_points, group)


def thin_gf_sharded(sample, log_p, log_q, gradient_q, n_points: int, standardize: bool = True,
                    range_cap: Optional[float] = None, preconditioner='id', group=None) -> np.ndarray:
    integrand = _make_stein_gf_integrand(sample, log_p, log_q, gradient_q, standardize, range_cap,
                                         preconditioner)
    return _thin_sharded_integrand(integrand, n_points, group)


class _EagerRecords:
    """Records all-gathered per step from Python (gloo process group with device buffers: tests)."""

    mode = 'records-all-gather'

    def __init__(self, backend: HipShardBackend, n_points: int, group=None):
        self.backend, self.n_points, self.group = backend, n_points, group
        self.launch()

    def launch(self) -> None:
        _sharded_loop(self.backend, self.n_points, self.group)

    def indices(self) -> np.ndarray:
        return self.backend.indices()

    def run(self) -> np.ndarray:
        self.launch()
        return self.indices()


def sharded_runner(integrand: SteinIntegrand, n_points: int, group=None, use_graph: bool = True):
    """Collective: build this rank's runner for a row-sharded greedy run and complete one run with
    it (the validation run; its result is ``runner.indices()``).  Tries the device-exchange engine
    (exchange_engine) first; if the mailboxes cannot be set up or any rank's bounded wait expired,
    every rank falls back together: for d = 2, 4 to the replicated run (each GPU thins the whole
    sample; indices compared across ranks), otherwise -- or if that disagrees -- to the RCCL
    record all-gather.  ``runner.mode`` names the engine; ``runner.launch()`` enqueues a further
    run."""
    rank, world = _world(group)
    if world > 1 and not _group_same(np.array([nat.ARITHMETIC[nat.arithmetic()]], dtype=np.int64), group):
        raise ValueError('sharded thin: the ranks use different greedy-kernel arithmetics '
                         '(stein_thinning.set_arithmetic / ST_ARITH must agree on every rank)')
    engine = exchange_engine(integrand.sample.shape[1], world, integrand.n)
    if engine == 'persistent' and not persistent_supported(integrand, rank, world, n_points, group):
        engine = 'steps'   # e.g. d = 50 with more rows per block than the wide kernel holds
    runner = _engine_runner(integrand, n_points, group, use_graph, engine)
    runner.engine = engine   # the engine chosen; runner.mode names the one that ran
    return runner


def _engine_runner(integrand: SteinIntegrand, n_points: int, group, use_graph: bool, engine: str):
    import torch.distributed as dist
    rank, world = _world(group)
    d = integrand.sample.shape[1]
    note = ''
    if engine == 'replicated':
        runner = ReplicatedGreedy(integrand, n_points)
        runner.launch()
        idx = runner.indices()
        if _group_all(runner.completed(idx), group) and _group_same(idx, group):
            return runner
        note = 'replicated runs disagree; '
    elif engine != 'rccl':
        mb = peer_mailboxes(group)
        if mb.ok:
            if engine == 'persistent':
                runner = PersistentShardedGreedy(integrand, rank, world, n_points, mb)
                runner.launch()
                ok = runner.completed()
            else:
                r0, r1 = shard_bounds(integrand.n, rank, world)
                backend = HipShardBackend(integrand, r0, r1, world, n_points, mailboxes=mb, rank=rank)
                runner = GraphedShardedGreedy(backend, n_points, group, use_graph)
                runner.mode = 'device-exchange-steps-' + runner.mode
                ok = backend.exchange_ok()
            if mb._agree(ok):
                return runner
            mb.ok = False   # a bounded wait expired somewhere: no device exchange from now on
            mb.error = f'{engine} device exchange timed out'
            note = 'device exchange timed out; '
        else:
            note = f'device exchange unavailable ({mb.error}); '
        if engine == 'persistent' and d in (2, 4):
            runner = ReplicatedGreedy(integrand, n_points)
            runner.launch()
            idx = runner.indices()
            if _group_all(runner.completed(idx), group) and _group_same(idx, group):
                runner.mode = note + 'replicated'
                return runner
            note += 'replicated runs disagree; '
    r0, r1 = shard_bounds(integrand.n, rank, world)
    backend = HipShardBackend(integrand, r0, r1, world, n_points)
    if dist.is_initialized() and dist.get_backend(group) == 'nccl':
        runner = GraphedShardedGreedy(backend, n_points, group, use_graph)
        runner.mode = note + 'rccl-' + runner.mode
        return runner
    runner = _EagerRecords(backend, n_points, group)
    runner.mode = note + runner.mode
    return runner


def _problem_digest(integrand: SteinIntegrand, n_points: int) -> np.ndarray:
    """Cheap fingerprint of a thinning problem: shape, m, preconditioner, the greedy kernels'
    arithmetic (a rank that set another one would evaluate its shard by other rules) and 4 096 evenly
    spaced standardised rows (+ weights).  Ranks running independent thins (different chains) differ."""
    n = integrand.n
    rows = np.linspace(0, n - 1, min(n, 4096)).astype(np.int64)
    parts = [np.array([n, integrand.sample.shape[1], n_points, integrand.weights is not None,
                       nat.ARITHMETIC[nat.arithmetic()]], dtype=np.int64),
             np.array([integrand.linv_scale, integrand.linv_trace]),
             integrand.sample[rows], integrand.gradient[rows]]
    if integrand.weights is not None:
        parts.append(integrand.weights[rows])
    return np.concatenate([np.ascontiguousarray(p).view(np.uint8).reshape(-1) for p in parts])


def thin_across_ranks(integrand: SteinIntegrand, n_points: int, group=None) -> np.ndarray:
    """The drop-in ``thin`` / ``thin_gf`` under a multi-rank launch that opted in to sharding
    (``thinning._greedy_search`` routes here when torch.distributed is initialised with world > 1 and
    set_rank_sharding(True) / ST_SHARD_THIN=1): the candidate rows are sharded over the ranks exactly
    as ``thin_sharded`` does, and every rank returns the single-process indices.  Collective: every
    rank must call it with the same problem -- checked first; ranks thinning different samples (the
    reference's per-chain fan-out, ``code/src/utils/parallel.py:48-52``) get a ValueError and should
    leave sharding off."""
    if not _group_same(_problem_digest(integrand, n_points), group):
        raise ValueError('thin() under torch.distributed: the ranks hold different problems; '
                         'leave row sharding off (ST_SHARD_THIN unset / set_rank_sharding(False)) '
                         'to thin independently on every rank')
    return _thin_sharded_integrand(integrand, n_points, group)


def _thin_sharded_integrand(integrand: SteinIntegrand, n_points: int, group=None,
                            use_graph: bool = True) -> np.ndarray:
    n_points = int(n_points)
    if n_points < 1:
        raise ValueError('n_points must be >= 1')
    rank, world = _world(group)
    if world > integrand.n:
        raise ValueError(f'{world} ranks for {integrand.n} rows: every rank needs at least one row')
    from .thinning import _dedup
    view = integrand.run_starts_view() if _dedup() else None
    rows = None
    if view is not None and view[0].n >= world:
        integrand, rows = view   # the run starts only (thinning.set_dedup; same indices)
    if world > 1 and not _group_same(np.array([-1 if rows is None else rows.size], dtype=np.int64), group):
        raise ValueError('sharded thin: the ranks disagree on the repeated-row path '
                         '(stein_thinning.set_dedup / ST_DEDUP must agree, and so must the sample)')
    global last_mode, last_rows_kept, last_near_tie
    last_rows_kept = None if rows is None else int(rows.size)
    runner, last_near_tie = guarded_sharded_run(integrand, n_points, group, use_graph)
    last_mode = runner.mode
    idx = runner.indices()
    return idx if rows is None else rows[idx.astype(np.int64)].astype(np.uint32)


def sharded_guard_mode(d: int, world: int) -> Optional[str]:
    """The near-tie guard of a sharded thin (the single-device rule, DeviceProblem.guard_mode): None when
    nothing is needed (guard off -- nat.set_near_tie_guard / ST_NEAR_TIE=0 --, the exact arithmetic, or
    d > 8); 'kernel' for d = 2, 4 on the engines whose kernels flag (persistent device exchange,
    replicated); 'exact' for the step engines (other d, or ST_SHARDED_EXCHANGE=rccl): their kernels carry
    no flag, so the thin runs the exact arithmetic -- NumPy's evaluation order -- directly."""
    if not nat.near_tie_guard() or nat.arithmetic() != 'compact' or d > 8:
        return None
    return 'kernel' if exchange_engine(d, world) in ('persistent', 'replicated') else 'exact'


def guarded_sharded_run(integrand: SteinIntegrand, n_points: int, group=None, use_graph: bool = True):
    """Collective: sharded_runner plus the near-tie guard (sharded_guard_mode).  'kernel': after the compact
    run every rank reads its own word and one all-reduce combines them (combine_near_tie); a flagged run, or
    one whose engine fell back to kernels without a flag, is run again -- on every rank -- with the exact
    arithmetic.  Returns (runner, verdict): the verdict is None (no guard), -1 (no step flagged), t >= 0
    (step t flagged: re-ran exactly) or -2 (ran exactly: no flag available)."""
    rank, world = _world(group)
    mode = sharded_guard_mode(integrand.sample.shape[1], world)
    if mode == 'exact':
        with nat.arithmetic_override('exact'):
            return sharded_runner(integrand, n_points, group, use_graph), -2
    runner = sharded_runner(integrand, n_points, group, use_graph)
    if mode is None:
        return runner, None
    own = runner.near_tie_step() if hasattr(runner, 'near_tie_step') else -2
    verdict = combine_near_tie(own, group)
    if verdict == -1:
        return runner, -1
    with nat.arithmetic_override('exact'):   # every rank: the verdict is the same on all of them
        return sharded_runner(integrand, n_points, group, use_graph), verdict


last_mode = None   # exchange engine of the last sharded thin in this process (tests / bench)
last_rows_kept = None   # rows the last sharded thin kept after dropping repeats (None: all)
last_near_tie = None   # the near-tie verdict of the last sharded thin (guarded_sharded_run)
