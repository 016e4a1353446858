"""Row-sharded greedy Stein thinning across GPUs (one process per GPU, RCCL over xGMI).

The reference has no multi-device path (its only parallelism is joblib / Dask fan-out over chains,
``code/src/utils/parallel.py:18-52``).  Here the candidate axis n of one greedy run is split into
contiguous row blocks, one per rank.  Per step every rank streams its shard (fused kernel), reduces
it to ONE candidate record {value, global index, x row, g row, w} and the ranks all-gather those
records (``8 * stride`` bytes per rank; RCCL ``all_gather_into_tensor``).  Every rank then picks the
same winner (lowest value, then lowest global index, NaN first: np.argmin over the concatenated
array) at the start of its next kernel.  No n-length vector ever crosses xGMI; the design choice
vs. an all-reduce of the n-length column-sum vector is recorded in DESIGN.md.

Each rank passes the FULL host arrays: standardisation and the 'med' preconditioner are computed
from all rows exactly as the single-process reference does (bit-identical), then only the rank's
shard is uploaded.
"""
from __future__ import annotations

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
    """Device state of one rank's shard + the C-ABI step/finalize launches."""

    def __init__(self, integrand: SteinIntegrand, r0: int, r1: int, nranks: int, n_points: int):
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

    def step(self, t: int) -> None:
        p = self.prob
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
    collective = dist.is_available() and dist.is_initialized()
    for t in range(n_points):
        backend.step(t)
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

    def run(self) -> np.ndarray:
        self.launch()
        return self.backend.indices()


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


def _thin_sharded_integrand(integrand: SteinIntegrand, n_points: int, group=None,
                            use_graph: bool = True) -> np.ndarray:
    n_points = int(n_points)
    if n_points < 1:
        raise ValueError('n_points must be >= 1')
    rank, world = _world(group)
    if world > integrand.n:
        raise ValueError(f'{world} ranks for {integrand.n} rows: every rank needs at least one row')
    r0, r1 = shard_bounds(integrand.n, rank, world)
    backend = HipShardBackend(integrand, r0, r1, world, n_points)
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_backend(group) == 'nccl':
        return GraphedShardedGreedy(backend, n_points, group, use_graph).run()
    return run_sharded(backend, n_points, group)
