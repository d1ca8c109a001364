"""Multi-GPU TPE suggestion: one process per GPU over torch.distributed.

Two ways the suggest path shards:

* **Batched asynchronous suggestions** (config 5): every rank serves its own
  suggestions (distinct seeds) on the same history.  Nothing is exchanged:
  :func:`suggestion_slice` only decides which seeds a rank owns.

* **One suggestion sharded over ranks** (configs 2-4): rank r draws and
  scores the global candidate range :func:`shard_range` of every hp.  The
  device draws are counter-based (Philox keyed by seed, counter = global
  candidate index), so the union of the shards is exactly the candidate set
  of the unsharded suggest.  After each conditional level the per-hp
  ``(score, value, index)`` winners (32-byte ``tpe_result`` records,
  [S][P]) are all-gathered -- RCCL over xGMI on GPU, gloo in the CPU tests --
  and merged on the device by ``tpe_plan_merge`` with numpy argmax semantics
  (first maximum, a NaN wins at its first index, tpe.py:756), so the next
  level's activity test and the returned values are identical to one GPU's.

RCCL has no max-loc reduction; an all-gather of G x S x P x 32 bytes followed
by a deterministic device merge is both exact and, at these sizes
(kilobytes), latency-bound at one collective per level.
"""
from __future__ import annotations

import os

import numpy as np

from . import _engine as E

RECORD_BYTES = E.RESULT_DTYPE.itemsize  # sizeof(tpe_result) == 32


def shard_range(n: int, rank: int, world: int, align: int = 1):
    """(begin, count) of rank's share of [0, n): contiguous, covering [0, n)
    exactly once over all ranks, every boundary a multiple of ``align``
    (balanced to within one unit of ``align``).  With
    ``align=E.SHARD_ALIGN`` the shards' large draws are bucketed in the same
    global blocks as the unsharded suggest's, so the merged result is byte
    for byte the one-device result (include/tpe_engine.h TPE_SHARD_ALIGN)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError('bad rank/world %r/%r' % (rank, world))
    if n < 0:
        raise ValueError('n < 0')
    if align < 1:
        raise ValueError('align < 1')
    units = -(-n // align)
    base, extra = divmod(units, world)
    u0 = rank * base + min(rank, extra)
    u1 = u0 + base + (1 if rank < extra else 0)
    begin, end = min(n, u0 * align), min(n, u1 * align)
    return begin, end - begin


def suggestion_slice(n_suggest: int, rank: int, world: int):
    """Suggestion indices a rank serves in batched asynchronous mode."""
    b, c = shard_range(n_suggest, rank, world)
    return range(b, b + c)


def gather_records(local, group=None, out=None):
    """All-gather a rank's flat byte tensor of result records.

    Returns one contiguous tensor [world * local.numel()] in rank order, the
    [world][S][P] layout ``tpe_plan_merge`` expects (into ``out`` when given:
    a preallocated buffer of that size on the same device).  Uses the fused
    ``all_gather_into_tensor`` (one RCCL call) where the backend has it and a
    list all-gather otherwise (gloo on CPU)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if local.is_cuda and dist.get_backend(group) == 'nccl':
        if out is None:
            out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local, group=group)
        return out
    # gloo: stage through host memory (CPU tests; several ranks on one GPU)
    src = local.cpu()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    return torch.cat(parts).to(local.device)


def merge_records_host(gathered: np.ndarray) -> np.ndarray:
    """Host restatement of k_merge for tests and diagnostics only: combine
    [world][S][P] records with numpy argmax semantics.  The product path
    merges on the device (ShardedSuggest)."""
    world, S, P = gathered.shape
    out = np.empty((S, P), dtype=E.RESULT_DTYPE)
    for s in range(S):
        for p in range(P):
            best = None
            active = 0
            for r in range(world):
                q = gathered[r, s, p]
                active |= int(q['active'])
                if q['index'] < 0:
                    continue
                if best is None or _better(q, best):
                    best = q
            if best is None or not active:
                out[s, p] = (np.nan, np.nan, -1, active, 0)
            else:
                out[s, p] = (best['score'], best['value'], best['index'], 1, 0)
    return out


def _better(a, b):
    na, nb = np.isnan(a['score']), np.isnan(b['score'])
    if na or nb:
        return a['index'] < b['index'] if (na and nb) else bool(na)
    if a['score'] != b['score']:
        return a['score'] > b['score']
    return a['index'] < b['index']


class ShardedSuggest(object):
    """One suggestion's candidates sharded over the ranks of ``group``.

    ``plan`` is this rank's :class:`hyperopt_amd._engine.Plan` (same space,
    same history).  Every engine call, record copy and collective runs on
    one torch stream (``self.stream``), which waits on torch's current stream
    at each call: fit the plan with :meth:`fit` (on that stream), or order a
    fit made elsewhere before :meth:`suggest` yourself -- the engine's calls
    are stream-ordered, not synchronous (include/tpe_engine.h).  Candidate
    shards are aligned to ``E.SHARD_ALIGN``, so the merged winners are the
    one-device winners byte for byte.
    """

    def __init__(self, plan, group=None):
        import torch
        import torch.distributed as dist
        self.plan = plan
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = torch.device('cuda', plan.engine.device)
        # a real (non-null) stream shared by the engine launches, the record
        # copies and the collective: stream 0 would mean "the engine's own
        # stream" at the C ABI and leave torch unordered with it
        self.stream = torch.cuda.Stream(self.device)
        self.gather = lambda t, out=None: gather_records(t, self.group, out)
        # (RCCL: the level's all-gather issued directly -- the backend and
        # world size looked up once here, not per level on the host path)
        self._rccl = self.device.type == 'cuda' and dist.get_backend(group) == 'nccl'
        self._all_gather = dist.all_gather_into_tensor
        self._bufs = {}  # S -> (local records, gathered records): reused per call
        self._views = {}  # (address, bytes) -> tensor over the plan's records
        # TPE_EXCHANGE_COPY=1 (A/B): the records copied out of the plan before
        # the all-gather (the round-6 exchange) instead of gathered in place
        self.copy_exchange = os.environ.get('TPE_EXCHANGE_COPY') == '1'

    def _plan_records(self, nbytes):
        """A uint8 tensor over the plan's own device records (the first
        ``nbytes`` of tpe_plan_results_device, through
        ``__cuda_array_interface__``), cached per (address, size); None where
        torch cannot wrap a device pointer (gloo on CPU: the caller copies)."""
        import torch
        if self.copy_exchange or self.device.type != 'cuda' or not torch.cuda.is_available():
            return None
        ptr = self.plan.results_device_ptr()
        if not ptr:
            return None
        key = (ptr, nbytes)
        view = self._views.get(key)
        if view is None and key not in self._views:
            class _Dev(object):
                pass
            d = _Dev()
            d.__cuda_array_interface__ = {'shape': (nbytes,), 'typestr': '|u1',
                                          'data': (ptr, False), 'version': 2}
            try:
                view = torch.as_tensor(d, device=self.device)
                if view.data_ptr() != ptr:
                    view = None
            except (TypeError, RuntimeError, ValueError):
                view = None
            self._views[key] = view
        return view

    def fit(self, **kw):
        """tpe_plan_fit on the sharded stream (ordered before the next
        :meth:`suggest`, after torch's current stream)."""
        import torch
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.plan.fit(stream=self.stream.cuda_stream, **kw)

    def suggest(self, seeds, n_cand, fetch=True):
        import torch
        seeds = E._seeds(seeds)
        S, P = seeds.size, self.plan.n_hp
        begin, count = shard_range(int(n_cand), self.rank, self.world, E.SHARD_ALIGN)
        stream = self.stream.cuda_stream
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            # (the record buffers are allocated once per batch size: the
            # exchange of a level is then one all-gather and one merge launch,
            # nothing allocated on the host path between them)
            bufs = self._bufs.get(S)
            if bufs is None:
                nb = S * P * RECORD_BYTES
                bufs = (torch.empty(nb, dtype=torch.uint8, device=self.device),
                        torch.empty(self.world * nb, dtype=torch.uint8, device=self.device))
                self._bufs[S] = bufs
            local, gbuf = bufs
            lptr = local.data_ptr()
            for level in range(self.plan.n_levels):
                # the level's records stay in the plan (no copy launch); the
                # all-gather reads them there and the merge stores the merged
                # slots both into the plan and into `local` (out_on_device 2)
                self.plan.suggest(seeds, count, cand_begin=begin, level=level, fetch=False,
                                  stream=stream, n_total=int(n_cand))
                mine = self._plan_records(S * P * RECORD_BYTES)
                if mine is None:        # (no device view: the records copied out)
                    self.plan.get_results(out=lptr, stream=stream)
                    mine = local
                if self._rccl and mine.is_cuda:
                    self._all_gather(gbuf, mine, group=self.group)
                    gathered = gbuf
                else:
                    gathered = self.gather(mine, gbuf)
                self.plan.merge(gathered.data_ptr(), self.world, level, out=lptr,
                                stream=stream, n_suggest=S, in_place=not self.copy_exchange)
            if not fetch:  # (the device records: overwritten by the next suggest of S)
                torch.cuda.current_stream(self.device).wait_stream(self.stream)
                return local
            return local.cpu().numpy().view(E.RESULT_DTYPE).reshape(S, P)
