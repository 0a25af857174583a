"""Multi-GPU combine: segments sharded across the GPUs of a node, partial results merged over xGMI.

The reference combines per-segment results on one server with a thread pool
(GroupByCombineOperator.java:125-197: ``ConcurrentIndexedTable.upsert`` per key; aggregation-only:
AggregationResultsBlockMerger.java:33-45).  Here every GPU (one process per GPU, ``torch.distributed``)
scans its own segments into DENSE partial tables over table-level dictionaries (``ph_query_execute_dense``),
so the cross-GPU merge is a reduction of same-shaped tensors:

* group-by: one ``reduce_scatter`` per table by key range -- each rank ends up owning 1/N of the keys,
  fully merged -- then ``ph_dense_finalize`` materialises only that shard (keys decoded, values converted);
* aggregation-only (one group): ``all_reduce``, finalised on rank 0.

Reduce ops per table come from the layout (COUNT/SUM add, MIN/MAX min/max on int64 values or order keys,
HLL registers max == ``HyperLogLog.addAll``).  On ROCm the "nccl" backend is RCCL; its ring/direct
algorithms run over the xGMI links.  The gloo backend (CPU tests) has no reduce-scatter, so the same
code path falls back to all_reduce + slice there.

A merged shard is the server-side combine result for its key range (what ``GroupByCombineOperator``
hands to ``InstanceResponseOperator``); ``gather_to_root`` concatenates shards on rank 0 when a single
result is wanted.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import native as N

# reduce op -> (torch dtype name, identity value used for padding)
_OP_DTYPE = {
    N.PH_REDUCE_SUM_I64: ("int64", 0),
    N.PH_REDUCE_SUM_F64: ("float64", 0.0),
    N.PH_REDUCE_MIN_I64: ("int64", np.iinfo(np.int64).max),
    N.PH_REDUCE_MAX_I64: ("int64", np.iinfo(np.int64).min),
    N.PH_REDUCE_MAX_U32: ("int32", 0),  # registers <= 32: int32 max == uint32 max
}


@dataclass
class Layout:
    num_groups: int
    elems_per_group: List[int]
    reduce_ops: List[int]

    @staticmethod
    def from_native(lay) -> "Layout":
        n = lay.num_tables
        return Layout(int(lay.num_groups), [int(x) for x in lay.elems_per_group[:n]],
                      [int(x) for x in lay.reduce_op[:n]])


def shard_bounds(num_groups: int, world: int, rank: int, align: int = 64) -> Tuple[int, int, int]:
    """Key shard of ``rank``: (shard size S, g0, g1) with S a multiple of ``align`` groups."""
    s = -(-num_groups // world)
    s = -(-s // align) * align
    g0 = min(num_groups, rank * s)
    g1 = min(num_groups, g0 + s)
    return s, g0, g1


def alloc_tables(layout: Layout, world: int, device):
    """Dense tables padded to ``world`` equal key shards, padding set to each op's identity."""
    import torch
    s, _, _ = shard_bounds(layout.num_groups, world, 0)
    padded = s * world
    tabs = []
    for per, op in zip(layout.elems_per_group, layout.reduce_ops):
        dt, ident = _OP_DTYPE[op]
        t = torch.empty(padded * per, dtype=getattr(torch, dt), device=device)
        if padded > layout.num_groups:
            t[layout.num_groups * per:].fill_(ident)
        tabs.append(t)
    return tabs


def _torch_op(op):
    import torch.distributed as dist
    if op in (N.PH_REDUCE_SUM_I64, N.PH_REDUCE_SUM_F64):
        return dist.ReduceOp.SUM
    if op == N.PH_REDUCE_MIN_I64:
        return dist.ReduceOp.MIN
    return dist.ReduceOp.MAX


def reduce_tables(tables, layout: Layout, group=None, small_groups: int = 4096):
    """Merge the ranks' dense tables.  Returns (shard tables, g0, g1): rank r owns merged keys [g0, g1).
    Aggregation-only and small key spaces are all-reduced and owned by rank 0 alone."""
    import torch
    import torch.distributed as dist
    G = layout.num_groups
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return [t[: G * per] for t, per in zip(tables, layout.elems_per_group)], 0, G
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if G <= small_groups:
        for t, op in zip(tables, layout.reduce_ops):
            dist.all_reduce(t, op=_torch_op(op), group=group)
        return ([t[: G * per] for t, per in zip(tables, layout.elems_per_group)], 0, G) if rank == 0 else \
            ([t[:0] for t in tables], G, G)
    s, g0, g1 = shard_bounds(G, world, rank)
    gloo = dist.get_backend(group) == "gloo"
    out = []
    for t, op, per in zip(tables, layout.reduce_ops, layout.elems_per_group):
        if gloo:  # no reduce_scatter in gloo: all_reduce + own slice
            dist.all_reduce(t, op=_torch_op(op), group=group)
            shard = t[rank * s * per:(rank + 1) * s * per]
        else:
            shard = torch.empty(s * per, dtype=t.dtype, device=t.device)
            dist.reduce_scatter_tensor(shard, t, op=_torch_op(op), group=group)
        out.append(shard[: (g1 - g0) * per])
    return out, g0, g1


class DistributedQuery:
    """One rank's view of a multi-GPU query over its own pinned segments (ctx: GpuContext on this GPU)."""

    def __init__(self, ctx, group=None):
        self.ctx = ctx
        self.group = group
        # (query, segment set) -> (layout, padded tables): planning the layout and allocating / filling the tables
        # once per query shape, not per step (ph_query_execute_dense re-initialises the live rows every call; the
        # padding rows keep their reduction identities through every reduction)
        self._cache = {}

    def execute(self, q, segments: Sequence, copy: bool = True):
        """Returns (this rank's finalised key shard or None, (g0, g1), scan statistics of this rank).  The scan
        statistics come from ph_query_execute_dense (device_ms = this rank's scan kernels); the shard's own
        statistics describe only the finalisation."""
        import time

        import torch
        dev = torch.device("cuda", self.ctx.device)
        # run the library on torch's current stream so RCCL and the scan are ordered without host syncs
        self.ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        import torch.distributed as dist
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        t0 = time.perf_counter()
        key = (repr(q), tuple(id(s) for s in segments), world, self.ctx.device)
        hit = self._cache.get(key)
        if hit is None:
            layout = Layout.from_native(self.ctx.dense_layout(q, segments))
            hit = (layout, alloc_tables(layout, world, dev), list(segments))  # holds the segments: ids stay unique
            if len(self._cache) >= 16:
                self._cache.pop(next(iter(self._cache)))
            self._cache[key] = hit
        layout, tables = hit[0], hit[1]
        scan_stats = self.ctx.execute_dense(q, segments, [t.data_ptr() for t in tables])  # returns after the scan
        t1 = time.perf_counter()
        shards, g0, g1 = reduce_tables(tables, layout, self.group)
        torch.cuda.current_stream(dev).synchronize()  # the collectives ran on torch's stream
        t2 = time.perf_counter()
        res = None
        if g1 > g0:
            res = self.ctx.dense_finalize(q, segments, [t.data_ptr() for t in shards], g0, g1, copy=copy)
        # host-clock phase times of this rank (ms): plan + scan, cross-GPU reduction, shard finalisation
        self.last_times = {"scan_ms": (t1 - t0) * 1e3, "reduce_ms": (t2 - t1) * 1e3,
                           "finalize_ms": (time.perf_counter() - t2) * 1e3}
        return res, (g0, g1), scan_stats


def gather_to_root(res, group=None) -> Optional[list]:
    """(keys, aggs) of every rank's shard, concatenated on rank 0 (None elsewhere)."""
    import torch.distributed as dist
    payload = None if res is None else (res.keys, res.aggs)
    out = [None] * dist.get_world_size(group) if dist.get_rank(group) == 0 else None
    dist.gather_object(payload, out, dst=0, group=group)
    if out is None:
        return None
    keys, aggs = [], []
    for p in out:
        if p is not None:
            keys += p[0]
            aggs += p[1]
    return [keys, aggs]
