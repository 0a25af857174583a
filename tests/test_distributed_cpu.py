"""Multi-GPU combine logic on CPU: world_size-2 gloo runs of pinot_amd.distributed.reduce_tables.

Each rank holds half of the segments; its dense partial tables (the layout ph_query_dense_layout
produces: count, then SUM/MIN/MAX per value column) are built from the oracle's per-rank results, merged
with reduce_tables (all_reduce + slice on gloo; reduce_scatter on RCCL), finalised per key shard and
gathered on rank 0, which compares with the oracle over ALL segments -- the GroupByCombineOperator result.
Covers the three merge shapes: aggregation-only (one group), a small key space (all-reduce, rank 0 owns
it) and a large one (key-range shards on both ranks).
"""
import math
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

QUERIES = [
    "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), SUM(d) FROM t WHERE f BETWEEN 10 AND 70",
    "SELECT a, COUNT(*), SUM(m), MIN(d), MAX(m) FROM t WHERE f < 50 GROUP BY a ORDER BY a LIMIT 1000",
    "SET numGroupsLimit=200000; SELECT a, b, COUNT(*), SUM(m), MIN(m), MAX(d), SUM(d) FROM t "
    "GROUP BY a, b ORDER BY a, b LIMIT 200000",
]


def _tables(seed=11, nseg=4, n=3000):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        out.append({
            "a": (rng.integers(0, 37, n).astype(np.int32) * 3, "INT"),
            "b": (rng.integers(0, 300, n).astype(np.int32) - 100, "INT"),
            "f": (rng.integers(0, 100, n).astype(np.int32), "INT"),
            "m": (rng.integers(-1000, 1 << 20, n).astype(np.int32), "INT"),
            "d": (np.round(rng.normal(0, 100, n), 2), "DOUBLE"),
        })
    return out


def _layout(q, types):
    """Python mirror of ph_query_dense_layout: [(kind, column)]."""
    vals = []
    ops = {}
    for a in q.aggregations:
        if a.function == "COUNT":
            continue
        if a.column not in ops:
            vals.append(a.column)
            ops[a.column] = set()
        ops[a.column].add(a.function)
    lay = [("COUNT", None)]
    for c in vals:
        for f in ("SUM", "MIN", "MAX"):
            if f in ops[c]:
                lay.append((f, c))
    return lay


def _dicts(q, tables):
    return {g: np.unique(np.concatenate([t[g][0] for t in tables])) for g in q.group_by}


def _dense(q, res, lay, dicts, types):
    import torch
    sizes = [len(dicts[g]) for g in q.group_by]
    G = int(np.prod(sizes)) if sizes else 1
    strides = np.cumprod([1] + sizes[:-1]) if sizes else []
    ident = {"COUNT": 0, "SUM": 0, "MIN": np.iinfo(np.int64).max, "MAX": np.iinfo(np.int64).min}
    arrs = []
    for kind, col in lay:
        if kind == "SUM" and types[col] == "DOUBLE":
            arrs.append(np.zeros(G, np.float64))
        else:
            arrs.append(np.full(G, ident[kind], np.int64))
    fidx = {(a.function, a.column): i for i, a in enumerate(q.aggregations)}
    count_idx = [i for i, a in enumerate(q.aggregations) if a.function == "COUNT"][0]
    for key, agg in zip(res.keys, res.aggs):
        gid = 0
        for j, g in enumerate(q.group_by):
            gid += int(np.searchsorted(dicts[g], key[j])) * int(strides[j])
        for t, (kind, col) in enumerate(lay):
            v = agg[count_idx] if kind == "COUNT" else agg[fidx[(kind, col)]]
            if kind in ("MIN", "MAX") and types[col] == "DOUBLE":
                # order key of a double, as the device tables hold it
                b = np.array([v], np.float64).view(np.int64)[0]
                v = b if b >= 0 else b ^ np.iinfo(np.int64).max
            arrs[t][gid] = v
    return G, [torch.from_numpy(a) for a in arrs]


def _finalize(q, shards, g0, g1, lay, dicts, types):
    sizes = [len(dicts[g]) for g in q.group_by]
    strides = np.cumprod([1] + sizes[:-1]) if sizes else []
    cnt = shards[0].numpy()
    rows = []
    for i in np.nonzero(cnt)[0] if q.group_by else [0]:
        g = g0 + int(i)
        key = tuple(dicts[c][(g // int(strides[j])) % sizes[j]].item() for j, c in enumerate(q.group_by))
        vals = {}
        for t, (kind, col) in enumerate(lay):
            v = shards[t].numpy()[i]
            if kind in ("MIN", "MAX") and types[col] == "DOUBLE":
                v = int(v)
                b = v if v >= 0 else v ^ np.iinfo(np.int64).max
                v = float(np.array([b], np.int64).view(np.float64)[0])
            vals[(kind, col)] = v
        agg = []
        for a in q.aggregations:
            if a.function == "COUNT":
                agg.append(int(cnt[i]))
            else:
                agg.append(float(vals[(a.function, a.column)]))
        rows.append((key, agg))
    return rows


def _worker(rank, world, port, sql):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from oracle import oracle as O
    from pinot_amd.distributed import Layout, reduce_tables
    from pinot_amd.query import parse_sql
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q = parse_sql(sql)
        tables = _tables()
        types = {c: tables[0][c][1] for c in tables[0]}
        mine = [O.build_segment(f"s{i}", t) for i, t in enumerate(tables) if i % world == rank]
        res = O.execute(q, mine)
        lay = _layout(q, types)
        dicts = _dicts(q, tables)
        G, dense = _dense(q, res, lay, dicts, types)
        layout = Layout(G, [1] * len(lay),
                        [{"COUNT": 0, "SUM": 1 if (k == "SUM" and types[c] == "DOUBLE") else 0,
                          "MIN": 2, "MAX": 3}[k] for k, c in lay])
        shards, g0, g1 = reduce_tables(dense, layout)
        rows = _finalize(q, shards, g0, g1, lay, dicts, types) if g1 > g0 else []
        got = [None] * world if rank == 0 else None
        dist.gather_object(rows, got, dst=0)
        if rank == 0:
            merged = sorted([r for part in got for r in part])
            exp = O.execute(q, [O.build_segment(f"s{i}", t) for i, t in enumerate(tables)])
            want = sorted(zip(exp.keys, exp.aggs)) if q.group_by else [((), exp.aggs[0])]
            assert len(merged) == len(want), (len(merged), len(want))
            for (k1, a1), (k2, a2) in zip(merged, want):
                assert k1 == tuple(k2), (k1, k2)
                for x, y in zip(a1, a2):
                    if isinstance(y, float) and y != 0 and not math.isinf(y):
                        assert abs(x - y) <= 1e-9 * abs(y), (k1, x, y)
                    else:
                        assert x == y, (k1, x, y)
            # the large key space really was split across both ranks
            if G > 4096:
                assert all(len(p) > 0 for p in got)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("sql", QUERIES, ids=["agg_only", "small_groups", "key_shards"])
def test_gloo_world2_combine(sql):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), sql), nprocs=2, join=True)


def test_shard_bounds_cover_key_space():
    from pinot_amd.distributed import shard_bounds
    for G in (1, 63, 64, 65, 1000, 999_999, 1_000_000):
        for world in (1, 2, 3, 8):
            covered = []
            for r in range(world):
                s, g0, g1 = shard_bounds(G, world, r)
                assert s % 64 == 0 and s * world >= G
                covered.append((g0, g1))
            assert covered[0][0] == 0 and covered[-1][1] == G
            for (a0, a1), (b0, b1) in zip(covered, covered[1:]):
                assert a1 == b0
