"""GPU: the dense-partials C-ABI (ph_query_dense_layout / ph_query_execute_dense / ph_dense_finalize) that the
multi-GPU combine is built on.  Finalising the dense tables whole, or as key shards concatenated, must give
exactly ph_query_execute's result -- for every plan mode (aggregation-only, LDS table, HBM table,
partitioned) -- and DistributedQuery at world size 1 must match too.
"""
import os

import numpy as np
import pytest

from pinot_amd.query import parse_sql
from pinot_amd.segment import create_segment

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _segs(ctx, seed, n=200_000, nseg=3, ca=50, cb=2000):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(nseg):
        cols = {
            "a": (rng.integers(0, ca, n).astype(np.int32), "INT"),
            "b": (rng.integers(0, cb, n).astype(np.int32), "INT"),
            "f": (rng.integers(0, 100, n).astype(np.int32), "INT"),
            "m": (rng.integers(0, 1 << 20, n).astype(np.int32), "INT"),
            "d": (np.round(rng.normal(0, 10, n), 3), "DOUBLE"),
        }
        out.append(ctx.pin(create_segment(f"dense_{seed}_{i}", cols)))
    ctx.set_table_dictionary("a", "INT", np.arange(ca, dtype=np.int32))
    ctx.set_table_dictionary("b", "INT", np.arange(cb, dtype=np.int32))
    return out


def _rows(r):
    return sorted(zip(r.keys, [tuple(a) for a in r.aggs]))


def _assert_rows_match(got, exp, msg):
    """Keys, COUNT, integer SUM and MIN/MAX bit-exact; a non-integral value (DOUBLE SUM over column d, whose
    float64 atomics make the summation order run-dependent) within 1e-9 relative (BASELINE north_star)."""
    assert len(got) == len(exp), msg
    for (kg, ag), (ke, ae) in zip(got, exp):
        assert kg == ke, msg
        assert len(ag) == len(ae), msg
        for x, y in zip(ag, ae):
            if x == y:
                continue
            assert float(y) != round(float(y)), (msg, kg, x, y)  # only non-integral (DOUBLE) sums may differ
            assert abs(x - y) <= 1e-9 * abs(y), (msg, kg, x, y)


QUERIES = [
    ("SELECT COUNT(*), SUM(m), MIN(m), MAX(m), SUM(d) FROM t WHERE f BETWEEN 10 AND 70", 1),
    ("SELECT a, COUNT(*), SUM(m), MIN(d), MAX(m) FROM t WHERE f < 50 GROUP BY a", 2),
    ("SET numGroupsLimit=200000; SELECT a, b, COUNT(*), SUM(m), MAX(d) FROM t GROUP BY a, b", 3),
    ("SET numGroupsLimit=200000; SELECT a, b, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE f < 60 "
     "GROUP BY a, b", 4),
]


@pytest.mark.parametrize("sql,mode", QUERIES, ids=["agg", "lds", "global", "partition"])
def test_dense_matches_execute(ctx, sql, mode):
    import torch

    from pinot_amd.distributed import Layout, alloc_tables, shard_bounds
    segs = _segs(ctx, 5)
    q = parse_sql(sql)
    ref = ctx.execute(q, segs)
    assert ref.stats.mode == mode
    lay = Layout.from_native(ctx.dense_layout(q, segs))
    assert lay.num_groups == (1 if mode == 1 else (50 if mode == 2 else 100_000))
    for world in (1, 3):
        tabs = alloc_tables(lay, world, torch.device("cuda", 0))
        ctx.execute_dense(q, segs, [t.data_ptr() for t in tabs])
        torch.cuda.synchronize()
        rows = []
        for r in range(world):
            s, g0, g1 = shard_bounds(lay.num_groups, world, r)
            if g1 <= g0:
                continue
            shard = [t[g0 * per:g1 * per] for t, per in zip(tabs, lay.elems_per_group)]
            res = ctx.dense_finalize(q, segs, [t.data_ptr() for t in shard], g0, g1)
            rows += _rows(res)
        _assert_rows_match(sorted(rows), _rows(ref), world)


def test_empty_rank_layout_follows_schema(ctx):
    # a rank holding no segment must build the same dense layout as the others: DOUBLE SUM reduces as f64 and
    # MIN/MAX finalise as doubles (the value type defaulted to integer on an empty rank)
    from pinot_amd import native as N
    from pinot_amd.distributed import Layout, alloc_tables
    import torch
    segs = _segs(ctx, 6)
    q = parse_sql("SELECT a, COUNT(*), SUM(d), MIN(d), MAX(m) FROM t GROUP BY a")
    full = Layout.from_native(ctx.dense_layout(q, segs))
    with pytest.raises(N.PinotHipError):
        ctx.dense_layout(parse_sql("SELECT a, SUM(zz) FROM t GROUP BY a"), [])
    ctx.set_schema({"d": "DOUBLE", "m": "INT"})
    empty = Layout.from_native(ctx.dense_layout(q, []))
    assert empty.reduce_ops == full.reduce_ops and empty.num_groups == full.num_groups
    # the empty rank's tables are the reduction identities and finalise to no rows
    tabs = alloc_tables(empty, 1, torch.device("cuda", 0))
    ctx.execute_dense(q, [], [t.data_ptr() for t in tabs])
    torch.cuda.synchronize()
    res = ctx.dense_finalize(q, [], [t.data_ptr() for t in tabs], 0, empty.num_groups)
    assert len(res.keys) == 0


def test_distributed_query_world1(ctx):
    import torch.distributed as dist

    from pinot_amd.distributed import DistributedQuery
    segs = _segs(ctx, 9)
    q = parse_sql("SET numGroupsLimit=200000; SELECT a, b, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t "
                  "WHERE f < 60 GROUP BY a, b")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        res, (g0, g1), scan = DistributedQuery(ctx).execute(q, segs)
        assert (g0, g1) == (0, 100_000)
        assert _rows(res) == _rows(ctx.execute(q, segs))
        # the scan's device time is what bench.py's roofline divides by (it was dropped)
        assert scan.device_ms > 0
    finally:
        dist.destroy_process_group()
        ctx.set_stream(0)


def test_dense_partials_reject_segment_trim(ctx):
    # GroupByOperator's segment trim (ORDER BY + minSegmentGroupTrimSize > 0) cannot run on whole dense partials: the
    # dense entry points refuse it (PH_ERR_UNSUPPORTED) instead of returning untrimmed groups; DistributedQuery too
    from pinot_amd import native as N
    from pinot_amd.distributed import DistributedQuery
    segs = _segs(ctx, 41, n=50_000, nseg=2)
    q = parse_sql("SET minSegmentGroupTrimSize=10; SELECT a, b, SUM(m) FROM t GROUP BY a, b ORDER BY SUM(m) DESC "
                  "LIMIT 5")
    with pytest.raises(N.UnsupportedError):
        ctx.dense_layout(q, segs)
    with pytest.raises(N.UnsupportedError):
        DistributedQuery(ctx).execute(q, segs)
    # without the ORDER BY the option does not apply (GroupByOperator trims only ordered group-bys)
    ctx.dense_layout(parse_sql("SET minSegmentGroupTrimSize=10; SELECT a, b, SUM(m) FROM t GROUP BY a, b LIMIT 5"),
                     segs)
