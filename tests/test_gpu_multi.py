"""GPU: the in-library multi-GPU combine (ph_ctx_create_multi) -- a Pinot server combines all of a query's segments in
one JVM (GroupByCombineOperator.java:125-197), so one context spans the node's GPUs: segments are placed by pinned
rows and the devices' dense partial tables merge inside libpinot_hip by a reduce-scatter over key shards, each device
finalising its own shard.  The GPU box has one MI355X, so the contexts are LOGICAL shards of cuda:0 (devices [0, 0]
and [0, 0, 0]): each shard scans its own segments into its own tables, the peer transport (peer copies of the other
shards' key shards + the reduce kernel, PH_TRANSPORT_PEER) builds every merged shard, and every shard finalises --
including a shard whose device holds none of the query's segments (moved to an active device) and shards past the
key space (G < 64 D).  The RCCL transport needs distinct devices: its test runs only where hipGetDeviceCount() >= 2.
Every result must equal the oracle's and the one-device context's: bit-exact COUNT / integer SUM / MIN / MAX / HLL
registers, DOUBLE SUM within 1e-9 relative."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment

pytestmark = pytest.mark.gpu

RTOL = 1e-9


def _tables():
    rng = np.random.default_rng(4242)
    out = []
    for n in (400_000, 250_013, 300_007, 120_001):
        out.append({"g1": (rng.integers(0, 1000, n).astype(np.int32), "INT"),
                    "g2": (rng.integers(0, 1000, n).astype(np.int32), "INT"),
                    "f": (rng.integers(0, 1000, n).astype(np.int32), "INT"),
                    "m": (rng.integers(0, 1 << 20, n).astype(np.int32), "INT"),
                    "md": (np.round(rng.random(n), 6), "DOUBLE"),
                    "c": (rng.integers(0, 1000, n).astype(np.int32), "INT"),
                    "u": (rng.integers(0, 1 << 27, n).astype(np.int32), "INT"),
                    "s": (np.array(["k%d" % i for i in range(37)], dtype=object)[rng.integers(0, 37, n)], "STRING"),
                    "h1": (rng.integers(0, 20000, n).astype(np.int32), "INT"),
                    "h2": (rng.integers(0, 20000, n).astype(np.int32), "INT"),
                    "h3": (rng.integers(0, 20000, n).astype(np.int32), "INT")})
    return out


@pytest.fixture(scope="module")
def setup():
    from pinot_amd.engine import GpuContext
    tables = _tables()
    multi = GpuContext(devices=[0, 0])
    single = GpuContext(0)
    segs_m = [multi.pin(create_segment(f"mg{i}", t, inverted=("c",)), hll_columns=("u",)) for i, t in enumerate(tables)]
    segs_s = [single.pin(create_segment(f"sg{i}", t, inverted=("c",))) for i, t in enumerate(tables)]
    ora = [O.build_segment(f"og{i}", t, inverted=("c",)) for i, t in enumerate(tables)]
    yield multi, single, segs_m, segs_s, ora
    multi.close()
    single.close()


def _rows_equal(got, exp):
    assert len(got) == len(exp), (len(got), len(exp))
    for g, e in zip(got, exp):
        for a, b in zip(g, e):
            if isinstance(b, float) and b != 0 and not np.isinf(b):
                assert abs(a - b) <= RTOL * abs(b), (g, e)
            else:
                assert np.array_equal(a, b) if isinstance(b, np.ndarray) else a == b, (g, e)


def test_placement_balances_rows(setup):
    multi, _, segs, _, _ = setup
    dev = [multi.segment_device(s) for s in segs]
    rows = [0, 0]
    for s, d in zip(segs, dev):
        rows[d] += s.num_docs
    # greedy by pinned rows: 400k -> 0, 250k -> 1, 300k -> 1 (250k < 400k), 120k -> 0 (400k < 550k)
    assert dev == [0, 1, 1, 0]
    assert sorted(rows) == [520_001, 550_020]


QUERIES = [
    # config 3's shape: filter + 2-dim group-by, ~1M key space (partitioned plan on each shard)
    "SET numGroupsLimit=2000000; SELECT g1, g2, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t WHERE f BETWEEN 0 AND 499 "
    "GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 2000000",
    # DOUBLE SUM
    "SELECT g1, SUM(md), MIN(md), MAX(md), COUNT(*) FROM t WHERE f < 700 GROUP BY g1 ORDER BY g1 LIMIT 2000",
    # config 5's shape: DISTINCTCOUNTHLL under an inverted-index filter (aggregation-only: one group)
    "SELECT DISTINCTCOUNTHLL(u) FROM t WHERE c IN (1, 5, 9, 77, 300, 301, 302, 500, 600, 999)",
    "SELECT g1, DISTINCTCOUNTHLL(u), COUNT(*) FROM t WHERE c IN (1, 5, 9) GROUP BY g1 ORDER BY g1 LIMIT 2000",
    # aggregation-only with MIN / MAX, and STRING keys (no table dictionary: one union over both shards)
    "SELECT COUNT(*), SUM(m), MIN(m), MAX(m), SUM(md) FROM t WHERE f BETWEEN 100 AND 300",
    "SELECT s, COUNT(*), SUM(m) FROM t WHERE f > 10 GROUP BY s ORDER BY s LIMIT 100",
    # a key space beyond the dense budget (20000^3): per-shard hash tables, merged on the host by value
    "SET numGroupsLimit=10000000; SELECT h1, h2, h3, COUNT(*), SUM(m) FROM t WHERE f < 3 GROUP BY h1, h2, h3 "
    "ORDER BY h1, h2, h3 LIMIT 10000000",
    # segment group trim: per segment, each on its own shard
    "SET minSegmentGroupTrimSize=30; SELECT g1, SUM(m), COUNT(*) FROM t WHERE f < 100 GROUP BY g1 "
    "ORDER BY SUM(m) DESC LIMIT 5",
]


@pytest.mark.parametrize("sql", QUERIES)
def test_multi_shard_matches_oracle_and_one_device(setup, sql):
    multi, single, segs_m, segs_s, ora = setup
    q = parse_sql(sql)
    r = multi.execute(q, segs_m)
    e = O.execute(q, ora)
    _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, e.keys, e.aggs).rows)
    s = single.execute(q, segs_s)
    _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, s.keys, s.aggs).rows)
    assert r.num_groups == s.num_groups
    for a in ("num_docs_scanned", "num_entries_scanned_in_filter", "num_entries_scanned_post_filter",
              "num_total_docs"):
        assert getattr(r.stats, a) == getattr(s.stats, a), a
    if "minSegmentGroupTrimSize" not in sql:
        assert r.stats.num_devices == 2


def test_forced_host_merge_matches(setup, monkeypatch):
    # the value-keyed host combine (the fallback for shapes the dense tables do not serve), forced on a dense shape
    multi, single, segs_m, segs_s, _ = setup
    monkeypatch.setenv("PH_MULTI_HOST_MERGE", "1")
    for sql in QUERIES[:3]:
        q = parse_sql(sql)
        r = multi.execute(q, segs_m)
        s = single.execute(q, segs_s)
        _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, s.keys, s.aggs).rows)


@pytest.fixture(scope="module")
def setup3():
    """three logical shards; the queries below touch only the segments placed on shards 0 and 1"""
    from pinot_amd.engine import GpuContext
    tables = _tables()
    multi = GpuContext(devices=[0, 0, 0])
    single = GpuContext(0)
    segs_m = [multi.pin(create_segment(f"m3g{i}", t, inverted=("c",)), hll_columns=("u",)) for i, t in enumerate(tables)]
    segs_s = [single.pin(create_segment(f"s3g{i}", t, inverted=("c",))) for i, t in enumerate(tables)]
    ora = [O.build_segment(f"o3g{i}", t, inverted=("c",)) for i, t in enumerate(tables)]
    yield multi, single, segs_m, segs_s, ora
    multi.close()
    single.close()


@pytest.mark.parametrize("sql", QUERIES[:6])
def test_sharded_finalize_with_idle_shard(setup3, sql):
    multi, single, segs_m, segs_s, ora = setup3
    dev = [multi.segment_device(s) for s in segs_m]
    # greedy by pinned rows over three shards: 400k -> 0, 250k -> 1, 300k -> 2, 120k -> 1
    assert dev == [0, 1, 2, 1]
    pick = [i for i, d in enumerate(dev) if d != 2]  # shard 2 holds none of the query's segments
    q = parse_sql(sql)
    r = multi.execute(q, [segs_m[i] for i in pick])
    e = O.execute(q, [ora[i] for i in pick])
    _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, e.keys, e.aggs).rows)
    s = single.execute(q, [segs_s[i] for i in pick])
    _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, s.keys, s.aggs).rows)
    assert r.num_groups == s.num_groups
    assert r.stats.num_devices == 2
    # and over all three shards
    r = multi.execute(q, segs_m)
    e = O.execute(q, ora)
    _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, e.keys, e.aggs).rows)
    assert r.stats.num_devices == 3


def _device_count():
    import torch
    return torch.cuda.device_count()


@pytest.mark.skipif("_device_count() < 2")
@pytest.mark.parametrize("transport", ["peer", "rccl"])
def test_distinct_devices(transport):
    """two real GPUs: both transports against the oracle (only on a multi-GPU node)"""
    from pinot_amd.engine import GpuContext
    tables = _tables()
    multi = GpuContext(devices=[0, 1], transport=transport)
    try:
        segs = [multi.pin(create_segment(f"dd{i}", t, inverted=("c",)), hll_columns=("u",)) for i, t in enumerate(tables)]
        ora = [O.build_segment(f"odd{i}", t, inverted=("c",)) for i, t in enumerate(tables)]
        for sql in QUERIES[:6]:
            q = parse_sql(sql)
            r = multi.execute(q, segs)
            e = O.execute(q, ora)
            _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, e.keys, e.aggs).rows)
            # one device idle: shard 1's keys finalise on device 0
            on0 = [i for i, s in enumerate(segs) if multi.segment_device(s) == 0]
            r = multi.execute(q, [segs[i] for i in on0])
            e = O.execute(q, [ora[i] for i in on0])
            _rows_equal(reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, e.keys, e.aggs).rows)
    finally:
        multi.close()


def test_phases_reported(setup):
    multi, _, segs_m, _, _ = setup
    r = multi.execute(parse_sql(QUERIES[0]), segs_m)
    assert r.stats.merge_ms > 0 and r.stats.finalize_ms > 0 and r.stats.device_ms > 0
