"""GPU: range-indexed columns (FilterOperatorUtils.java:97-120, RangeIndexBasedFilterOperator,
BitSlicedRangeIndexReader).  A column with an exact (version 2) bit-sliced range index turns RANGE -- and EQ when the
column has no inverted index -- into an index-based leaf: no entries scanned in filter, bitmap-based in the AND
order; RANGE never uses an inverted index.  On a dictionary column the leaf's doc bitmap is composed from the index's
bit slices by k_range_slices (BitSlicedRangeIndexReader.getMatchingDocIds :123-211 over RoaringBitmap's RangeBitmap);
test_leaf_reads_the_slices proves it by pinning a forward index that disagrees with the index.  Checked against the
oracle's leaf choice on pinned buffers and on V3 / V1 directories whose index_map / <col>.bitmap.range carry the
index.  Bar: bit-exact results and identical ExecutionStatistics."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment, range_index_bytes
from tests import segment_dirs as SD

pytestmark = pytest.mark.gpu

SQL = [
    ("SELECT COUNT(*) FROM t WHERE r BETWEEN 100 AND 700", 0),        # range-index leaf: nothing scanned
    ("SELECT COUNT(*), SUM(m) FROM t WHERE r > 950", 0),
    ("SELECT COUNT(*), MAX(m) FROM t WHERE r = 17", 0),                # EQ, no inverted index: range index
    ("SELECT COUNT(*), MIN(m) FROM t WHERE s BETWEEN 3 AND 30", 0),    # RANGE on an inverted + range column
    ("SELECT COUNT(*) FROM t WHERE s = 5", 0),                          # EQ with an inverted index: inverted
    ("SELECT g, COUNT(*), SUM(m) FROM t WHERE r < 400 AND f < 300 GROUP BY g ORDER BY g LIMIT 100", None),
    ("SELECT COUNT(*) FROM t WHERE r IN (3, 5, 9)", None),              # IN: no range-index leaf (scan)
    ("SELECT COUNT(*), SUM(m) FROM t WHERE r < 100 OR f BETWEEN 10 AND 20", None),
]


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _cols(n, seed):
    rng = np.random.default_rng(seed)
    return {"r": (rng.integers(0, 1000, n).astype(np.int32), "INT"), "s": (rng.integers(0, 60, n).astype(np.int32), "INT"),
            "f": (rng.integers(0, 1000, n).astype(np.int32), "INT"), "g": (rng.integers(0, 25, n).astype(np.int32), "INT"),
            "m": (rng.integers(-1000, 1 << 20, n).astype(np.int32), "INT")}


def _check(ctx, segs, osegs, sql, entries):
    q = parse_sql(sql)
    r = ctx.execute(q, segs)
    e = O.execute(q, osegs)
    assert reduce_groups(q, r.keys, r.aggs).rows == reduce_groups(q, e.keys, e.aggs).rows, sql
    assert r.stats.num_docs_scanned == e.stats.num_docs_scanned, sql
    assert r.stats.num_entries_scanned_in_filter == e.stats.num_entries_scanned_in_filter, sql
    if entries is not None:
        assert r.stats.num_entries_scanned_in_filter == entries, sql


def test_range_index_leaf_pinned(ctx):
    tables = [_cols(150_000, 1), _cols(90_001, 2)]
    segs = [ctx.pin(create_segment(f"ri{i}", t, inverted=("s",), range_index=("r", "s"))) for i, t in enumerate(tables)]
    osegs = [O.build_segment(f"ri{i}", t, inverted=("s",), range_index=("r", "s")) for i, t in enumerate(tables)]
    for sql, entries in SQL:
        _check(ctx, segs, osegs, sql, entries)
    # the same column without a range index scans every doc
    plain = [ctx.pin(create_segment(f"np{i}", t)) for i, t in enumerate(tables)]
    r = ctx.execute(parse_sql(SQL[0][0]), plain)
    assert r.stats.num_entries_scanned_in_filter == sum(len(t["r"][0]) for t in tables)


@pytest.mark.parametrize("layout", ["v3", "v1"])
def test_range_index_from_directories(ctx, tmp_path, layout):
    buf = create_segment("ridir", _cols(120_000, 3), inverted=("s",), range_index=("r", "s"))
    path = str(tmp_path / layout)
    (SD.write_v3 if layout == "v3" else SD.write_v1)(buf, path)
    seg = ctx.load_segment_dir(path)
    ora, _ = SD.read_dir(path)
    for sql, entries in SQL:
        if " s " in sql:
            continue  # the directory oracle (segment_dirs.read_dir) models no inverted index
        _check(ctx, [seg], [ora], sql, entries)


LEGACY_SQL = [
    ("SELECT COUNT(*), SUM(m) FROM t WHERE r BETWEEN 100 AND 700", None),
    ("SELECT COUNT(*) FROM t WHERE r > 950", None),                      # upper bound past every range
    ("SELECT COUNT(*), MAX(m) FROM t WHERE r BETWEEN 3 AND 5", None),     # both bounds in one range
    ("SELECT COUNT(*), MIN(m) FROM t WHERE r = 17", None),                # EQ: an inexact index cannot (scan)
    ("SELECT COUNT(*) FROM t WHERE r > 100 AND r < 300", None),          # merged into one RANGE, planned once
    ("SELECT g, COUNT(*), SUM(m) FROM t WHERE r < 400 AND f < 300 GROUP BY g ORDER BY g LIMIT 100", None),
    ("SELECT COUNT(*), SUM(m) FROM t WHERE r < 100 OR f BETWEEN 10 AND 20", None),
    ("SELECT COUNT(*) FROM t WHERE NOT r BETWEEN 200 AND 800", None),
]


@pytest.mark.parametrize("nr", [20, 7])
def test_legacy_range_index(ctx, nr):
    # a legacy version-1 range index (RangeIndexReaderImpl, inexact): RANGE leaves are index-based with the exact
    # doc set, and scan the docs of their boundary ranges (RangeIndexBasedFilterOperator.evaluateLegacyRangeFilter
    # :82-107) -- numEntriesScannedInFilter checked against the oracle's restatement of the reader
    from pinot_amd.segment import legacy_range_index_bytes
    tables = [_cols(60_000, 31), _cols(45_001, 32)]
    segs, osegs = [], []
    for i, t in enumerate(tables):
        buf = create_segment(f"lg{i}", t)
        ids = np.searchsorted(buf.columns["r"].dictionary_values, t["r"][0])
        blob, ranges = legacy_range_index_bytes(ids, nr)
        buf.columns["r"].range_index = blob
        segs.append(ctx.pin(buf))
        osegs.append(O.build_segment(f"lg{i}", t, legacy_ranges={"r": ranges}))
    for sql, entries in LEGACY_SQL:
        _check(ctx, segs, osegs, sql, entries)
    q = parse_sql("SELECT COUNT(*) FROM t WHERE r BETWEEN 100 AND 700")
    r = ctx.execute(q, segs)
    assert 0 < r.stats.num_entries_scanned_in_filter < sum(len(t["r"][0]) for t in tables)


RAW_LEGACY_SQL = [
    "SELECT COUNT(*), SUM(m) FROM t WHERE r BETWEEN {a} AND {b}",
    "SELECT COUNT(*) FROM t WHERE r > {a}",                              # exclusive lower bound: lo + 1 / nextUp
    "SELECT COUNT(*), MIN(m) FROM t WHERE r < {b}",                      # unbounded lower: the type's minimum
    "SELECT COUNT(*) FROM t WHERE r >= {x}",                             # a bound equal to a range start
    "SELECT COUNT(*) FROM t WHERE r > {x}",                              # ... exclusive: the range before it
    "SELECT COUNT(*), MAX(m) FROM t WHERE r > {a} AND r <= {b}",         # merged into one RANGE (raw bounds)
    "SELECT g, COUNT(*), SUM(m) FROM t WHERE r < {b} AND f < 300 GROUP BY g ORDER BY g LIMIT 100",
    "SELECT COUNT(*), SUM(m) FROM t WHERE r < {a} OR f BETWEEN 10 AND 20",
    "SELECT COUNT(*) FROM t WHERE NOT r BETWEEN {a} AND {b}",
    "SELECT COUNT(*) FROM t WHERE r = {x}",                              # EQ: an inexact index cannot (scan)
]


@pytest.mark.parametrize("dtype", ["INT", "LONG", "FLOAT", "DOUBLE"])
def test_legacy_range_index_raw(ctx, dtype):
    # a legacy version-1 index over a raw (no-dictionary) column's values (RangeIndexCreator of the stored type,
    # RangeIndexReaderImpl.findRangeId over typed starts): RANGE leaves are index-based with the exact doc set and
    # scan the docs of the ranges holding the predicate's raw inclusive bounds
    # (RangeIndexBasedFilterOperator.getPartiallyMatchingDocIds :143-166 with the raw evaluators' bounds)
    from pinot_amd.segment import legacy_range_index_bytes
    rng = np.random.default_rng(hash(dtype) % 1000)
    segs, osegs = [], []
    starts = None
    for i, n in enumerate((60_000, 33_331)):
        t = _cols(n, 40 + i)
        v = rng.integers(-5000, 5000, n)
        if dtype == "FLOAT":
            v = (v / 8.0).astype(np.float32)
        elif dtype == "DOUBLE":
            v = v / 16.0
        elif dtype == "LONG":
            v = v.astype(np.int64) * 1_000_000_007
        t["r"] = (v.astype({"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}[dtype]),
                  dtype)
        buf = create_segment(f"lr{i}", t, raw=("r",))
        blob, ranges = legacy_range_index_bytes(t["r"][0], 13 + 4 * i, dtype)
        buf.columns["r"].range_index = blob
        segs.append(ctx.pin(buf))
        osegs.append(O.build_segment(f"lr{i}", t, legacy_raw={"r": ranges}))
        starts = ranges
    lit = (lambda x: repr(float(x))) if dtype in ("FLOAT", "DOUBLE") else (lambda x: str(int(x)))
    vals = np.sort(np.unique(np.concatenate([o.columns["r"].dictionary for o in osegs])))
    a, b, x = vals[len(vals) // 5], vals[3 * len(vals) // 5], starts[len(starts) // 2]
    for sql in RAW_LEGACY_SQL:
        _check(ctx, segs, osegs, sql.format(a=lit(a), b=lit(b), x=lit(x)), None)
    r = ctx.execute(parse_sql(f"SELECT COUNT(*) FROM t WHERE r BETWEEN {lit(a)} AND {lit(b)}"), segs)
    assert 0 < r.stats.num_entries_scanned_in_filter < sum(s.num_docs for s in segs)


SLICE_SQL = [
    "SELECT COUNT(*), SUM(m) FROM t WHERE k BETWEEN 0 AND 1022",        # skewed: array containers
    "SELECT COUNT(*), MIN(m) FROM t WHERE k = 1023",
    "SELECT COUNT(*), MAX(m) FROM t WHERE k < 7",
    "SELECT COUNT(*), SUM(m) FROM t WHERE q BETWEEN 1000 AND 30000",   # nearly sorted: run containers
    "SELECT COUNT(*) FROM t WHERE q >= 49000",
    "SELECT g, COUNT(*), SUM(m) FROM t WHERE q < 20000 AND k > 100 GROUP BY g ORDER BY g LIMIT 100",
    "SELECT g, MAX(m) FROM t WHERE r BETWEEN 0 AND 999 GROUP BY g ORDER BY g LIMIT 100",  # the whole dictionary
    "SELECT COUNT(*) FROM t WHERE r BETWEEN 500 AND 500 OR q < 100",
]


def _slice_cols(n, seed):
    rng = np.random.default_rng(seed)
    c = _cols(n, seed)
    k = np.full(n, 1023, np.int32)
    k[rng.integers(0, n, n // 200)] = rng.integers(0, 1023, n // 200)
    q = np.sort(rng.integers(0, 50_000, n)).astype(np.int32)
    sw = rng.integers(0, n - 1, 50)
    q[sw], q[sw + 1] = q[sw + 1].copy(), q[sw].copy()  # not sorted: no sorted-index leaf
    c["k"], c["q"] = (k, "INT"), (q, "INT")
    return c


@pytest.mark.parametrize("n", [131_072, 200_003, 40_000])
def test_slice_containers_every_kind(ctx, n):
    t = _slice_cols(n, n)
    seg = ctx.pin(create_segment("sl", t, range_index=("r", "k", "q")))
    ora = O.build_segment("sl", t, range_index=("r", "k", "q"))
    for sql in SLICE_SQL:
        _check(ctx, [seg], [ora], sql, None)


def test_leaf_reads_the_slices(ctx):
    # the index says A's r, the forward index holds B's r (same dictionary): a range-index leaf must follow the
    # index (the reference never reads the forward index for it), a scan leaf (IN) the forward index
    a, b = _cols(100_000, 21), _cols(100_000, 22)
    assert np.array_equal(np.unique(a["r"][0]), np.unique(b["r"][0]))
    buf = create_segment("mix", b, range_index=("r",))
    ids_a = np.searchsorted(buf.columns["r"].dictionary_values, a["r"][0])
    buf.columns["r"].range_index = range_index_bytes(ids_a, len(buf.columns["r"].dictionary_values) - 1)
    seg = ctx.pin(buf)
    for lo, hi in [(100, 700), (0, 17), (950, 999), (17, 17)]:
        q = parse_sql(f"SELECT COUNT(*) FROM t WHERE r BETWEEN {lo} AND {hi}")
        r = ctx.execute(q, [seg])
        got = reduce_groups(q, r.keys, r.aggs).rows[0][0]
        assert got == int(((a["r"][0] >= lo) & (a["r"][0] <= hi)).sum()), (lo, hi)
    q = parse_sql("SELECT COUNT(*) FROM t WHERE r IN (3, 5, 9)")
    r = ctx.execute(q, [seg])
    assert reduce_groups(q, r.keys, r.aggs).rows[0][0] == int(np.isin(b["r"][0], [3, 5, 9]).sum())


def test_slices_full_segment(ctx):
    # one 10M-doc segment, cardinality 2^20 (20 slices, 153 keys, a ragged last key): the leaf's count and SUM equal
    # the dictId interval's, for bounds on both sides of every power-of-two boundary tried
    rng = np.random.default_rng(77)
    n = 10_000_000
    r = rng.integers(0, 1 << 20, n).astype(np.int32)
    r[:1 << 20] = np.arange(1 << 20)  # every value present: dictIds == values
    m = rng.integers(0, 1000, n).astype(np.int32)
    seg = ctx.pin(create_segment("big", {"r": (r, "INT"), "m": (m, "INT")}, range_index=("r",)))
    for lo, hi in [(0, (1 << 19) - 1), (1 << 19, (1 << 20) - 2), (12345, 987654), (65535, 65536), (777, 777)]:
        q = parse_sql(f"SELECT COUNT(*), SUM(m) FROM t WHERE r BETWEEN {lo} AND {hi}")
        res = ctx.execute(q, [seg])
        sel = (r >= lo) & (r <= hi)
        assert reduce_groups(q, res.keys, res.aggs).rows[0] == [int(sel.sum()), float(m[sel].sum())], (lo, hi)
        assert res.stats.num_entries_scanned_in_filter == 0
