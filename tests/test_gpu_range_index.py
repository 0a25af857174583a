"""GPU: range-indexed columns (FilterOperatorUtils.java:97-120, RangeIndexBasedFilterOperator,
BitSlicedRangeIndexReader).  A column with an exact (version 2) bit-sliced range index turns RANGE -- and EQ when the
column has no inverted index -- into an index-based leaf: no entries scanned in filter, bitmap-based in the AND
order; RANGE never uses an inverted index.  The kernels evaluate the leaf from the packed dictIds (the same doc set
as the exact index).  Checked against the oracle's leaf choice on pinned buffers and on V3 / V1 directories whose
index_map / <col>.bitmap.range carry the index (the fixture writes the BitSlicedRangeIndexCreator header; the GPU
path reads no bit slice).  Bar: bit-exact results and identical ExecutionStatistics."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment
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


def test_inexact_range_index_takes_the_cpu_plan(ctx):
    # a legacy version-1 range index (ranges + a partial scan of the boundary ranges) is still a
    # RangeIndexBasedFilterOperator leaf in the reference (RangeIndexBasedFilterOperator.java:59-60), whose entries
    # the GPU statistics do not model: its RANGE / EQ leaves are PH_ERR_UNSUPPORTED (the plan maker's CPU fallback);
    # other predicates on the column still run on the GPU
    from pinot_amd import native as N
    buf = create_segment("riv1", _cols(20_000, 9), range_index=("r",))
    hdr = buf.columns["r"].range_index.copy()
    hdr[:4] = np.frombuffer(np.array([1], ">i4").tobytes(), np.uint8)  # version 1
    buf.columns["r"].range_index = hdr
    seg = ctx.pin(buf)
    with pytest.raises(N.UnsupportedError):
        ctx.execute(parse_sql("SELECT COUNT(*) FROM t WHERE r BETWEEN 100 AND 700"), [seg])
    r = ctx.execute(parse_sql("SELECT COUNT(*) FROM t WHERE r IN (3, 5, 9)"), [seg])
    assert r.stats.num_entries_scanned_in_filter == 20_000
