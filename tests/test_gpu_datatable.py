"""GPU: server -> broker DataTable V4 (ph_result_datatable) decoded and merged the broker's way
(pinot_amd.datatable: DataTableImplV4(ByteBuffer) + GroupByDataTableReducer / AggregationDataTableReducer) against
the oracle over all segments.  Segments are split over 3 "servers" (one DataTable each), so keys repeat across
tables and the broker merge (COUNT / SUM add, MIN / MAX, HLL register max) is exercised; STRING keys go through the
DataTable string dictionary, HLL through the OBJECT column.  Bar: bit-exact, DOUBLE SUM within 1e-9 relative."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd import datatable as DT
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    from pinot_amd.engine import GpuContext
    ctx = GpuContext(0)
    rng = np.random.default_rng(99)
    parts, segs, osegs = [], [], []
    for i in range(6):
        n = 50_000 + 1000 * i
        cols = {"g": (rng.integers(0, 30, n).astype(np.int32), "INT"),
                "s": (np.array(["red", "green", "blue", "", "teal"])[rng.integers(0, 5, n)], "STRING"),
                "l": (rng.integers(0, 7, n).astype(np.int64) * 10**11, "LONG"),
                "m": (rng.integers(0, 1 << 20, n).astype(np.int32), "INT"),
                "d": (np.round(rng.normal(0, 10, n), 2) + 0.0, "DOUBLE")}
        segs.append(ctx.pin(create_segment(f"dt{i}", cols)))
        osegs.append(O.build_segment(f"dt{i}", cols))
    yield ctx, segs, osegs
    ctx.close()


SQL = ["SELECT g, s, COUNT(*), SUM(m), MIN(d), MAX(l), DISTINCTCOUNTHLL(m) FROM t WHERE d > -5 "
       "GROUP BY g, s ORDER BY g, s LIMIT 1000",
       "SELECT s, SUM(d), COUNT(*) FROM t GROUP BY s ORDER BY SUM(d) DESC LIMIT 3",
       "SELECT COUNT(*), SUM(m), MIN(m), MAX(d), DISTINCTCOUNTHLL(l) FROM t WHERE s IN ('red', 'teal')",
       "SELECT COUNT(*), SUM(m) FROM t WHERE m < 0",
       "SELECT g, SUM(m * d) FROM t WHERE g < 5 GROUP BY g ORDER BY g LIMIT 10"]


@pytest.mark.parametrize("sql", SQL)
def test_datatable_broker_reduce(setup, sql):
    ctx, segs, osegs = setup
    q = parse_sql(sql)
    servers = [segs[0:2], segs[2:5], segs[5:]]
    tables = [DT.decode(ctx.execute_datatable(q, part, {"numSegmentsQueried": len(part), "requestId": 7}))
              for part in servers]
    got = DT.reduce_datatables(q, tables).rows
    e = O.execute(q, osegs)
    exp = reduce_groups(q, e.keys, e.aggs).rows
    assert len(got) == len(exp)
    for g, x in zip(got, exp):
        for a, b in zip(g, x):
            assert a == b or (isinstance(b, float) and abs(a - b) <= 1e-9 * abs(b)), (sql, g, x)
    # schema and metadata as the reference's server writes them
    t = tables[1]
    nk = len(q.group_by)
    assert t.column_names[:nk] == q.group_by
    ops = {"*": "times", "-": "minus", "+": "plus"}
    for name, a in zip(t.column_names[nk:], q.aggregations):  # AggregationFunction.getResultColumnName()
        arg = a.column if a.op is None else f"{ops[a.op]}({a.column},{a.column2})"
        assert name == ("count(*)" if a.function == "COUNT" else f"{a.function.lower()}({arg})")
    # the Python broker's result columns carry the same names as the DataTable schema
    names = {a.result_name() for a in q.aggregations}
    assert set(t.column_names[nk:]) == names, (t.column_names, names)
    assert t.column_types[nk:] == [{"COUNT": "LONG", "DISTINCTCOUNTHLL": "OBJECT"}.get(a.function, "DOUBLE")
                                   for a in q.aggregations]
    r = ctx.execute(q, servers[1])
    md = t.metadata
    assert int(md["numDocsScanned"]) == r.stats.num_docs_scanned
    assert int(md["totalDocs"]) == r.stats.num_total_docs
    assert int(md["numEntriesScannedPostFilter"]) == r.stats.num_entries_scanned_post_filter
    assert md["numSegmentsQueried"] == "3" and md["requestId"] == "7"
    assert ("numResizes" in md) == bool(nk)


def test_hll_object_round_trip(setup):
    ctx, segs, _ = setup
    q = parse_sql("SELECT DISTINCTCOUNTHLL(m) FROM t")
    t = DT.decode(ctx.execute_datatable(q, segs))
    otype, payload = t.rows[0][0]
    assert otype == DT.HLL_OBJECT_TYPE
    log2m, regs = DT.hll_deserialize(payload)
    r = ctx.execute(q, segs)
    assert log2m == 8 and np.array_equal(regs, r.aggs[0][0])
