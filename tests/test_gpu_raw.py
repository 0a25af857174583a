"""GPU: raw (no-dictionary) columns against the CPU oracle.

A raw column's results in the reference come from the raw-value operators (raw predicate evaluators,
NoDictionary*GroupKeyGenerator, SUM/MIN/MAX/DISTINCTCOUNTHLL over the values; DefaultGroupByExecutor.java:94-104,
ForwardIndexReaderFactory.java:75-82), which give the same answer as the dictionary path over the same values;
so the oracle runs the same SQL over a dictionary-encoded segment of the same values.  Every stored fixed-width
type, every supported chunk compression, writer versions 2 / 3 / 4, raw and dictionary segments of one column in
one query, and raw columns loaded from V3 / V1 directories.  Bar: bit-exact, DOUBLE SUM within 1e-9 relative."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment
from tests import segment_dirs as SD

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _cols(n, seed):
    rng = np.random.default_rng(seed)
    return {"k": (rng.integers(0, 300, n).astype(np.int64) * 10**10, "LONG"),
            "g": (rng.integers(0, 40, n).astype(np.int32), "INT"),
            "m": (rng.integers(-(1 << 20), 1 << 20, n).astype(np.int32), "INT"),
            "d": (np.round(rng.normal(0, 50, n), 3) + 0.0, "DOUBLE"),  # + 0.0: no -0.0 (Double.compare ties)
            "f": (rng.integers(-500, 500, n).astype(np.float32) / 4, "FLOAT"),
            "u": (rng.integers(0, 1 << 24, n).astype(np.int32), "INT")}


SQL = ["SELECT k, COUNT(*), SUM(m), MIN(d), MAX(f) FROM t WHERE m > 0 GROUP BY k ORDER BY k LIMIT 1000",
       "SELECT g, k, SUM(d), MAX(m) FROM t WHERE f BETWEEN -50 AND 60.5 AND k <> 30000000000 "
       "GROUP BY g, k ORDER BY g, k LIMIT 100000",
       "SELECT COUNT(*), SUM(m), MIN(m), MAX(d), SUM(f) FROM t WHERE k IN (0, 10000000000, 990000000000)",
       "SELECT DISTINCTCOUNTHLL(u), DISTINCTCOUNTHLL(k) FROM t WHERE d < 10",
       "SELECT COUNT(*) FROM t WHERE d >= 0 AND f < 0",
       "SELECT g, SUM(m * f), SUM(k - m) FROM t WHERE g < 20 GROUP BY g ORDER BY g LIMIT 100"]


def _check(ctx, segs, osegs, sql):
    q = parse_sql(sql)
    r = ctx.execute(q, segs)
    e = O.execute(q, osegs)
    got, exp = reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, e.keys, e.aggs).rows
    assert len(got) == len(exp), sql
    for g, x in zip(got, exp):
        for a, b in zip(g, x):
            assert a == b or (isinstance(b, float) and abs(a - b) <= 1e-9 * abs(b)), (sql, g, x)
    for k, a in enumerate(q.aggregations):  # HLL registers raw
        if a.function == "DISTINCTCOUNTHLL":
            assert all(np.array_equal(x[k], y[k]) for x, y in zip(r.aggs, e.aggs)), sql


@pytest.mark.parametrize("comp,version", [("PASS_THROUGH", 2), ("LZ4", 3), ("SNAPPY", 2),
                                          ("LZ4_LENGTH_PREFIXED", 4), ("ZSTANDARD", 3)])
def test_raw_columns_match_oracle(ctx, comp, version):
    cols = _cols(200_003, 11)
    seg = ctx.pin(create_segment("raw0", cols, raw=("k", "m", "d", "f", "u"), raw_compression=comp,
                                 raw_version=version))
    ora = O.build_segment("raw0", cols)
    for sql in SQL:
        _check(ctx, [seg], [ora], sql)


def test_raw_and_dictionary_segments_together(ctx):
    # one table, the same columns raw in some segments and dictionary-encoded in others
    parts = [_cols(120_000, 20 + i) for i in range(3)]
    segs = [ctx.pin(create_segment(f"mix{i}", c, raw=("k", "d") if i != 1 else (), raw_compression="LZ4"))
            for i, c in enumerate(parts)]
    osegs = [O.build_segment(f"mix{i}", c) for i, c in enumerate(parts)]
    for sql in SQL:
        _check(ctx, segs, osegs, sql)


@pytest.mark.parametrize("layout", ["v3", "v1"])
def test_raw_columns_from_directories(ctx, tmp_path, layout):
    cols = _cols(150_000, 5)
    buf = create_segment("rawdir", cols, raw=("m", "d", "k"), raw_compression="SNAPPY")
    path = str(tmp_path / layout)
    (SD.write_v3 if layout == "v3" else SD.write_v1)(buf, path)
    seg = ctx.load_segment_dir(path)
    ora, _ = SD.read_dir(path)
    for sql in SQL:
        _check(ctx, [seg], [ora], sql)


def test_raw_real_predicates_primitive_semantics(ctx):
    # raw FLOAT / DOUBLE predicates compare primitives (EqualsPredicateEvaluatorFactory / RangePredicateEvaluatorFactory
    # raw-value evaluators, RangePredicateEvaluatorFactory.java:482-522): 0 matches -0.0 and 0.0, NaN matches no EQ /
    # IN / RANGE (not even an unbounded one) and every NOT_EQ / NOT_IN.  The pinned column is dictionary-encoded in
    # Double.compare order (-0.0 < 0.0, NaN last), so the planner must not map these to plain dictId ranges
    # (ADVICE r2).  Expected counts / sums from numpy's IEEE comparisons, which are the primitive semantics.
    rng = np.random.default_rng(404)
    n = 100_003
    d = np.round(rng.normal(0, 4, n), 1)
    d[rng.integers(0, n, 3000)] = -0.0
    d[rng.integers(0, n, 3000)] = 0.0
    d[rng.integers(0, n, 500)] = np.nan
    f = d.astype(np.float32)
    m = rng.integers(-1000, 1000, n).astype(np.int32)
    cols = {"d": (d, "DOUBLE"), "f": (f, "FLOAT"), "m": (m, "INT")}
    seg = ctx.pin(create_segment("rawnan", cols, raw=("d", "f"), raw_compression="LZ4"))
    cases = {
        "d = 0": d == 0, "d = -0.0": d == 0, "d <> 0": ~(d == 0), "d IN (0, 1.5)": (d == 0) | (d == 1.5),
        "d NOT IN (0, 1.5)": ~((d == 0) | (d == 1.5)), "d > 1": d > 1, "d >= 0": d >= 0, "d < 0": d < 0,
        "d <= 0": d <= 0, "d BETWEEN -1 AND 0": (d >= -1) & (d <= 0), "d = 'NaN'": np.zeros(n, bool), "d <> 'NaN'": np.ones(n, bool),
        "f = 0": f == 0, "f > -0.5": f > np.float32(-0.5), "f < 0.3": f < np.float32(0.3), "f <> 0": ~(f == 0),
    }
    for where, mask in cases.items():
        q = parse_sql(f"SELECT COUNT(*), SUM(m) FROM t WHERE {where}")
        r = ctx.execute(q, [seg])
        got = reduce_groups(q, r.keys, r.aggs).rows
        cnt = int(np.count_nonzero(mask))
        exp_sum = float(m[mask].astype(np.int64).sum()) if cnt else None
        assert got[0][0] == cnt, (where, got, cnt)
        if cnt:
            assert got[0][1] == exp_sum, (where, got, exp_sum)
    seg.unpin()
