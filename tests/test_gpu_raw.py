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
                                          ("LZ4_LENGTH_PREFIXED", 4)])
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
