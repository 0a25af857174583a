"""GPU: segment group trim (GroupByOperator.java:114-130) -- ORDER BY + minSegmentGroupTrimSize > 0: each segment keeps
max(5 * limit, minSegmentGroupTrimSize) groups (GroupByUtils.getTableCapacity) chosen by TableResizer's heap over the
ORDER BY values in the group-key iterator's order, before the combine merges the segments' partial aggregates.  The
library runs each segment as its own query, trims on the host (trim.cpp) and merges; the oracle trims the same way
(oracle.py _segment_trim).  Key spaces of <= 10 000 groups are the reference's ArrayBasedHolder (raw-key order, ties at
the boundary resolved exactly); the larger one is ordered by a tie-free SUM.  Bar: bit-exact rows and statistics."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment
from tests.seeds import seed_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _tables(name, n_list, acard, bcard):
    rng = np.random.default_rng(seed_of(name))
    out = []
    for n in n_list:
        a = rng.zipf(1.6, n) % acard  # skewed: a few heavy groups, many light ones (ties in COUNT)
        out.append({"a": (a.astype(np.int32), "INT"), "b": (rng.integers(0, bcard, n).astype(np.int32), "INT"),
                    "m": (rng.integers(-50, 1 << 24, n).astype(np.int32), "INT"),
                    "f": (rng.integers(0, 100, n).astype(np.int32), "INT"),
                    "d": (np.round(rng.normal(0, 10, n), 3), "DOUBLE")})
    return out


SMALL = [  # a x b = 50 x 40 groups: ArrayBasedHolder
    "SET minSegmentGroupTrimSize=40; SELECT a, b, COUNT(*) FROM t GROUP BY a, b ORDER BY COUNT(*) DESC LIMIT 5",
    "SET minSegmentGroupTrimSize=30; SELECT a, b, SUM(m), COUNT(*) FROM t WHERE f < 70 GROUP BY a, b "
    "ORDER BY SUM(m) DESC LIMIT 4",
    "SET minSegmentGroupTrimSize=25; SELECT a, b, MAX(m), MIN(d) FROM t GROUP BY a, b ORDER BY b DESC, a LIMIT 3",
    "SET minSegmentGroupTrimSize=30; SELECT a, COUNT(*), SUM(d) FROM t GROUP BY a ORDER BY COUNT(*), a DESC LIMIT 6",
    "SET minSegmentGroupTrimSize=100000; SELECT a, b, COUNT(*) FROM t GROUP BY a, b ORDER BY COUNT(*) DESC LIMIT 5",
    # extractFinalResult order (TableResizer.java:425-447): HyperLogLog.cardinality() of each group's registers
    "SET minSegmentGroupTrimSize=30; SELECT a, b, DISTINCTCOUNTHLL(m), COUNT(*) FROM t GROUP BY a, b "
    "ORDER BY DISTINCTCOUNTHLL(m) DESC, a LIMIT 5",
    "SET minSegmentGroupTrimSize=20; SELECT a, DISTINCTCOUNTHLL(f, 6), SUM(m) FROM t GROUP BY a "
    "ORDER BY DISTINCTCOUNTHLL(f, 6), a DESC LIMIT 4",
]


def _check(ctx, segs, osegs, sql):
    q = parse_sql(sql)
    r = ctx.execute(q, segs)
    e = O.execute(q, osegs)
    got, exp = reduce_groups(q, r.keys, r.aggs).rows, reduce_groups(q, e.keys, e.aggs).rows
    assert len(got) == len(exp), sql
    for g, x in zip(got, exp):
        for a, b in zip(g, x):
            assert a == b or (isinstance(b, float) and abs(a - b) <= 1e-9 * abs(b)), (sql, g, x)
    assert r.num_groups == len(e.keys), sql  # the merged table after the trims holds the same groups
    assert r.stats.num_docs_scanned == e.stats.num_docs_scanned
    return r, e


@pytest.mark.parametrize("sql", SMALL)
def test_segment_trim_array_based(ctx, sql):
    tables = _tables("trim-small", (60_000, 45_001, 30_017), 50, 40)
    segs = [ctx.pin(create_segment(f"tr{i}", t)) for i, t in enumerate(tables)]
    osegs = [O.build_segment(f"tr{i}", t) for i, t in enumerate(tables)]
    r, e = _check(ctx, segs, osegs, sql)
    untrimmed = ctx.execute(parse_sql(sql.replace("minSegmentGroupTrimSize", "minServerGroupTrimSize")), segs)
    if "100000" not in sql:
        assert r.num_groups < untrimmed.num_groups  # the trim dropped groups (their partial aggregates too)


def test_segment_trim_large_key_space(ctx):
    # 300 x 300 groups (> 10 000: the reference iterates a hash map) ordered by a tie-free SUM
    tables = _tables("trim-large", (200_000, 150_001), 300, 300)
    segs = [ctx.pin(create_segment(f"tl{i}", t)) for i, t in enumerate(tables)]
    osegs = [O.build_segment(f"tl{i}", t) for i, t in enumerate(tables)]
    _check(ctx, segs, osegs, "SET minSegmentGroupTrimSize=500; SELECT a, b, SUM(m), COUNT(*) FROM t GROUP BY a, b "
                             "ORDER BY SUM(m) DESC LIMIT 10")


def test_segment_trim_string_keys_of_differing_widths(ctx):
    # no table dictionary: each segment's own query pads its STRING keys to that segment's max_string_len, so the
    # merge must key on the unpadded values (the same string from two segments is ONE group) and the output must
    # take the widest width; ORDER BY the string column itself and a two-column key exercise the comparator offsets
    rng = np.random.default_rng(seed_of("trim-strings"))
    words = [["s%d" % i for i in range(40)],                                  # width 3
             ["s%d" % i for i in range(20, 60)] + ["long-%02d-" % i + "x" * i for i in range(30)],  # width up to 38
             ["s%d" % i for i in range(0, 60, 3)]]
    tables = []
    for w, n in zip(words, (40_000, 35_003, 20_011)):
        s = np.array(w, dtype=object)[rng.integers(0, len(w), n)]
        tables.append({"s": (s, "STRING"), "b": (rng.integers(0, 7, n).astype(np.int32), "INT"),
                       "m": (rng.integers(0, 1 << 20, n).astype(np.int32), "INT")})
    segs = [ctx.pin(create_segment(f"ts{i}", t)) for i, t in enumerate(tables)]
    osegs = [O.build_segment(f"ts{i}", t) for i, t in enumerate(tables)]
    for sql in ("SET minSegmentGroupTrimSize=12; SELECT s, COUNT(*), SUM(m) FROM t GROUP BY s ORDER BY s DESC LIMIT 3",
                "SET minSegmentGroupTrimSize=15; SELECT b, s, MAX(m) FROM t GROUP BY b, s ORDER BY s, b DESC LIMIT 4",
                "SET minSegmentGroupTrimSize=20; SELECT s, b, SUM(m) FROM t GROUP BY s, b ORDER BY SUM(m) DESC LIMIT 5"):
        r, _ = _check(ctx, segs, osegs, sql)
        assert len(r.keys) == len(set(r.keys)), sql  # no group twice
