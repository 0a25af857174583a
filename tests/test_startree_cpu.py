"""CPU: the star-tree index (SURVEY 8(f) row f4's star-tree leaf).  The oracle's parse is pinned by the reference's own
star-tree (pinot-segment-local/src/test/resources/data/startree/segment: star_tree_index, star_tree_index_map,
metadata.properties, committed under tests/golden/startree_segment/): its node count, split order and aggregated
documents agree with the segment's metadata (totalDocs, ArrDelay's maxValue) and with the records under every node.
The builder (pinot_amd.startree, a restatement of BaseSingleTreeBuilder / OnHeapSingleTreeBuilder) writes trees with
the same invariants, the library's host parse (ph_star_tree_check) reads both, and the oracle's star-tree execution
(StarTreeFilterOperator traversal + pair-column aggregation) equals its raw execution on random queries."""
import ctypes
import os

import numpy as np
import pytest

from oracle import oracle as O
from oracle import startree as S
from pinot_amd import native as N
from pinot_amd.query import parse_sql
from pinot_amd.segment import create_segment, read_raw_forward_index
from pinot_amd.startree import build_star_tree

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "startree_segment")


def _props(path):
    out = {}
    for line in open(path, encoding="utf-8"):
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        out.setdefault(k.strip(), []).append(v.strip())
    return out


def _reference():
    meta = _props(os.path.join(GOLD, "metadata.properties"))
    imap = {k: int(v[0]) for k, v in _props(os.path.join(GOLD, "star_tree_index_map")).items()}
    blob = np.fromfile(os.path.join(GOLD, "star_tree_index"), np.uint8)

    def buf(col, idx):
        o, n = imap[f"0.{col}.{idx}.OFFSET"], imap[f"0.{col}.{idx}.SIZE"]
        return blob[o:o + n]
    return meta, buf


def _check_tree_invariants(t, count):
    nodes = t.nodes
    n = len(nodes)
    first_star = min(int(x[2]) for x in nodes if x[1] == S.ALL and x[0] >= 0)
    for i in range(n):
        d, v, s, e, agg, fc, lc = (int(x) for x in nodes[i])
        if fc != -1:
            kids = nodes[fc:lc + 1]
            assert (kids[:, 0] == d + 1).all()
            assert (np.diff(kids[:, 1]) > 0).all()  # sorted by value, the star node (-1) first
            if kids[0, 1] == S.ALL:
                assert agg == int(kids[0, 4])  # a node with a star child shares its aggregated document
        if i == 0:
            s, e = 0, first_star  # the root covers every raw (segment-aggregated) record
        if v != S.ALL:
            assert count[agg] == count[s:e].sum(), i


def test_reference_star_tree_parses():
    meta, buf = _reference()
    tree = buf("null", "STAR_TREE")
    t = S.parse_tree(tree.tobytes())
    assert t.dimensions == meta["startree.v2.0.split.order"]
    nd = int(meta["startree.v2.0.total.docs"][0])
    count = read_raw_forward_index(buf("count__*", "FORWARD_INDEX"), "LONG", nd)
    mx = read_raw_forward_index(buf("max__ArrDelay", "FORWARD_INDEX"), "DOUBLE", nd)
    root_agg = int(t.nodes[0, 4])
    assert count[root_agg] == int(meta["segment.total.docs"][0]) == 313
    assert mx[root_agg] == float(meta["column.ArrDelay.maxValue"][0]) == 343.0
    _check_tree_invariants(t, count)
    # the dimensions' forward indexes are fixed-bit at the segment columns' widths, values inside the dictionaries
    for d in t.dimensions:
        bits = int(meta[f"column.{d}.bitsPerElement"][0])
        card = int(meta[f"column.{d}.cardinality"][0])
        fwd = buf(d, "FORWARD_INDEX")
        assert fwd.nbytes == (nd * bits + 7) // 8
        ids = O.fixed_bit_unpack(fwd, nd, bits)
        assert ids.max() < card
    # the library's host parse agrees
    nn, ndim = ctypes.c_int32(), ctypes.c_int32()
    N.check(N.lib().ph_star_tree_check(tree.ctypes.data, tree.nbytes, ctypes.byref(nn), ctypes.byref(ndim)))
    assert (nn.value, ndim.value) == (len(t.nodes), 3) == (666, 3)
    bad = tree.copy()
    bad[0] ^= 1
    assert N.lib().ph_star_tree_check(bad.ctypes.data, bad.nbytes, None, None) == N.PH_ERR_INVALID_ARGUMENT
    assert N.lib().ph_star_tree_check(tree.ctypes.data, tree.nbytes - 28, None, None) == N.PH_ERR_INVALID_ARGUMENT


def star_table(rng, n):
    return {
        "d1": (rng.integers(0, 6, n).astype(np.int32) * 10, "INT"),
        "d2": (rng.choice(np.array(["ca", "ny", "tx", "wa", "or", "fl", "il", "ga"]), n), "STRING"),
        "d3": (rng.integers(0, 40, n).astype(np.int64) * 1000 + 7, "LONG"),
        "m": (rng.integers(-500, 5000, n).astype(np.int32), "INT"),
        "x": (np.round(rng.normal(10, 50, n), 2), "DOUBLE"),
        "z": (rng.integers(0, 9, n).astype(np.int32), "INT"),
    }


PAIRS = [("count", "*"), ("sum", "m"), ("min", "m"), ("max", "m"), ("max", "x"), ("sum", "x")]


def make_star(cols, name="st", max_leaf=10, dims=("d1", "d2", "d3"), skip=()):
    seg = create_segment(name, cols)
    st = build_star_tree(seg, list(dims), PAIRS, max_leaf, skip, values={c: v for c, (v, _) in cols.items()})
    oseg = O.build_segment(name, cols)
    bits = {d: seg.columns[d].bits for d in dims}
    osd = S.from_buffers(st.tree.tobytes(), st.num_docs, st.dim_fwd, bits, st.metrics)
    return seg, st, oseg, osd


STAR_QUERIES = [
    "SELECT COUNT(*), SUM(m) FROM t",
    "SELECT d1, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t GROUP BY d1",
    "SELECT d3, COUNT(*), MAX(x) FROM t WHERE d2 = 'ny' GROUP BY d3",
    "SELECT d2, SUM(m), SUM(x) FROM t WHERE d1 IN (10, 30, 50) AND d3 BETWEEN 5007 AND 31007 GROUP BY d2",
    "SELECT d1, d2, COUNT(*), MIN(m) FROM t WHERE (d3 = 7 OR d3 = 12007 OR d3 > 36000) AND d2 <> 'tx' GROUP BY d1, d2",
    "SELECT COUNT(*), MAX(m), MIN(m) FROM t WHERE d3 > 20000 AND d3 < 30000",
    "SELECT d3, COUNT(*) FROM t WHERE d1 NOT IN (0, 20) AND d2 IN ('ca', 'wa') GROUP BY d3",
    "SELECT COUNT(*) FROM t WHERE d2 = 'zz'",
    "SELECT d1, COUNT(*) FROM t WHERE d1 = 40 AND d1 > 10 GROUP BY d1",
    "SELECT SUM(m) FROM t WHERE d3 = 39007",
]


def _rows(keys, aggs):
    return sorted((tuple(k), tuple(a)) for k, a in zip(keys, aggs))


@pytest.mark.parametrize("max_leaf", [1, 10, 200])
def test_builder_tree_invariants(max_leaf):
    rng = np.random.default_rng(61 + max_leaf)
    cols = star_table(rng, 3000)
    seg, st, oseg, osd = make_star(cols, max_leaf=max_leaf)
    t = S.parse_tree(st.tree.tobytes())
    assert t.dimensions == ["d1", "d2", "d3"]
    _check_tree_invariants(t, st.metrics["count__*"])
    assert st.metrics["count__*"][int(t.nodes[0, 4])] == 3000
    nn = ctypes.c_int32()
    N.check(N.lib().ph_star_tree_check(st.tree.ctypes.data, st.tree.nbytes, ctypes.byref(nn), None))
    assert nn.value == len(t.nodes)
    # the pair columns read back through the raw-forward-index reader
    assert np.array_equal(read_raw_forward_index(st.metric_fwd["sum__m"], "DOUBLE", st.num_docs), st.metrics["sum__m"])


@pytest.mark.parametrize("sql", STAR_QUERIES)
@pytest.mark.parametrize("max_leaf", [3, 40])
def test_oracle_star_tree_equals_raw(sql, max_leaf):
    rng = np.random.default_rng(len(sql) * 7 + max_leaf)
    cols = star_table(rng, 4000)
    _, _, oseg, osd = make_star(cols, max_leaf=max_leaf)
    q = parse_sql(sql)
    keys, aggs, stats, served = S.execute_with_star_trees(q, [(oseg, osd)])
    r = O.execute(q, [oseg])
    assert served == (0 if sql == "SELECT COUNT(*) FROM t WHERE d2 = 'zz'" else 1)
    got, exp = _rows(keys, aggs), _rows(r.keys, r.aggs)
    assert len(got) == len(exp)
    for (gk, ga), (ek, ea) in zip(got, exp):
        assert gk == ek
        for a, b in zip(ga, ea):
            assert a == pytest.approx(b, rel=1e-9, abs=1e-6)
    assert stats["num_total_docs"] == 4000
    assert stats["num_docs_scanned"] <= r.stats.num_docs_scanned


def test_star_tree_not_fit():
    rng = np.random.default_rng(5)
    cols = star_table(rng, 2000)
    _, _, oseg, osd = make_star(cols)
    for sql in ["SELECT z, COUNT(*) FROM t GROUP BY z",           # group-by column not a dimension
                "SELECT SUM(z) FROM t WHERE d1 = 10",              # no sum__z pair
                "SELECT COUNT(*) FROM t WHERE NOT d1 = 10",        # NOT is not solved by the star-tree
                "SELECT COUNT(*) FROM t WHERE d1 = 10 OR d2 = 'ca'",  # an OR over two columns
                "SELECT SET_SKIP FROM t",
                "SELECT MAX(m) FROM t"]:                           # metadata plan first
        if sql == "SELECT SET_SKIP FROM t":
            q = parse_sql("SET skipStarTree=true; SELECT d1, COUNT(*) FROM t GROUP BY d1")
        else:
            q = parse_sql(sql)
        assert S.fit(q, oseg, osd) is None or sql == "SELECT MAX(m) FROM t"
        _, _, _, served = S.execute_with_star_trees(q, [(oseg, osd)])
        assert served == 0, sql


def test_raw_inclusive_bounds():
    # RangePredicateEvaluatorFactory's raw evaluators (:70-92, :314-499): unbounded = inclusive type min / max, an
    # exclusive bound moved by one (INT wraps) or by Math.nextUp / nextDown in the column's own precision
    from pinot_amd.query import parse_sql as P
    def b(where, t):
        return O.raw_inclusive_bounds(P("SELECT COUNT(*) FROM t WHERE " + where).filter.predicate, t)
    assert b("r > 5", "INT") == (6, 2 ** 31 - 1)
    assert b("r <= 5", "LONG") == (-2 ** 63, 5)
    assert b("r < -2147483648", "INT") == (-2 ** 31, 2 ** 31 - 1)  # (-2^31) - 1 wraps, as Java int arithmetic
    lo, hi = b("r > 1.5", "FLOAT")
    assert lo == float(np.nextafter(np.float32(1.5), np.float32(np.inf))) and hi == np.inf
    lo, hi = b("r BETWEEN 0.1 AND 0.2", "DOUBLE")
    assert (lo, hi) == (0.1, 0.2)
