"""GPU: the segment-level drop-in (SURVEY 8(b) plug point 2) -- ph_filter_execute, what a GpuFilterOperator extends
BaseFilterOperator returns from FilterPlanNode.run (FilterPlanNode.java:83-114): the segment's doc bitmap
(BitmapDocIdSet, BitmapDocIdSet.java:29), its matching count (canOptimizeCount / getNumMatchingDocs,
BaseFilterOperator.java:59-68) and the statistic of the reference's iterator tree
(BlockDocIdSet.getNumEntriesScannedInFilter).  Checked through the C-ABI against the oracle's doc set
(oracle.filter_docs: the planned tree evaluated per doc) and oracle.filter_entries, on fixed shapes, random filter
trees, every leaf kind (scan, sorted, inverted, range-index slices, legacy paths) and ragged segment sizes.
Bar: bit-exact words, count and statistic."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.segment import create_segment
from tests import kat_sv
from tests.seeds import seed_of
from tests.test_gpu_parity import FILTERS, _random_table

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _check(ctx, seg, oseg, where, words=True):
    q = parse_sql("SELECT COUNT(*) FROM t" + where)
    got, cnt, st = ctx.filter(q, seg, words=words)
    mask, entries = O.filter_docs(q, oseg)
    assert cnt == int(mask.sum()), where
    if words:
        exp = O.doc_words(mask)
        assert got.shape == exp.shape
        bad = np.nonzero(got != exp)[0]
        assert bad.size == 0, (where, bad[:5], got[bad[:5]], exp[bad[:5]])
    assert st.num_entries_scanned_in_filter == entries, (where, st.num_entries_scanned_in_filter, entries)
    assert st.num_total_docs == oseg.num_docs
    return got, cnt, st


def test_kat_filter_segment(ctx):
    # InterSegmentAggregationSingleValueQueriesTest: 24516 docs and 252256 entries over 4 copies of the segment
    cols = kat_sv.load_columns()
    seg = ctx.pin(create_segment("kat", cols, inverted=kat_sv.INVERTED))
    words, cnt, st = ctx.filter(parse_sql("SELECT COUNT(*) FROM testTable" + kat_sv.FILTER), seg)
    assert cnt * 4 == 24516
    assert st.num_entries_scanned_in_filter * 4 == 252256
    assert int(np.unpackbits(words.view(np.uint8)).sum()) == cnt
    oseg = O.build_segment("kat", cols, inverted=kat_sv.INVERTED)
    _check(ctx, seg, oseg, kat_sv.FILTER.replace("testTable", "t"))


@pytest.mark.parametrize("where", FILTERS)
@pytest.mark.parametrize("n", [20_000, 777, 64 * 300 + 1])
def test_filter_shapes(ctx, where, n):
    rng = np.random.default_rng(seed_of(where) + n)
    t = _random_table(rng, n)
    seg = ctx.pin(create_segment("f", t, inverted=("a", "str")))
    oseg = O.build_segment("f", t, inverted=("a", "str"))
    _check(ctx, seg, oseg, where)
    _check(ctx, seg, oseg, where, words=False)  # canOptimizeCount: the count alone


def _random_where(rng, depth=0):
    leaves = [
        lambda: f"a = {rng.integers(0, 8)}",
        lambda: f"a IN ({rng.integers(0, 7)}, {rng.integers(0, 7)})",
        lambda: f"a NOT IN ({rng.integers(0, 7)})",
        lambda: f"b BETWEEN {rng.integers(-4000, 0)} AND {rng.integers(0, 4000)}",
        lambda: f"b > {rng.integers(-4000, 4000)}",
        lambda: f"m < {rng.integers(0, 1 << 30)}",
        lambda: f"s BETWEEN {rng.integers(0, 20)} AND {rng.integers(20, 41)}",
        lambda: f"s <> {rng.integers(0, 40)}",
        lambda: f"str = '{['P', 'gFuH', 'o', 't'][rng.integers(0, 4)]}'",
        lambda: f"str NOT IN ('t', 'zz')",
        lambda: f"c < {int(rng.integers(0, 5000)) * 1_000_003}",
    ]
    if depth >= 3 or rng.random() < 0.35:
        return leaves[rng.integers(0, len(leaves))]()
    op = ["AND", "OR", "NOT"][rng.integers(0, 3)]
    if op == "NOT":
        return f"NOT ({_random_where(rng, depth + 1)})"
    k = int(rng.integers(2, 4))
    return "(" + f" {op} ".join(_random_where(rng, depth + 1) for _ in range(k)) + ")"


@pytest.mark.parametrize("trial", range(24))
def test_random_filter_trees(ctx, trial):
    rng = np.random.default_rng(1000 + trial)
    n = int(rng.integers(1, 60_000))
    t = _random_table(rng, n)
    seg = ctx.pin(create_segment("r", t, inverted=("a", "str")))
    oseg = O.build_segment("r", t, inverted=("a", "str"))
    for _ in range(4):
        _check(ctx, seg, oseg, " WHERE " + _random_where(rng))


def test_no_filter_matches_all(ctx):
    rng = np.random.default_rng(5)
    t = _random_table(rng, 1000)
    seg = ctx.pin(create_segment("all", t))
    words, cnt, st = ctx.filter(parse_sql("SELECT COUNT(*) FROM t"), seg)
    assert cnt == 1000 and st.num_entries_scanned_in_filter == 0
    assert np.array_equal(words, O.doc_words(np.ones(1000, bool)))


def _ri_cols(n, seed):
    rng = np.random.default_rng(seed)
    return {"r": (rng.integers(0, 1000, n).astype(np.int32), "INT"), "s": (rng.integers(0, 60, n).astype(np.int32), "INT"),
            "f": (rng.integers(0, 1000, n).astype(np.int32), "INT")}


RANGE_WHERE = [
    " WHERE r BETWEEN 100 AND 700",
    " WHERE r = 17",
    " WHERE r > 950 AND s = 5",                          # a slice leaf beside an inverted leaf
    " WHERE r < 400 AND f < 300",
    " WHERE r >= 300 AND r < 200",                       # merged range leaves: an empty interval
    " WHERE r >= 300 AND r <= 450 AND f > 10",           # merged range leaves (MergeRangeFilterOptimizer)
    " WHERE (r < 100 OR s IN (1, 2)) AND NOT f = 3",
]


@pytest.mark.parametrize("atomic", [False, True])
def test_range_index_leaves(ctx, monkeypatch, atomic):
    # the device-atomic roaring build (PH_ROARING_ATOMIC) must also compose the slice-evaluated range leaves
    if atomic:
        monkeypatch.setenv("PH_ROARING_ATOMIC", "1")
    t = _ri_cols(150_001, 11)
    seg = ctx.pin(create_segment("ri", t, inverted=("s",), range_index=("r", "s")))
    oseg = O.build_segment("ri", t, inverted=("s",), range_index=("r", "s"))
    for w in RANGE_WHERE:
        _check(ctx, seg, oseg, w)


def test_tiny_segment_array_only_slices(ctx):
    # a few hundred docs: every RangeBitmap slice is an array container, the index smaller than one thread stride
    t = _ri_cols(300, 12)
    seg = ctx.pin(create_segment("tiny", t, range_index=("r",)))
    oseg = O.build_segment("tiny", t, range_index=("r",))
    for w in RANGE_WHERE[:2] + RANGE_WHERE[3:6]:
        _check(ctx, seg, oseg, w)


def test_bad_and_null_arguments(ctx):
    from pinot_amd import native as N
    rng = np.random.default_rng(9)
    t = _random_table(rng, 130)
    seg = ctx.pin(create_segment("bad", t))
    with pytest.raises(N.BadQueryError):
        ctx.filter(parse_sql("SELECT COUNT(*) FROM t WHERE nosuch = 1"), seg)
    import ctypes
    from pinot_amd.engine import _QueryStruct
    qs = _QueryStruct(parse_sql("SELECT COUNT(*) FROM t WHERE a = 1"))
    small = np.zeros(1, np.uint64)  # 130 docs need 3 words
    rc = N.lib().ph_filter_execute(ctx.handle, ctypes.byref(qs.struct), seg.handle, small.ctypes.data, 1, None)
    assert rc == N.PH_ERR_INVALID_ARGUMENT
