"""Pins the CPU oracle (oracle/) against the reference's own known-answer tests.

* test_data-sv.avro KATs (tests/kat_sv.py) -- COUNT/SUM/MIN/MAX/DISTINCTCOUNTHLL, group-by tables.
* FastFilteredCountTest (pinot-core/src/test/java/org/apache/pinot/queries/FastFilteredCountTest.java:
  99-112 data, 144-200 closed-form expectations).
* RangeQueriesTest (pinot-core/.../queries/RangeQueriesTest.java:95-108 data) range counts.
* FixedBitIntReaderTest (pinot-segment-local/.../io/reader/impl/FixedBitIntReaderTest.java:43-81):
  round trip for every width 1..31, plus a hand-computed MSB-first big-endian layout.
"""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from tests import kat_sv
from tests.seeds import seed_of


@pytest.fixture(scope="module")
def sv_segments():
    cols = kat_sv.load_columns()
    seg = O.build_segment("testTable_126164076_167572854", cols, inverted=kat_sv.INVERTED)
    return [seg] * 4


def run(sql, segs):
    q = parse_sql(sql)
    r = O.execute(q, segs)
    return reduce_groups(q, r.keys, r.aggs), r.stats


def test_segment_metadata_matches_reference_header(sv_segments):
    # BaseSingleValueQueriesTest.java:54-68 (column12 is 9 in the data; the comment says 5)
    seg = sv_segments[0]
    card = {c: seg.columns[c].cardinality for c in seg.columns}
    assert card["column1"] == 6582 and card["column3"] == 21910 and card["column6"] == 608
    assert card["column7"] == 146 and card["column9"] == 1737 and card["column11"] == 5
    assert card["column17"] == 24 and card["column18"] == 1440 and card["daysSinceEpoch"] == 2
    assert seg.columns["column5"].is_sorted and seg.columns["daysSinceEpoch"].is_sorted
    assert not seg.columns["column1"].is_sorted


@pytest.mark.parametrize("sql,rows,stats,src", kat_sv.KATS, ids=[k[3] for k in kat_sv.KATS])
def test_reference_kat(sv_segments, sql, rows, stats, src):
    table, st = run(sql, sv_segments)
    assert table.rows == rows, src
    docs, _post, total = stats
    assert st.num_total_docs == total
    if "WHERE" in sql or "GROUP BY" in sql or "SUM(" in sql.upper():
        assert st.num_docs_scanned == docs
        assert st.num_entries_scanned_post_filter == stats[1]


APPLY_AND = [
    # (filter, numpy expectation per segment): ANDs of index-based children (sorted daysSinceEpoch, inverted column6 /
    # column7 EQ, an OR of inverted leaves) and scans: |D0| + |D0 n S1| + ... (AndDocIdSet.java:128-170 applyAnd)
    (" WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND daysSinceEpoch = 126164076",
     lambda c: _apply_and(c, [c["daysSinceEpoch"] == 126164076],
                          [c["column1"] > 100000000, (c["column3"] >= 20000000) & (c["column3"] <= 1000000000)])),
    (" WHERE (column7 = 363 OR column11 = 'P') AND column9 > 1000000 AND column1 < 900000000 AND column3 > 5",
     lambda c: _apply_and(c, [(c["column7"] == 363) | (c["column11"] == "P")],
                          [c["column9"] > 1000000, c["column1"] < 900000000, c["column3"] > 5])),
]


def _apply_and(c, idx, scans):
    d = np.ones(len(c["column1"]), bool)
    for m in idx:
        d &= m
    total = 0
    for s in scans:
        if s.all():  # matches every dictionary value: a MatchAll child, dropped from the AND (FilterPlanNode)
            continue
        total += int(d.sum())
        d &= s
    return total


@pytest.mark.parametrize("k", range(len(APPLY_AND)))
def test_apply_and_filter_entries(sv_segments, k):
    # the oracle's applyAnd statistic against an independent numpy restatement of the reference's order of work
    where, expect = APPLY_AND[k]
    cols = {c: v for c, (v, _) in kat_sv.load_columns().items()}
    _, st = run("SELECT COUNT(*) FROM testTable" + where, sv_segments)
    assert st.num_entries_scanned_in_filter == 4 * expect(cols)


def test_kat_filter_entries_definition(sv_segments):
    # The KAT filter's AND holds an OR with a scan child (column6 RANGE: RANGE never uses the inverted index,
    # FilterOperatorUtils.java:97-104), which the reference drives with advance() calls (AndDocIdIterator /
    # OrDocIdIterator) after applyAnd of column1 / column3 over the sorted daysSinceEpoch range:
    # InterSegmentAggregationSingleValueQueriesTest.java:58 pins 252 256 entries
    _, st = run("SELECT COUNT(*) FROM testTable" + kat_sv.FILTER, sv_segments)
    assert st.num_entries_scanned_in_filter == 252256


# ------------------------------------------------------------------ FastFilteredCountTest
def _fast_filtered_segment():
    n = 1000  # FastFilteredCountTest.java:99-112: class = i % 8 (inverted), sorted = i (sorted, inverted)
    i = np.arange(n, dtype=np.int32)
    return [O.build_segment("fast", {"class": (i % 8, "INT"), "sorted": (i, "INT")}, inverted=("class", "sorted"))]


@pytest.mark.parametrize("where,expected", [
    ("class = 3", 125),
    ("class IN (1, 2, 3)", 375),
    ("class NOT IN (1, 2)", 750),
    ("class <> 5", 875),
    ("sorted BETWEEN 100 AND 199", 100),
    ("NOT sorted BETWEEN 100 AND 199", 900),
    ("class = 3 AND sorted BETWEEN 0 AND 499", 63),
    ("class = 3 OR sorted BETWEEN 0 AND 499", 500 + 62),
    ("NOT (class = 3 OR class = 4)", 750),
    ("sorted > 990", 9),
    ("sorted >= 990", 10),
    ("sorted < 10", 10),
    ("sorted <= 10", 11),
])
def test_fast_filtered_count(where, expected):
    segs = _fast_filtered_segment()
    t, st = run("SELECT COUNT(*) FROM testTable WHERE " + where, segs)
    # closed form: docs i in [0,1000) with class = i % 8
    assert t.rows == [[expected]]


# ------------------------------------------------------------------ RangeQueriesTest
def test_range_queries_closed_form():
    # RangeQueriesTest.java:95-108: v = ((100000 + 500) - i * 100) % 100000, NUM_RECORDS = 1000
    n = 1000
    i = np.arange(n, dtype=np.int64)
    v = ((100000 + 500) - i * 100) % 100000
    segs = [O.build_segment("range", {"intCol": (v.astype(np.int32), "INT"), "longCol": (v, "LONG"),
                                      "doubleCol": (v.astype(np.float64), "DOUBLE")})]
    for lo, hi in [(0, 500), (50000, 60000), (99500, 100000), (-5, 5), (123, 124)]:
        exp = int(np.sum((v >= lo) & (v <= hi)))
        for col in ("intCol", "longCol", "doubleCol"):
            t, _ = run(f"SELECT COUNT(*) FROM t WHERE {col} BETWEEN {lo} AND {hi}", segs)
            assert t.rows == [[exp]], (col, lo, hi)
        exp2 = int(np.sum((v > lo) & (v < hi)))
        t, _ = run(f"SELECT COUNT(*) FROM t WHERE intCol > {lo} AND intCol < {hi}", segs)
        assert t.rows == [[exp2]]


# ------------------------------------------------------------------ fixed-bit codec
def test_num_bits_per_value():
    # PinotDataBitSet.getNumBitsPerValue
    assert O.num_bits_per_value(0) == 1 and O.num_bits_per_value(1) == 1
    assert O.num_bits_per_value(2) == 2 and O.num_bits_per_value(255) == 8
    assert O.num_bits_per_value(256) == 9 and O.num_bits_per_value(999_999) == 20
    assert O.num_bits_per_value(2**31 - 1) == 31


def test_fixed_bit_layout_hand_computed():
    # 3-bit values 5,3,7,0,1 -> bit stream 101 011 111 000 001 (MSB first) -> bytes 0xAF 0x82
    buf = O.fixed_bit_pack(np.array([5, 3, 7, 0, 1]), 3)
    assert buf.tolist() == [0b10101111, 0b10000010]


@pytest.mark.parametrize("bits", range(1, 32))
def test_fixed_bit_round_trip(bits):
    # FixedBitIntReaderTest.java:43-81 -- 95 random values per width, read at every offset
    rng = np.random.default_rng(bits)
    vals = rng.integers(0, 1 << bits, size=95, dtype=np.int64).astype(np.int32)
    buf = O.fixed_bit_pack(vals, bits)
    assert len(buf) == (95 * bits + 7) // 8
    assert np.array_equal(O.fixed_bit_unpack(buf, 95, bits), vals)
    for s in (0, 1, 31, 64):
        assert np.array_equal(O.fixed_bit_unpack(buf, 95 - s, bits, start=s), vals[s:])


def test_hll_serialized_layout_against_reference_fixture():
    # pinot-core/src/test/resources/data/rawhllresults.txt format: header (8, 172), 43 BE words, 5-bit regs.
    from pinot_amd.reduce import hll_serialize
    regs = np.arange(256) % 17
    b = hll_serialize(regs.astype(np.uint8), 8)
    assert len(b) == 180 and b[:8] == bytes([0, 0, 0, 8, 0, 0, 0, 172])
    words = np.frombuffer(b[8:], dtype=">u4")
    dec = [(int(words[i // 6]) >> (5 * (i % 6))) & 31 for i in range(256)]
    assert dec == regs.tolist()


def test_segment_trim_heap_keeps_the_top_groups():
    # TableResizer's heap (oracle._segment_trim) keeps exactly the top `size` groups when the ORDER BY values are
    # distinct; a trimmed segment's dropped groups lose that segment's partial aggregates in the combine
    rng = np.random.default_rng(5)
    n = 20_000
    t = {"a": (rng.integers(0, 100, n).astype(np.int32), "INT"), "m": (rng.permutation(n).astype(np.int32), "INT")}
    seg = O.build_segment("trim", t)
    q = parse_sql("SET minSegmentGroupTrimSize=30; SELECT a, MAX(m) FROM t GROUP BY a ORDER BY MAX(m) DESC LIMIT 2")
    r = O.execute(q, [seg])
    full = O.execute(parse_sql("SELECT a, MAX(m) FROM t GROUP BY a ORDER BY MAX(m) DESC LIMIT 1000"), [seg])
    top = sorted(zip(full.keys, [row[0] for row in full.aggs]), key=lambda x: -x[1])[:30]
    assert sorted(r.keys) == sorted(k for k, _ in top)


def test_table_resizer_in_segment_trim_kat():
    # TableResizerTest.testInSegmentTrim (TableResizerTest.java:336-377): five groups (d1, d2, d3 | SUM(m1), MAX(m2),
    # DISTINCTCOUNT(m3)) in group-id order, trimmed to 3; the returned list is the heap array (index 0 first)
    recs = [("a", 10, 1.0, 10.0, 100.0, 1), ("b", 10, 2.0, 20.0, 200.0, 2), ("c", 200, 3.0, 30.0, 300.0, 2),
            ("c", 50, 4.0, 30.0, 200.0, 3), ("c", 300, 5.0, 20.0, 100.0, 4)]

    def by(cols):  # the intermediate-record comparator over (column index, ascending) pairs
        def inter(a, b):
            for ci, asc in cols:
                c = O._java_compare(a[ci], b[ci])
                if c:
                    return c if asc else -c
            return 0
        return inter

    def kept(cols):
        return [recs.index(r) for r in O.table_resizer_heap(recs, by(cols), 3)]

    h = kept([(2, False)])  # ORDER BY d3 DESC -> records 2, {3, 4}
    assert h[0] == 2 and sorted(h[1:]) == [3, 4]
    h = kept([(3, False), (4, False), (5, False)])  # SUM(m1) DESC, MAX(m2) DESC, DISTINCTCOUNT(m3) DESC
    assert h[0] == 1 and sorted(h[1:]) == [2, 3]
    h = kept([(5, False)] + [(0, True)])  # DISTINCTCOUNT(m3) DESC, then a tie-free key (the KAT's AVG(m4) ASC tie-break)
    assert h[0] == 1 and sorted(h[1:]) == [3, 4]


def test_java_string_order_is_utf16():
    # String.compareTo compares UTF-16 code units: a supplementary character (surrogates D800-DBFF) sorts BEFORE
    # U+E000..U+FFFF, where code-point / UTF-8 byte order puts it after
    assert O._java_compare("\U0001F600", "") == -1
    assert O._java_compare("", "\U0001F600") == 1
    assert O._java_compare("ab", "abc") == -1 and O._java_compare("b", "abc") == 1


def _and_or_iterator_entries(c):
    """The KAT filter's reference iterator tree on one segment, simulated: AndDocIdSet (AndDocIdSet.java:128-185)
    merges the sorted daysSinceEpoch range, applies the column1 and column3 scans to it (applyAnd) and ANDs the result
    with the remaining OR(column6 RANGE scan, column11 NOT IN bitmap) through AndDocIdIterator.next / advance
    (AndDocIdIterator.java:38-75) and OrDocIdIterator.advance (OrDocIdIterator.java:73-101), whose scan child counts
    every doc it examines (SVScanDocIdIterator.advance :101-112)."""
    n = len(c["column1"])
    d0 = c["daysSinceEpoch"] == 126164076
    s1 = c["column1"] > 100000000
    s2 = (c["column3"] >= 20000000) & (c["column3"] <= 1000000000)
    cand = np.nonzero(d0 & s1 & s2)[0]
    o1 = np.nonzero(c["column6"] < 500000000)[0]
    o2 = np.nonzero(~np.isin(c["column11"], ["t", "P"]))[0]
    scanned = [int(d0.sum() + (d0 & s1).sum())]  # the two applyAnd steps

    def scan_advance(t):
        i = np.searchsorted(o1, t)
        if i < len(o1):
            scanned[0] += int(o1[i]) - t + 1
            return int(o1[i])
        scanned[0] += n - t
        return -1

    def bitmap_advance(t):
        i = np.searchsorted(o2, t)
        return int(o2[i]) if i < len(o2) else -1

    nxt, alive = [-1, -1], [True, True]

    def or_advance(t):
        best = None
        for i, f in ((0, scan_advance), (1, bitmap_advance)):
            if not alive[i]:
                continue
            if nxt[i] < t:
                nxt[i] = f(t)
                if nxt[i] == -1:
                    alive[i] = False
                    continue
            best = nxt[i] if best is None else min(best, nxt[i])
        return -1 if best is None else best

    def r_advance(t):
        i = np.searchsorted(cand, t)
        return int(cand[i]) if i < len(cand) else -1

    its, next_doc, matches = [r_advance, or_advance], 0, 0
    while True:
        max_doc, max_idx, idx = next_doc, -1, 0
        while idx < 2:
            if idx == max_idx:
                idx += 1
                continue
            doc = its[idx](max_doc)
            if doc == -1:
                return scanned[0], matches
            if doc == max_doc:
                idx += 1
            else:
                max_doc, max_idx, idx = doc, idx, 0
        matches += 1
        next_doc = max_doc + 1


def _iterator_entries(d0, scans, b_kids, n):
    """Literal simulation of AndDocIdIterator(RangelessBitmapDocIdIterator(applyAnd(D0, scans)), OrDocIdIterator(
    kids)): b_kids = [(is_scan, bool array)]; scan kids count every doc their advance() examines."""
    cur = d0.copy()
    scanned = 0
    for sc in scans:
        scanned += int(cur.sum())
        cur &= sc
    cand = np.nonzero(cur)[0]
    kids = [(is_scan, np.nonzero(m)[0]) for is_scan, m in b_kids]
    nxt, alive = [-1] * len(kids), [True] * len(kids)

    def kid_advance(i, t):
        nonlocal scanned
        is_scan, pos = kids[i]
        j = np.searchsorted(pos, t)
        if is_scan:
            scanned += (int(pos[j]) - t + 1) if j < len(pos) else n - t
        return int(pos[j]) if j < len(pos) else -1

    def or_advance(t):
        best = None
        for i in range(len(kids)):
            if not alive[i]:
                continue
            if nxt[i] < t:
                nxt[i] = kid_advance(i, t)
                if nxt[i] == -1:
                    alive[i] = False
                    continue
            best = nxt[i] if best is None else min(best, nxt[i])
        return -1 if best is None else best

    def r_advance(t):
        i = np.searchsorted(cand, t)
        return int(cand[i]) if i < len(cand) else -1

    its, next_doc = [r_advance, or_advance], 0
    while True:
        max_doc, max_idx, idx = next_doc, -1, 0
        while idx < 2:
            if idx == max_idx:
                idx += 1
                continue
            doc = its[idx](max_doc)
            if doc == -1:
                return scanned
            if doc == max_doc:
                idx += 1
            else:
                max_doc, max_idx, idx = doc, idx, 0
        next_doc = max_doc + 1


@pytest.mark.parametrize("case", range(60))
def test_and_or_entries_closed_form_vs_iterators(case):
    # oracle.and_or_entries (the per-candidate closed form the GPU path's host pass also uses) against the literal
    # iterator simulation, on random densities
    rng = np.random.default_rng(seed_of(f"and-or-{case}"))
    n = int(rng.integers(1, 3000))
    dens = rng.uniform(0.001, 0.9, 8)
    d0 = rng.random(n) < dens[0]
    scans = [rng.random(n) < dens[1 + k] for k in range(int(rng.integers(0, 3)))]
    b_kids = [(bool(rng.integers(0, 2)), rng.random(n) < dens[4 + k]) for k in range(int(rng.integers(1, 4)))]
    b = np.logical_or.reduce([m for _, m in b_kids])
    ors = [m for is_scan, m in b_kids if is_scan]
    assert O.and_or_entries(d0, scans, b, ors) == _iterator_entries(d0, scans, b_kids, n)


def test_kat_filter_entries_oracle():
    # the oracle's exact AND-with-a-remaining-OR statistic on the KAT filter: 252 256 over the 4 segments
    e = O.execute(parse_sql("SELECT COUNT(*) FROM testTable" + kat_sv.FILTER),
                  [O.build_segment("kat", kat_sv.load_columns(), inverted=kat_sv.INVERTED)] * 4)
    assert e.stats.num_entries_scanned_in_filter == 252256


def test_kat_filter_entries_reference_iterators():
    # InterSegmentAggregationSingleValueQueriesTest.java:58: 252 256 entries over the 4 segments (2 copies x 2 servers)
    cols = {k: v for k, (v, _) in kat_sv.load_columns().items()}
    entries, matches = _and_or_iterator_entries(cols)
    assert 4 * matches == 24516 and 4 * entries == 252256


def test_filter_docs_matches_execute():
    # oracle.filter_docs (the segment-level filter's doc set + statistic, ph_filter_execute's checker) agrees with the
    # KAT-pinned execute path on the reference's filter
    from pinot_amd.query import parse_sql
    from tests import kat_sv
    seg = O.build_segment("kat", kat_sv.load_columns(), inverted=kat_sv.INVERTED)
    q = parse_sql("SELECT COUNT(*) FROM testTable" + kat_sv.FILTER)
    mask, entries = O.filter_docs(q, seg)
    e = O.execute(q, [seg])
    assert int(mask.sum()) * 4 == 24516 and entries * 4 == 252256
    assert int(mask.sum()) == e.stats.num_docs_scanned and entries == e.stats.num_entries_scanned_in_filter
    w = O.doc_words(mask)
    assert len(w) == (seg.num_docs + 63) // 64 and int(np.unpackbits(w.view(np.uint8)).sum()) == int(mask.sum())
