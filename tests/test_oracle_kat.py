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


def test_kat_filter_entries_definition(sv_segments):
    # Under this build's definition every scan leaf is evaluated on every doc: column1 (RANGE, scan) and
    # column3 (RANGE, scan) and column6 (RANGE on an inverted column -> scan; FilterOperatorUtils.java:97-104).
    _, st = run("SELECT COUNT(*) FROM testTable" + kat_sv.FILTER, sv_segments)
    assert st.num_entries_scanned_in_filter == 3 * 120000


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
