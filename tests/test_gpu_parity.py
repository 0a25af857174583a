"""GPU parity: libpinot_hip.so (through the C-ABI) vs the CPU oracle and the reference KATs.

Bar: bit-exact for COUNT, integer SUM, MIN/MAX, HLL registers and group keys; DOUBLE SUM within 1e-9
relative (BASELINE.json north_star).
"""
import math

import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment
from tests import kat_sv
from tests.seeds import seed_of

pytestmark = pytest.mark.gpu

DOUBLE_RTOL = 1e-9


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def sv(ctx):
    cols = kat_sv.load_columns()
    buf = create_segment("testTable_126164076_167572854", cols, inverted=kat_sv.INVERTED)
    seg = ctx.pin(buf)
    return [seg] * 4


def rows_equal(got, exp, rtol=0.0):
    assert len(got) == len(exp), (len(got), len(exp))
    for g, e in zip(got, exp):
        assert len(g) == len(e)
        for a, b in zip(g, e):
            if isinstance(b, float) and rtol and not (math.isinf(b) or b == 0):
                assert abs(a - b) <= rtol * abs(b), (a, b)
            else:
                assert a == b, (g, e)


@pytest.mark.parametrize("sql,rows,stats,src", kat_sv.KATS, ids=[k[3] for k in kat_sv.KATS])
def test_reference_kat_on_gpu(ctx, sv, sql, rows, stats, src):
    q = parse_sql(sql)
    r = ctx.execute(q, sv)
    table = reduce_groups(q, r.keys, r.aggs)
    assert table.rows == rows, src
    docs, post, total = stats
    assert r.stats.num_total_docs == total
    assert r.stats.num_docs_scanned == docs
    assert r.stats.num_entries_scanned_post_filter == post


@pytest.mark.parametrize("where", [
    " WHERE column1 > 100000000 AND column3 BETWEEN 20000000 AND 1000000000 AND daysSinceEpoch = 126164076",
    " WHERE (column7 = 363 OR column11 = 'P') AND column9 > 1000000 AND column1 < 900000000 AND column3 > 5",
    " WHERE column6 = 1095 AND column1 > 100000000",
])
def test_apply_and_filter_entries_gpu(ctx, sv, where):
    # ANDs of index-based children + scans: numEntriesScannedInFilter = |D0| + |D0 n S1| + ... (applyAnd), counted
    # per doc by the flagged AND of the GPU program; the oracle's count is pinned by a numpy restatement
    # (test_oracle_kat.py::test_apply_and_filter_entries)
    from oracle import oracle as O
    q = parse_sql("SELECT COUNT(*) FROM testTable" + where)
    r = ctx.execute(q, sv)
    e = O.execute(q, [O.build_segment("kat", kat_sv.load_columns(), inverted=kat_sv.INVERTED)] * 4)
    assert r.stats.num_entries_scanned_in_filter == e.stats.num_entries_scanned_in_filter
    assert reduce_groups(q, r.keys, r.aggs).rows == reduce_groups(q, e.keys, e.aggs).rows
    q2 = parse_sql("SELECT column9, COUNT(*) FROM testTable" + where + " GROUP BY column9 ORDER BY column9 LIMIT 10")
    r2 = ctx.execute(q2, sv)
    assert r2.stats.num_entries_scanned_in_filter == e.stats.num_entries_scanned_in_filter


def test_kat_filter_entries_gpu(ctx, sv):
    # InterSegmentAggregationSingleValueQueriesTest.java:58: the AND's remaining OR (column6 scan, column11 NOT IN
    # bitmap) is driven by advance() -- k_filter_bitmaps + the host closed form
    r = ctx.execute(parse_sql("SELECT COUNT(*) FROM testTable" + kat_sv.FILTER), sv)
    assert r.stats.num_entries_scanned_in_filter == 252256
    assert r.stats.num_docs_scanned == 24516


@pytest.mark.parametrize("where", [
    " WHERE daysSinceEpoch = 126164076 AND column1 > 100000000 AND (column6 < 500000000 OR column9 > 1000000)",
    " WHERE column5 = 'gFuH' AND column11 = 'P' AND (column3 > 20000000 OR column11 = 'o' OR column1 < 5000000)",
    " WHERE column7 = 788414092 AND column3 < 1500000000 "
    "AND (column6 BETWEEN 3000 AND 900000000 OR column9 < 50000000)",
])
def test_and_or_filter_entries_gpu(ctx, sv, where):
    # ANDs with one remaining OR of scans / index leaves: the reference's advance()-driven statistic on the GPU path
    # equals the oracle's (whose closed form is checked against a literal iterator simulation)
    from oracle import oracle as O
    q = parse_sql("SELECT COUNT(*) FROM testTable" + where)
    r = ctx.execute(q, sv)
    e = O.execute(q, [O.build_segment("kat", kat_sv.load_columns(), inverted=kat_sv.INVERTED)] * 4)
    assert r.stats.num_entries_scanned_in_filter == e.stats.num_entries_scanned_in_filter
    assert reduce_groups(q, r.keys, r.aggs).rows == reduce_groups(q, e.keys, e.aggs).rows


# ------------------------------------------------------------------ randomized parity vs the oracle
def _random_table(rng, n, int_cards=(7, 300, 5000), with_strings=True, with_double=True):
    cols = {
        "a": (rng.integers(0, int_cards[0], n).astype(np.int32), "INT"),
        "b": (rng.integers(-1000, 1000, n).astype(np.int32) * int(rng.integers(1, 5)), "INT"),
        "c": (rng.integers(0, int_cards[2], n).astype(np.int64) * 1_000_003 - 7, "LONG"),
        "m": (rng.integers(0, 1 << 30, n).astype(np.int32), "INT"),
        "s": (np.sort(rng.integers(0, 40, n)).astype(np.int32), "INT"),  # sorted
    }
    if with_strings:
        words = np.array(["", "P", "gFuH", "o", "t", "zz", "Ünï"])
        cols["str"] = (words[rng.integers(0, len(words), n)], "STRING")
    if with_double:
        cols["d"] = (np.round(rng.normal(0, 1000, n), 3), "DOUBLE")
    return cols


def _both(ctx, cols_list, sql, inverted=(), run_opt=False, rtol=DOUBLE_RTOL):
    q = parse_sql(sql)
    gpu_segs = [ctx.pin(create_segment(f"s{i}", c, inverted=inverted, run_optimize=run_opt))
                for i, c in enumerate(cols_list)]
    ora_segs = [O.build_segment(f"s{i}", c, inverted=inverted) for i, c in enumerate(cols_list)]
    r = ctx.execute(q, gpu_segs)
    e = O.execute(q, ora_segs)
    got = reduce_groups(q, r.keys, r.aggs)
    exp = reduce_groups(q, e.keys, e.aggs)
    rows_equal(got.rows, exp.rows, rtol)
    # HLL registers are compared raw (bit-exact), not only via the estimate
    for k, a in enumerate(q.aggregations):
        if a.function == "DISTINCTCOUNTHLL":
            gmap = {key: row[k] for key, row in zip(r.keys, r.aggs)}
            for key, row in zip(e.keys, e.aggs):
                assert np.array_equal(gmap[key], row[k])
    assert r.stats.num_docs_scanned == e.stats.num_docs_scanned
    assert r.stats.num_total_docs == e.stats.num_total_docs
    assert r.stats.num_entries_scanned_post_filter == e.stats.num_entries_scanned_post_filter
    # numEntriesScannedInFilter: the reference's iterator counts, for every filter shape (oracle.filter_entries)
    assert r.stats.num_entries_scanned_in_filter == e.stats.num_entries_scanned_in_filter, sql
    return r, got


FILTERS = [
    "",
    " WHERE a = 3",
    " WHERE a <> 3",
    " WHERE a IN (1, 2, 5)",
    " WHERE a NOT IN (0, 6)",
    " WHERE b BETWEEN -500 AND 250",
    " WHERE b > 0 AND m < 536870912",
    " WHERE (a = 1 OR b >= 900) AND NOT c < 0",
    " WHERE s BETWEEN 10 AND 20",
    " WHERE s IN (3, 7, 30) OR a = 2",
    " WHERE s <> 5 AND a NOT IN (1)",
    " WHERE str = 'gFuH'",
    " WHERE str NOT IN ('t', 'P') AND b < 100",
    " WHERE str > 'o'",
    " WHERE d > 0.5",
    " WHERE a = 99",
    " WHERE a >= 0",
    " WHERE NOT (a IN (0, 1, 2, 3, 4, 5, 6))",
    " WHERE str > ''",  # '' is a literal, not an open bound (RangePredicateEvaluatorFactory)
    " WHERE str <= '' OR a = 1",
]


@pytest.mark.parametrize("where", FILTERS)
def test_random_aggregation_only(ctx, where):
    rng = np.random.default_rng(seed_of(where))
    tables = [_random_table(rng, n) for n in (20_000, 777, 64 * 300 + 1)]
    _both(ctx, tables, "SELECT COUNT(*), SUM(m), MIN(b), MAX(c), SUM(d), MIN(d), MAX(d) FROM t" + where,
          inverted=("a", "str"))


@pytest.mark.parametrize("where", FILTERS[:12])
@pytest.mark.parametrize("group", ["a", "str", "s", "a, str", "s, a, str", "b", "c"])
def test_random_group_by(ctx, where, group):
    rng = np.random.default_rng(seed_of(where + group))
    tables = [_random_table(rng, n) for n in (9_999, 30_000)]
    _both(ctx, tables, f"SET numGroupsLimit=10000000; SELECT {group}, COUNT(*), SUM(m), MIN(d), MAX(b), SUM(d) "
                       f"FROM t{where} GROUP BY {group} ORDER BY {group} LIMIT 100000", inverted=("a", "str"))


@pytest.mark.parametrize("bits", list(range(1, 23)))
def test_every_bit_width_scan(ctx, bits):
    rng = np.random.default_rng(bits)
    n = max(50_000, (1 << (bits - 1)) + 5_000)
    card = min(1 << bits, n)
    vals = rng.permutation(np.concatenate([np.arange(card), rng.integers(0, card, n - card)])).astype(np.int32)
    t = {"v": (vals, "INT"), "m": (rng.integers(0, 100, n).astype(np.int32), "INT")}
    lo, hi = card // 4, card // 4 + max(1, card // 3)
    _both(ctx, [t], f"SELECT COUNT(*), SUM(m), MIN(v), MAX(v) FROM t WHERE v BETWEEN {lo} AND {hi}")


@pytest.mark.parametrize("bits", list(range(1, 32)))
def test_device_unpack_every_width(ctx, bits):
    # the per-doc gather routine (generic filter programs, value re-encoding, HLL reads) on raw packed
    # streams of every width 1..31 (FixedBitIntReaderTest widths, FixedBitIntReaderTest.java:43-81)
    from pinot_amd import native as N
    rng = np.random.default_rng(1000 + bits)
    for n in (1, 63, 64, 65, 100_003):
        ids = rng.integers(0, 1 << bits, n, dtype=np.int64).astype(np.int32)
        packed = O.fixed_bit_pack(ids, bits)
        out = np.zeros(n, np.int32)
        N.check(N.lib().ph_selftest_unpack(ctx.handle, packed.ctypes.data, packed.nbytes, n, bits,
                                           out.ctypes.data))
        assert np.array_equal(out, ids), (bits, n)


@pytest.mark.parametrize("bits", list(range(1, 32)))
def test_device_staged_unpack_every_width(ctx, bits):
    # the scan kernels' own staged decode (tile_load -> tile_store -> BitCursor, the code k_scan runs) for every
    # width 1..31 and every tile size the planner picks, on streams whose length is not a tile multiple
    from pinot_amd import native as N
    rng = np.random.default_rng(2000 + bits)
    for tw in (4, 8, 16, 32):
        if (tw * 8 * bits + 8 + 1023) // 1024 > 12:  # wider than the prefetch pool: the planner halves the tile
            continue
        for n in (1, 64, 64 * tw + 1, 200_003):
            ids = rng.integers(0, 1 << bits, n, dtype=np.int64).astype(np.int32)
            ids[:2] = [0, (1 << bits) - 1][: min(2, n)]
            packed = O.fixed_bit_pack(ids, bits)
            out = np.full(n, -7, np.int32)
            N.check(N.lib().ph_selftest_unpack_staged(ctx.handle, packed.ctypes.data, packed.nbytes, n, bits, tw,
                                                      out.ctypes.data))
            assert np.array_equal(out, ids), (bits, tw, n)


def test_wide_bits_31(ctx):
    rng = np.random.default_rng(31)
    n = 4096 + 17
    vals = rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype(np.int32)
    vals[:2] = [-2**31, 2**31 - 1]
    t = {"v": (vals, "INT")}
    _both(ctx, [t], "SELECT COUNT(*), SUM(v), MIN(v), MAX(v) FROM t WHERE v > -1000000")


def test_hll_parity(ctx):
    rng = np.random.default_rng(3)
    tables = []
    for n in (50_000, 12_345):
        tables.append({"u": (rng.integers(0, 1 << 27, n).astype(np.int32), "INT"),
                       "l": (rng.integers(0, 1 << 40, n).astype(np.int64), "LONG"),
                       "st": (np.array([f"k{v}" for v in rng.integers(0, 3000, n)]), "STRING"),
                       "dd": (rng.normal(size=n), "DOUBLE"),
                       "c": (rng.integers(0, 100, n).astype(np.int32), "INT")})
    _both(ctx, tables, "SELECT DISTINCTCOUNTHLL(u), DISTINCTCOUNTHLL(l), DISTINCTCOUNTHLL(st), "
                       "DISTINCTCOUNTHLL(dd) FROM t WHERE c IN (1, 5, 9, 77)", inverted=("c",))
    _both(ctx, tables, "SELECT DISTINCTCOUNTHLL(u) FROM t WHERE c IN (1, 5, 9, 77)", inverted=("c",), run_opt=True)
    _both(ctx, tables, "SELECT c, DISTINCTCOUNTHLL(u, 10) FROM t WHERE c < 20 GROUP BY c ORDER BY c", inverted=("c",))
    _both(ctx, tables, "SELECT DISTINCTCOUNTHLL(u, 12) FROM t")


def test_hll_float_column(ctx):
    # DISTINCTCOUNTHLL on FLOAT (DistinctCountHLLAggregationFunction.java:127-131 offers the Float: clearspring hashes
    # hashLong(floatToRawIntBits)); registers compared raw with the oracle's restatement (parity unpinned: no KAT)
    rng = np.random.default_rng(33)
    tables = []
    for n in (40_000, 9_999):
        tables.append({"fl": (np.round(rng.normal(size=n), 3).astype(np.float32), "FLOAT"),
                       "c": (rng.integers(0, 100, n).astype(np.int32), "INT")})
    _both(ctx, tables, "SELECT DISTINCTCOUNTHLL(fl) FROM t WHERE c < 60")
    _both(ctx, tables, "SELECT c, DISTINCTCOUNTHLL(fl) FROM t WHERE c < 20 GROUP BY c ORDER BY c")


def test_inverted_index_containers(ctx):
    # dense values -> bitmap containers; runs -> run containers; sparse -> array containers
    n = 300_000
    a = np.zeros(n, np.int32)
    a[::2] = 1
    a[100_000:180_000] = 2
    a[rng_idx(n, 50)] = 3
    t = {"a": (a, "INT"), "m": (np.arange(n, dtype=np.int32) % 1000, "INT")}
    for run_opt in (False, True):
        for where in ("a = 1", "a IN (2, 3)", "a NOT IN (1)", "a <> 0"):
            _both(ctx, [t], f"SELECT COUNT(*), SUM(m) FROM t WHERE {where}", inverted=("a",), run_opt=run_opt)


@pytest.mark.parametrize("force", [False, True])
def test_agg_sparse_from_containers(ctx, monkeypatch, force):
    # k_agg_sparse straight from the roaring containers of EQ / IN leaves (PH_KERNEL_AGG_CONTAINERS: no doc bitmap):
    # array, bitmap and run containers, several ids per leaf (disjoint doc sets), segments ending mid-container,
    # COUNT / SUM / MIN / MAX / DISTINCTCOUNTHLL against the oracle; forced also onto the non-selective leaves
    if force:
        monkeypatch.setenv("PH_AGG_SPARSE", "1")
    rng = np.random.default_rng(77)
    tables = []
    for n in (300_000, 65_536, 131_171):
        a = rng.integers(10, 400, n).astype(np.int32)  # sparse ids -> array containers
        a[::2] = 1  # dense -> bitmap containers
        a[n // 3: n // 3 + 70_000] = 2  # a long run -> run containers (run_opt) / bitmap containers
        a[-5:] = 3
        tables.append({"a": (a, "INT"), "m": (rng.integers(-5000, 5000, n).astype(np.int32), "INT")})
    sel = "COUNT(*), SUM(m), MIN(m), MAX(m), DISTINCTCOUNTHLL(m)"
    for run_opt in (False, True):
        for where, selective in (("a = 17", True), ("a IN (17, 99, 3, 250)", True), ("a = 1", False),
                                 ("a IN (2, 3)", False), ("a IN (1, 2, 17)", False), ("a = 12345", True)):
            r, _ = _both(ctx, tables, f"SELECT {sel} FROM t WHERE {where}", inverted=("a",), run_opt=run_opt)
            if (force or selective) and "12345" not in where:
                assert r.stats.scan_kernel == 14, (where, run_opt, r.stats.scan_kernel)
    monkeypatch.setenv("PH_AGG_CONT", "0")  # the bitmap form of the same plan
    r, _ = _both(ctx, tables, f"SELECT {sel} FROM t WHERE a IN (17, 99, 3, 250)", inverted=("a",))
    assert r.stats.scan_kernel == 3


@pytest.mark.parametrize("atomic", [False, True])
@pytest.mark.parametrize("n", [131072, 131172, 65536 * 3 - 1])
def test_inverted_bitmap_chunk_edges(ctx, monkeypatch, n, atomic):
    # the chunked LDS build (65536-doc chunks, padding words stored by the last chunk) and the device-atomic build
    # (PH_ROARING_ATOMIC) on segments that end on, just past and just before a chunk boundary
    if atomic:
        monkeypatch.setenv("PH_ROARING_ATOMIC", "1")
    rng = np.random.default_rng(n)
    a = rng.integers(0, 40, n).astype(np.int32)
    a[: n // 3] = 7  # dense run -> bitmap / run containers
    a[-40:] = 9
    t = {"a": (a, "INT"), "m": (rng.integers(0, 1000, n).astype(np.int32), "INT")}
    for run_opt in (False, True):
        for where in ("a = 7", "a IN (9, 3, 11)", "a NOT IN (7)", "a = 9"):
            _both(ctx, [t, t], f"SELECT COUNT(*), SUM(m), MAX(m) FROM t WHERE {where}", inverted=("a",),
                  run_opt=run_opt)


def rng_idx(n, k):
    return np.random.default_rng(1).choice(n, k, replace=False)


def test_segments_with_different_dictionaries(ctx):
    rng = np.random.default_rng(8)
    t1 = {"g": (rng.integers(0, 10, 5000).astype(np.int32) * 2, "INT"), "m": (rng.integers(0, 9, 5000).astype(np.int32), "INT")}
    t2 = {"g": (rng.integers(5, 30, 7000).astype(np.int32), "INT"), "m": (rng.integers(0, 9, 7000).astype(np.int32) - 4, "INT")}
    t3 = {"g": (np.full(100, 1000, np.int32), "INT"), "m": (np.full(100, 7, np.int32), "INT")}
    _both(ctx, [t1, t2, t3], "SELECT g, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t GROUP BY g ORDER BY g LIMIT 1000")


def test_empty_and_no_match(ctx):
    rng = np.random.default_rng(9)
    t = _random_table(rng, 1000)
    r, got = _both(ctx, [t], "SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE a = 12345")
    assert got.rows == [[0, 0.0, math.inf, -math.inf]]
    r, got = _both(ctx, [t], "SELECT a, COUNT(*) FROM t WHERE b > 100000 GROUP BY a ORDER BY a")
    assert got.rows == []
    _both(ctx, [t], "SELECT COUNT(*) FROM t WHERE a = 1 AND a = 2")


def test_large_group_key_space_global_table(ctx):
    # product of cardinalities beyond the LDS budget -> HBM dense table with device-scope atomics
    rng = np.random.default_rng(12)
    n = 400_000
    t = {"g1": (rng.integers(0, 1000, n).astype(np.int32), "INT"),
         "g2": (rng.integers(0, 300, n).astype(np.int32), "INT"),
         "m": (rng.integers(0, 1 << 20, n).astype(np.int32), "INT"),
         "f": (rng.integers(0, 1000, n).astype(np.int32), "INT")}
    _both(ctx, [t, t], "SET numGroupsLimit=2000000; SELECT g1, g2, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t "
                       "WHERE f BETWEEN 0 AND 499 GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 2000000")


@pytest.mark.parametrize("where", ["", " WHERE f < 300"])
def test_hash_group_by_beyond_dense_budget(ctx, where):
    # 3 columns of ~12 000 values each: a ~1.7e12 key space, far beyond any dense table -> MODE_GROUP_HASH
    # (open addressing over the raw mixed-radix key, sized by the docs that can match; the map-based holders
    # of DictionaryBasedGroupKeyGenerator.java:598/:778).  Segments hold fewer docs than numGroupsLimit, so the
    # limit can never be reached and no group is dropped.
    rng = np.random.default_rng(31)
    tables = []
    for n in (300_000, 123_457):
        t = {c: (rng.integers(0, 12_000, n).astype(np.int32) * 3 + k, "INT") for k, c in enumerate(("g1", "g2", "g3"))}
        t["m"] = (rng.integers(-1 << 20, 1 << 30, n).astype(np.int32), "INT")
        t["f"] = (rng.integers(0, 1000, n).astype(np.int32), "INT")
        # a few hot keys so that slots see repeated hits
        t["g1"][0][: n // 10] = 5
        t["g2"][0][: n // 10] = 7
        t["g3"][0][: n // 10] = 11
        tables.append(t)
    sql = (f"SET numGroupsLimit=10000000; SELECT g1, g2, g3, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t{where} "
           f"GROUP BY g1, g2, g3 ORDER BY g1, g2, g3 LIMIT 10000000")
    r, got = _both(ctx, tables, sql)
    assert r.stats.mode == 5  # MODE_GROUP_HASH
    assert not r.stats.num_groups_limit_reached
    assert len(got.rows) > (300_000 if not where else 100_000)


@pytest.mark.parametrize("where", ["", " WHERE f < 300"])
def test_hash_group_by_hll(ctx, where):
    # DISTINCTCOUNTHLL per group over a key space beyond the dense budget: MODE_GROUP_HASH with 2^log2m registers
    # per slot (DistinctCountHLLAggregationFunction over the map-based group key holders); registers compared raw
    rng = np.random.default_rng(37)
    tables = []
    for n in (200_000, 77_777):
        t = {c: (rng.integers(0, 12_000, n).astype(np.int32) * 3 + k, "INT") for k, c in enumerate(("g1", "g2", "g3"))}
        t["g1"][0][: n // 4] = 5  # hot keys with many distinct u per group
        t["g2"][0][: n // 4] = 7
        t["g3"][0][: n // 4] = 11
        t["u"] = (rng.integers(0, 1 << 24, n).astype(np.int32), "INT")
        t["f"] = (rng.integers(0, 1000, n).astype(np.int32), "INT")
        tables.append(t)
    sql = (f"SET numGroupsLimit=10000000; SELECT g1, g2, g3, DISTINCTCOUNTHLL(u), COUNT(*) FROM t{where} "
           f"GROUP BY g1, g2, g3 ORDER BY g1, g2, g3 LIMIT 10000000")
    r, got = _both(ctx, tables, sql)
    assert r.stats.mode == 5  # MODE_GROUP_HASH
    assert len(got.rows) > 50_000


@pytest.mark.parametrize("where", ["", " WHERE f < 300", " WHERE f IN (1, 5, 9, 300, 301, 777) OR g1 < 9000"])
def test_hash_group_by_num_groups_limit(ctx, where):
    # numGroupsLimit over a key space beyond the dense budget (LongMapBasedHolder.getGroupId,
    # DictionaryBasedGroupKeyGenerator.java:629-637): the reference's DEFAULT limit of 100 000 on a ~1.7e12 key
    # space -- each segment keeps its first 100 000 keys in doc order and drops the docs of later keys; one small
    # segment cannot reach the limit and aggregates everything.  Bit-exact vs the oracle's IntGroupIdMap emulation.
    rng = np.random.default_rng(seed_of(f"hash-limit{where}"))
    tables = []
    for n in (500_000, 180_001, 40_000):  # the first segment matches > 100 000 keys under every filter
        t = {c: (rng.integers(0, 12_000, n).astype(np.int32) * 3 + k, "INT") for k, c in enumerate(("g1", "g2", "g3"))}
        t["m"] = (rng.integers(-1 << 20, 1 << 30, n).astype(np.int32), "INT")
        t["f"] = (rng.integers(0, 1000, n).astype(np.int32), "INT")
        t["g1"][0][: n // 10] = 5  # hot keys
        t["g2"][0][: n // 10] = 7
        tables.append(t)
    sql = (f"SELECT g1, g2, g3, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t{where} "
           f"GROUP BY g1, g2, g3 ORDER BY g1, g2, g3 LIMIT 10000000")
    q = parse_sql(sql)
    r, got = _both(ctx, tables, sql)
    e = O.execute(q, [O.build_segment(f"s{i}", t) for i, t in enumerate(tables)])
    assert r.stats.mode == 5  # MODE_GROUP_HASH
    assert e.stats.num_groups_limit_reached  # the oracle truncated: the case tests what it means to
    assert r.stats.num_groups_limit_reached
    assert r.stats.limit_pass == 2
    assert r.stats.num_docs_scanned == e.stats.num_docs_scanned


def test_remap_cache_bounded_over_segment_subsets(ctx):
    # without a table dictionary every distinct segment set unions its own dictionary, and each segment gets a
    # device remap to it; the union cache is a bounded FIFO (64 entries) and a segment's remaps must be released
    # with their union (they accumulated without bound)
    import itertools
    rng = np.random.default_rng(8)
    segs = []
    for i in range(9):
        vals = rng.choice(4000, 3000, replace=False).astype(np.int32)  # each segment its own value set
        t = {"g": (vals[rng.integers(0, 3000, 20_000)], "INT"),
             "m": (rng.integers(0, 100, 20_000).astype(np.int32), "INT")}
        segs.append(ctx.pin(create_segment(f"rm{i}", t)))
    ctx.execute(parse_sql("SELECT SUM(m) FROM t"), segs)  # value-stream caches, counted in device_bytes too
    base = sum(s.device_bytes for s in segs)
    q = parse_sql("SET numGroupsLimit=1000000; SELECT g, COUNT(*), SUM(m) FROM t GROUP BY g LIMIT 1000000")
    subsets = list(itertools.combinations(range(9), 3)) + list(itertools.combinations(range(9), 4))  # 84 + 126
    for sub in subsets:
        ctx.execute(q, [segs[i] for i in sub])
    # live remaps: at most the 64 cached unions x 4 segments each
    grown = sum(s.device_bytes for s in segs) - base
    per_remap = 3000 * 4
    assert 0 < grown <= (64 + 1) * 4 * per_remap, grown
    for s in segs:
        s.unpin()


@pytest.mark.parametrize("case", ["few", "many", "exact", "filtered", "three_cols"])
def test_num_groups_limit_first_seen(ctx, case):
    # DictionaryBasedGroupKeyGenerator keeps the first numGroupsLimit keys of each segment in doc order and drops
    # the docs of later keys (IntGroupIdMap.getGroupId :992-1017); numGroupsLimitReached = numGroups >= limit
    # (GroupByOperator.java:111).  Default limit 100 000, 2-column keys with a 1M cardinality product.
    rng = np.random.default_rng(seed_of(case))
    tables = []
    for n in (400_000, 250_003):
        if case == "few":  # 1 000 real groups (g2 follows g1) although the cardinality product is 1M
            g1 = rng.integers(0, 1000, n)
            g2 = (g1 * 7) % 1000
        else:
            g1 = rng.integers(0, 1000, n)
            g2 = rng.integers(0, 1000, n)
        t = {"g1": (g1.astype(np.int32), "INT"), "g2": (g2.astype(np.int32), "INT"),
             "m": (rng.integers(-1000, 1 << 20, n).astype(np.int32), "INT"),
             "f": (rng.integers(0, 100, n).astype(np.int32), "INT")}
        if case == "three_cols":
            t["g3"] = (rng.integers(0, 7, n).astype(np.int32), "INT")
        tables.append(t)
    # every value present in every segment, so dictionaries (and their cardinality products) are complete
    for t in tables:
        for c in ("g1", "g2"):
            v = t[c][0]
            v[:1000] = np.arange(1000) if c == "g1" or case != "few" else (np.arange(1000) * 7) % 1000
    limit = {"exact": 2500, "few": None, "many": None, "filtered": 30_000, "three_cols": 50_000}[case]
    opt = f"SET numGroupsLimit={limit}; " if limit else ""
    where = " WHERE f < 40" if case == "filtered" else ""
    cols = "g1, g2, g3" if case == "three_cols" else "g1, g2"
    sql = (f"{opt}SELECT {cols}, COUNT(*), SUM(m), MAX(m) FROM t{where} GROUP BY {cols} ORDER BY {cols} "
           f"LIMIT 2000000")
    q = parse_sql(sql)
    r, _ = _both(ctx, tables, sql)
    e = O.execute(q, [O.build_segment(f"s{i}", t) for i, t in enumerate(tables)])
    assert r.stats.num_groups_limit_reached == e.stats.num_groups_limit_reached
    if case in ("many", "filtered", "three_cols"):
        assert r.stats.num_groups_limit_reached
        assert r.stats.limit_pass == 2  # truncation ran: the first-seen pass and the rescan
    if case == "few":  # 1 000 real keys under a product of 1M >= limit: the optimistic scan suffices, no pass
        assert not r.stats.num_groups_limit_reached and r.stats.limit_pass == 1


@pytest.mark.parametrize("where", ["", " WHERE a IN (3, 5, 7, 11, 400, 1999) AND m > 100", " WHERE b NOT IN (3, 4)",
                                   " WHERE (a = 3 OR a = 1999) AND m > 100"])
@pytest.mark.parametrize("eager", [False, True])
def test_num_groups_limit_product_above_real_keys(ctx, eager, where, monkeypatch):
    # a cardinality product far above the limit but fewer real keys than the limit: numGroupsLimitReached stays
    # false and the result is the untruncated group-by (optimistic form: no first-seen pass at all); the
    # pass-first order (PH_LIMIT_EAGER) gives the same answer.  The filtered forms put a bitset leaf in the scan
    # (FK_CONJ set leaf, FK_SET): r3's optimistic scan read a segment table copied before those device bitsets
    # were attached, and filtered SSB Q3.3 / Q3.4 returned a fraction of their groups
    if eager:
        monkeypatch.setenv("PH_LIMIT_EAGER", "1")
    rng = np.random.default_rng(seed_of("product_above_real_keys"))
    tables = []
    for n in (300_000, 200_001):
        a = rng.integers(0, 2000, n).astype(np.int32)
        b = ((a * 13 + rng.integers(0, 3, n)) % 1500).astype(np.int32)  # ~6000 real (a, b) keys of 3M
        b[:1500] = np.arange(1500)  # every b value present: cardinality product 2000 x 1500 per segment
        a[:2000] = np.arange(2000)
        tables.append({"a": (a, "INT"), "b": (b, "INT"),
                       "m": (rng.integers(-50, 1 << 18, n).astype(np.int32), "INT")})
    sql = (f"SET numGroupsLimit=20000; SELECT a, b, COUNT(*), SUM(m), MIN(m) FROM t{where} GROUP BY a, b "
           f"ORDER BY a, b LIMIT 100000")
    r, _ = _both(ctx, tables, sql)
    q = parse_sql(sql)
    e = O.execute(q, [O.build_segment(f"s{i}", t) for i, t in enumerate(tables)])
    assert not r.stats.num_groups_limit_reached and not e.stats.num_groups_limit_reached
    assert r.num_groups < 20000
    assert r.stats.limit_pass == (2 if eager else 1)


@pytest.mark.parametrize("shape", ["pruned", "empty"])
def test_group_by_with_nothing_to_scan_fresh_context(shape):
    # a plain group-by (deferred-sync result path) whose filter prunes every segment / whose segments are empty,
    # on a fresh context (fresh lanes: no event was ever recorded): 0 groups, device_ms 0, no error
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    try:
        n = 0 if shape == "empty" else 5000
        rng = np.random.default_rng(seed_of(shape))
        cols = {"g": (rng.integers(0, 50, n).astype(np.int32), "INT"),
                "m": (rng.integers(0, 100, n).astype(np.int32), "INT")}
        segs = [c.pin(create_segment(f"e{i}", cols)) for i in range(3)]
        where = " WHERE m > 1000" if shape == "pruned" else ""
        sql = f"SELECT g, COUNT(*), SUM(m) FROM t{where} GROUP BY g ORDER BY g LIMIT 100"
        r = c.execute(parse_sql(sql), segs)
        assert r.num_groups == 0 and r.stats.num_docs_scanned == 0 and r.stats.device_ms == 0.0
        r2 = c.execute(parse_sql(sql), segs)  # the same lane again
        assert r2.num_groups == 0 and r2.stats.device_ms == 0.0
    finally:
        c.close()


def test_bad_query_is_reported(ctx, sv):
    from pinot_amd.native import BadQueryError
    with pytest.raises(BadQueryError):
        ctx.execute(parse_sql("SELECT COUNT(*) FROM t WHERE nope = 3"), sv)
    with pytest.raises(BadQueryError):
        ctx.execute(parse_sql("SELECT COUNT(*) FROM t WHERE column1 > 'abc'"), sv)


# ------------------------------------------------------------------ partitioned group-by (MODE_PARTITION)
def _big_key_table(rng, n, c1=1000, c2=300, mbits=20, skew=0.0):
    g1 = rng.integers(0, c1, n).astype(np.int32)
    g2 = rng.integers(0, c2, n).astype(np.int32)
    if skew:
        hot = rng.random(n) < skew
        g1[hot] = 7
        g2[hot] = 3
    return {"g1": (g1, "INT"), "g2": (g2, "INT"),
            "m": (rng.integers(-(1 << (mbits - 1)), 1 << (mbits - 1), n).astype(np.int32), "INT"),
            "f": (rng.integers(0, 1000, n).astype(np.int32), "INT")}


PART_SQL = ("SET numGroupsLimit=2000000; SELECT g1, g2, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t "
            "WHERE f BETWEEN 0 AND 499 GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 2000000")


@pytest.fixture
def small_batches(monkeypatch):
    monkeypatch.setenv("PH_PART_BATCH_ROWS", "100000")


def test_partition_multi_batch(ctx, small_batches):
    rng = np.random.default_rng(21)
    tables = [_big_key_table(rng, n) for n in (300_000, 250_001, 64 * 999)]
    r, _ = _both(ctx, tables, PART_SQL)
    assert r.stats.mode == 4


def test_partition_overflow_skew(ctx, small_batches):
    rng = np.random.default_rng(22)
    tables = [_big_key_table(rng, 400_000, skew=0.6), _big_key_table(rng, 100_000, skew=0.9)]
    r, _ = _both(ctx, tables, PART_SQL)
    assert r.stats.mode == 4


def test_partition_wide_records(ctx):
    # value range needs 30 bits: key_lo + value bits > 32 -> 64-bit records
    rng = np.random.default_rng(23)
    tables = [_big_key_table(rng, 300_000, mbits=30)]
    r, _ = _both(ctx, tables, PART_SQL)
    assert r.stats.mode == 4


def test_partition_count_only_and_no_filter(ctx, small_batches):
    rng = np.random.default_rng(24)
    tables = [_big_key_table(rng, 200_000), _big_key_table(rng, 150_000)]
    r, _ = _both(ctx, tables, "SET numGroupsLimit=2000000; SELECT g1, g2, COUNT(*) FROM t GROUP BY g1, g2 "
                              "ORDER BY g1, g2 LIMIT 2000000")
    assert r.stats.mode == 4
    _both(ctx, tables, "SET numGroupsLimit=2000000; SELECT g2, g1, MAX(m) FROM t WHERE f < 100 GROUP BY g2, g1 "
                       "ORDER BY g2, g1 LIMIT 2000000")


def test_global_table_two_value_columns(ctx):
    rng = np.random.default_rng(25)
    t = _big_key_table(rng, 200_000)
    t["d"] = (np.round(rng.normal(size=200_000), 4), "DOUBLE")
    r, _ = _both(ctx, [t], "SET numGroupsLimit=2000000; SELECT g1, g2, SUM(m), SUM(d), MIN(d) FROM t "
                           "GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 2000000")
    assert r.stats.mode == 3


def test_value_stream_reencoding_wide_values(ctx):
    # INT metric spanning the full int32 range: frame-of-reference needs 32 bits -> dictionary gather path
    rng = np.random.default_rng(26)
    m = rng.integers(-2**31, 2**31 - 1, 50_000, dtype=np.int64).astype(np.int32)
    m[:2] = [-2**31, 2**31 - 1]
    t = {"m": (m, "INT"), "a": (rng.integers(0, 5, 50_000).astype(np.int32), "INT")}
    _both(ctx, [t], "SELECT a, SUM(m), MIN(m), MAX(m) FROM t GROUP BY a ORDER BY a")
    t2 = {"m": (rng.integers(-2**40, 2**40, 50_000, dtype=np.int64), "LONG"),
          "a": (rng.integers(0, 5, 50_000).astype(np.int32), "INT")}
    _both(ctx, [t2], "SELECT a, SUM(m), MIN(m), MAX(m) FROM t GROUP BY a ORDER BY a")


# AND of scan leaves on different columns (FK_CONJ: every leaf decoded from its own staged stream), including
# same-column ORs / ANDs merged into one leaf (sets, ranges, contiguous sets -> ranges), exclusive sets, a leaf
# that is always true and an AND that matches nothing -- no inverted indexes, so every leaf is a scan
CONJ_FILTERS = [
    " WHERE a = 3 AND b > 0",
    " WHERE b BETWEEN -500 AND 250 AND m < 536870912 AND s IN (3, 7, 30)",
    " WHERE (a = 1 OR a = 5) AND (str = 'gFuH' OR str = 't') AND b >= -100",
    " WHERE b >= -100 AND b <= 300 AND a <> 2",
    " WHERE a NOT IN (0, 6) AND str > 'o' AND d > 0.5 AND c < 0",
    " WHERE a = 99 AND b > 0",
    " WHERE a >= 0 AND b > 0",
    " WHERE (a = 1 OR a = 2 OR a = 3) AND s BETWEEN 10 AND 20",
]


@pytest.mark.parametrize("where", CONJ_FILTERS)
@pytest.mark.parametrize("group", ["", "a, str", "s", "b"])
def test_conjunctive_scan_leaves(ctx, where, group):
    rng = np.random.default_rng(seed_of(where + group))
    tables = [_random_table(rng, n) for n in (12_345, 64 * 500 + 3)]
    if group:
        sql = (f"SET numGroupsLimit=10000000; SELECT {group}, COUNT(*), SUM(m), MIN(d), MAX(b) FROM t{where} "
               f"GROUP BY {group} ORDER BY {group} LIMIT 100000")
    else:
        sql = "SELECT COUNT(*), SUM(m), MIN(b), MAX(b), SUM(d), SUM(m * b) FROM t" + where
    _both(ctx, tables, sql, inverted=())


# MODE_GROUP_GLOBAL's per-workgroup LDS group cache (one value column): keys that all fit the cache, key spaces
# that overflow it (spilled keys go straight to the HBM table), integer and DOUBLE values with SUM / MIN / MAX,
# selective and unfiltered; a numGroupsLimit that truncates runs through the same path
@pytest.mark.parametrize("sql", [
    "SET numGroupsLimit=10000000; SELECT b, c, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE a < 4 GROUP BY b, c "
    "ORDER BY b, c LIMIT 1000000",
    "SET numGroupsLimit=10000000; SELECT b, c, SUM(d), MIN(d), MAX(d) FROM t GROUP BY b, c ORDER BY b, c LIMIT 1000000",
    "SET numGroupsLimit=10000000; SELECT a, b, COUNT(*), SUM(m) FROM t WHERE s > 25 GROUP BY a, b ORDER BY a, b "
    "LIMIT 1000000",
    "SET numGroupsLimit=300; SELECT b, c, COUNT(*), SUM(m) FROM t WHERE a IN (1, 2) AND m > 0 GROUP BY b, c "
    "ORDER BY b, c LIMIT 1000000",
])
def test_group_cache_global_table(ctx, sql):
    rng = np.random.default_rng(seed_of(sql))
    tables = [_random_table(rng, n) for n in (40_000, 64 * 700 + 9)]
    _both(ctx, tables, sql, inverted=())


@pytest.mark.parametrize("where", ["(a = 3 OR a = 17) AND (b = 5 OR b = 9) AND m > 0",
                                   "a IN (3, 17, 30) AND b BETWEEN 2 AND 20 AND m > 0"])
def test_conj_set_leaf_merged_from_equalities(ctx, where):
    # FK_CONJ with a set leaf merged from same-column EQ leaves (SSB Q3.3 / Q3.4's `c_city = .. OR c_city = ..`),
    # on a small key space (no numGroupsLimit pass): the set must be read as a bitset (r3: it kept the first EQ's
    # single-id range and the gathering kernel was not selected -> only that id matched)
    rng = np.random.default_rng(seed_of(where))
    tables = [{"a": (rng.integers(0, 40, n).astype(np.int32), "INT"), "b": (rng.integers(0, 30, n).astype(np.int32), "INT"),
               "m": (rng.integers(-100, 1000, n).astype(np.int32), "INT")} for n in (200_000, 77_777)]
    _both(ctx, tables, f"SELECT a, b, COUNT(*), SUM(m) FROM t WHERE {where} GROUP BY a, b ORDER BY a, b LIMIT 1000")


@pytest.mark.parametrize("inverted", [(), ("c",)])
def test_in_lists_with_repeats_and_absent_values(ctx, inverted):
    # InPredicateEvaluatorFactory: the literals' dictIds as a set -- repeated literals and literals outside the
    # dictionary change nothing; NOT IN of every value is alwaysFalse, IN of every value alwaysTrue
    rng = np.random.default_rng(seed_of("in-repeats"))
    cols = [{"c": (rng.integers(0, 6, n).astype(np.int32), "INT"), "g": (rng.integers(0, 9, n).astype(np.int32), "INT"),
             "m": (rng.integers(-100, 100, n).astype(np.int32), "INT")} for n in (3000, 1777)]
    for where in ("c IN (3, 3, 1, 3, 99)", "c NOT IN (2, 2, -7, 5)", "c IN (0, 1, 2, 3, 4, 5, 5)",
                  "c NOT IN (0, 1, 2, 3, 4, 5)", "c IN (4, 4) AND g IN (1, 8, 8, 1)", "c IN (77, 78)"):
        _both(ctx, cols, f"SELECT g, COUNT(*), SUM(m) FROM t WHERE {where} GROUP BY g ORDER BY g LIMIT 100",
              inverted=inverted)
        _both(ctx, cols, f"SELECT COUNT(*), MIN(m), MAX(m) FROM t WHERE {where}", inverted=inverted)
