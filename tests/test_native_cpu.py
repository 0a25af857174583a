"""CPU-only checks of the product library and host logic (no GPU compute calls)."""
import os
import re

import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd import native as N
from pinot_amd.query import parse_sql
from pinot_amd.segment import (build_inverted_index, create_column, fixed_bit_pack, num_bits_per_value,
                               roaring_serialize)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    header = open(os.path.join(ROOT, "include", "pinot_hip.h")).read()
    declared = set(re.findall(r"^\s*(?:int|int64_t|int32_t|const char\*|const void\*)\s+(ph_\w+)\(", header, re.M))
    assert declared == set(N.EXPORTED_SYMBOLS)
    L = N.lib()
    for s in declared:
        assert hasattr(L, s), s
    assert b"gfx950" in L.ph_version()


def test_no_gpu_is_reported_not_faked():
    import ctypes
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = ctypes.c_void_p()
    code = N.lib().ph_ctx_create(0, ctypes.byref(h))
    assert code == N.PH_ERR_DEVICE
    assert b"device" in N.lib().ph_last_error().lower()


@pytest.mark.parametrize("bits", list(range(1, 32)))
def test_product_packer_matches_oracle_writer(bits):
    rng = np.random.default_rng(100 + bits)
    for n in (1, 31, 32, 33, 95, 1000, 70_001):
        ids = rng.integers(0, 1 << bits, n, dtype=np.int64).astype(np.int32)
        a = fixed_bit_pack(ids, bits)
        b = O.fixed_bit_pack(ids, bits)
        assert np.array_equal(a, b), (bits, n)


def test_packer_parallel_path_large():
    rng = np.random.default_rng(5)
    ids = rng.integers(0, 1 << 20, 5_000_003, dtype=np.int64).astype(np.int32)
    a = fixed_bit_pack(ids, 20)
    assert np.array_equal(O.fixed_bit_unpack(a, len(ids), 20), ids)


def test_num_bits_matches_oracle():
    for v in list(range(0, 600)) + [2**k - 1 for k in range(1, 32)] + [2**k for k in range(1, 31)]:
        assert num_bits_per_value(v) == O.num_bits_per_value(v)


def _roaring_decode(blob: bytes) -> np.ndarray:
    """Independent decoder of the portable format (RoaringFormatSpec) for the writer's self-check."""
    b = np.frombuffer(blob, np.uint8)
    cookie = int.from_bytes(blob[0:4], "little")
    pos = 4
    runflags = None
    if cookie & 0xFFFF == 12347:
        size = (cookie >> 16) + 1
        runflags = blob[pos:pos + (size + 7) // 8]
        pos += (size + 7) // 8
        has_off = size >= 4
    else:
        assert cookie == 12346
        size = int.from_bytes(blob[4:8], "little")
        pos = 8
        has_off = True
    desc = np.frombuffer(blob[pos:pos + 4 * size], "<u2").reshape(size, 2)
    pos += 4 * size
    offs = np.frombuffer(blob[pos:pos + 4 * size], "<u4") if has_off else None
    if has_off:
        pos += 4 * size
    out = []
    for i in range(size):
        key, card = int(desc[i, 0]), int(desc[i, 1]) + 1
        at = int(offs[i]) if has_off else pos
        is_run = runflags is not None and (runflags[i // 8] >> (i % 8)) & 1
        if is_run:
            nr = int.from_bytes(blob[at:at + 2], "little")
            r = np.frombuffer(blob[at + 2:at + 2 + 4 * nr], "<u2").reshape(nr, 2)
            for s, l in r:
                out.append((key << 16) + np.arange(int(s), int(s) + int(l) + 1))
            pos = at + 2 + 4 * nr
        elif card <= 4096:
            out.append((key << 16) + np.frombuffer(blob[at:at + 2 * card], "<u2").astype(np.int64))
            pos = at + 2 * card
        else:
            words = np.frombuffer(blob[at:at + 8192], "<u8")
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")
            out.append((key << 16) + np.flatnonzero(bits))
            pos = at + 8192
    return np.concatenate(out) if out else np.zeros(0, np.int64)


@pytest.mark.parametrize("run_opt", [False, True])
def test_roaring_writer_round_trip(run_opt):
    rng = np.random.default_rng(11)
    cases = [np.array([], np.int64), np.arange(5), np.arange(0, 200000, 3), np.arange(65530, 65600),
             np.sort(rng.choice(10_000_000, 5000, replace=False)), np.arange(1 << 16, 1 << 18)]
    for docs in cases:
        blob = roaring_serialize(docs, run_opt)
        assert np.array_equal(_roaring_decode(blob), docs)


def test_inverted_index_layout():
    ids = np.array([2, 0, 1, 2, 2, 0], np.int32)
    inv = build_inverted_index(ids, 3)
    offs = np.frombuffer(inv[:16].tobytes(), ">u4")
    assert offs[0] == 16 and offs[-1] == len(inv)
    for d in range(3):
        blob = inv[offs[d]:offs[d + 1]].tobytes()
        assert _roaring_decode(blob).tolist() == np.flatnonzero(ids == d).tolist()


def test_column_buffers_sorted_and_dictionary():
    c = create_column("s", np.array([3, 3, 5, 7, 7, 7]), "INT")
    assert c.is_sorted and c.cardinality == 3
    pairs = np.frombuffer(c.forward_index.tobytes(), ">i4").reshape(-1, 2).tolist()
    assert pairs == [[0, 1], [2, 2], [3, 5]]
    assert np.frombuffer(c.dictionary.tobytes(), ">i4").tolist() == [3, 5, 7]
    s = create_column("str", np.array(["b", "", "abc", "b"]), "STRING")
    assert s.entry_size == 3 and not s.is_sorted
    assert bytes(s.dictionary[:3]) == b"\x00\x00\x00" and bytes(s.dictionary[3:6]) == b"abc"


def test_sql_parser_shapes():
    q = parse_sql("SET numGroupsLimit=2000000; SELECT g1, g2, SUM(m), COUNT(*), MIN(m), MAX(m) FROM t "
                  "WHERE f BETWEEN 0 AND 499 GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 2000000")
    assert q.num_groups_limit == 2000000 and q.group_by == ["g1", "g2"] and q.limit == 2000000
    assert [a.function for a in q.aggregations] == ["SUM", "COUNT", "MIN", "MAX"]
    q = parse_sql("SELECT COUNT(*) FROM t WHERE a NOT IN ('x', 'y') AND (b < 3 OR NOT c = 'q')")
    assert q.filter.type == "AND" and q.filter.children[1].type == "OR"


def test_expression_result_column_names():
    # AggregationFunction.getResultColumnName over the parser's canonical expression names (CalciteSqlParser.java:798:
    # SqlKind TIMES / MINUS / PLUS), the names datatable.cpp's agg_column_name writes into the DataTable schema
    q = parse_sql("SELECT SUM(a * b), SUM(a - b), MAX(a + b), COUNT(*), SUM(a) FROM t")
    assert q.result_columns() == ["sum(times(a,b))", "sum(minus(a,b))", "max(plus(a,b))", "count(*)", "sum(a)"]


def test_segment_group_trim_gate():
    # minSegmentGroupTrimSize > 0 with ORDER BY runs on the GPU path (per-segment tables + the TableResizer heap,
    # trim.cpp), an ORDER BY over DISTINCTCOUNTHLL included (by each group's HyperLogLog.cardinality())
    from pinot_amd.engine import check_plan_supported
    from pinot_amd.query import parse_sql
    base = "SELECT a, SUM(m) FROM t GROUP BY a"
    check_plan_supported(parse_sql("SET minSegmentGroupTrimSize=100; " + base + " ORDER BY SUM(m) DESC LIMIT 5"))
    check_plan_supported(parse_sql("SET minSegmentGroupTrimSize=100; SELECT a, DISTINCTCOUNTHLL(m) FROM t "
                                   "GROUP BY a ORDER BY DISTINCTCOUNTHLL(m) DESC LIMIT 5"))
    check_plan_supported(parse_sql("SET minSegmentGroupTrimSize=-1; " + base + " ORDER BY SUM(m) DESC LIMIT 5"))
    check_plan_supported(parse_sql("SET minSegmentGroupTrimSize=100; " + base + " LIMIT 5"))
    check_plan_supported(parse_sql(base + " ORDER BY a LIMIT 5"))


def _desc(num_docs, card, fwd_size, raw=0, name=b"v"):
    import ctypes
    fwd = np.zeros(16, np.uint8)
    dic = np.arange(max(1, min(card, 1 << 16)), dtype=">i4")
    cols = (N.ColumnDesc * 1)()
    d = cols[0]
    d.name = name
    d.data_type = 0
    d.cardinality = card
    d.bits_per_element = num_bits_per_value(card - 1)
    d.forward_index = fwd.ctypes.data
    d.forward_index_size = fwd_size
    d.dictionary = dic.ctypes.data
    d.dictionary_size = dic.nbytes
    d.dictionary_entry_size = 4
    d.raw_forward_index = raw
    desc = N.SegmentDesc(b"big", num_docs, 1, cols)
    return desc, (fwd, dic, cols)


def test_segment_check_refuses_streams_past_2gib():
    # the kernels address a packed stream with 32-bit buffer offsets: a forward index of >= 2 GiB (here 2^31 - 1
    # docs at b = 20: 5.4 GB, declared with a fake length -- the check reads no buffer) is PH_ERR_UNSUPPORTED, so
    # the plan maker keeps the segment on the CPU plan instead of answering from zeros past 2 GiB
    import ctypes
    n = (1 << 31) - 1
    desc, keep = _desc(n, 1 << 20, (n * 20 + 7) // 8)
    assert N.lib().ph_segment_check(ctypes.byref(desc)) == N.PH_ERR_UNSUPPORTED
    assert b"2 GiB" in N.lib().ph_last_error()
    # ... while a raw column passes the check: it is dictionary-encoded at pin, where its stream is sized by the real
    # cardinality (a bound from n distinct values refused large raw columns with small streams)
    desc, keep = _desc(n, 0, 1 << 40, raw=1)
    assert N.lib().ph_segment_check(ctypes.byref(desc)) == 0
    # just below the limit: 858 993 000 docs at 20 bits = 2 147 482 500 bytes - accepted up to the pad
    ok_docs = ((0x7fffffff - 1024 - 4096) * 8) // 20
    desc, keep = _desc(ok_docs, 1 << 20, (ok_docs * 20 + 7) // 8)
    assert N.lib().ph_segment_check(ctypes.byref(desc)) == N.PH_OK
    desc, keep = _desc(ok_docs + 64, 1 << 20, ((ok_docs + 64) * 20 + 7) // 8)
    assert N.lib().ph_segment_check(ctypes.byref(desc)) == N.PH_ERR_UNSUPPORTED
    # malformed: a forward index shorter than its packed size
    desc, keep = _desc(1000, 100, 10)
    assert N.lib().ph_segment_check(ctypes.byref(desc)) == N.PH_ERR_INVALID_ARGUMENT
