"""CPU: the segment-directory writer/reader used by the loader tests, on the reference's own V1 segment and on
V3 / V1 directories written from create_segment output (the GPU side is tests/test_gpu_loader.py)."""
import os

import numpy as np

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment
from tests import segment_dirs as SD

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_reference_v1_segment_reads():
    # paddingNull: 5 docs written by the reference (NUL string padding)
    seg, meta = SD.read_dir(os.path.join(GOLD, "v1_paddingNull"))
    assert seg.num_docs == 5 and meta["segment.name"] == "mySegment_0"
    assert list(seg.columns["name"].dictionary) == ["lynda", "lynda 2.0"]
    assert list(seg.columns["age"].dictionary) == [617, 824, 837, 1209, 1228]
    q = parse_sql("SELECT name, COUNT(*), SUM(age), MIN(outgoingName1), MAX(percent) FROM t GROUP BY name "
                  "ORDER BY name LIMIT 10")
    e = O.execute(q, [seg])
    rows = reduce_groups(q, e.keys, e.aggs).rows
    assert [r[0] for r in rows] == ["lynda", "lynda 2.0"] and sum(r[1] for r in rows) == 5


def test_v3_and_v1_round_trip(tmp_path):
    rng = np.random.default_rng(5)
    n = 50_000
    cols = {"a": (rng.integers(0, 50, n).astype(np.int32), "INT"),
            "s": (np.sort(rng.integers(0, 30, n)).astype(np.int32), "INT"),
            "x.y": (rng.integers(-10**12, 10**12, n).astype(np.int64), "LONG"),
            "d": (np.round(rng.normal(0, 10, n), 2), "DOUBLE"),
            "str": (np.array(["p", "qq", "", "zzz"])[rng.integers(0, 4, n)], "STRING")}
    buf = create_segment("rt", cols, inverted=("a",))
    SD.write_v3(buf, str(tmp_path / "v3seg"))
    SD.write_v1(buf, str(tmp_path / "v1seg"))
    q = parse_sql("SELECT a, str, COUNT(*), SUM(x.y), MIN(d), MAX(s) FROM t WHERE s BETWEEN 3 AND 20 "
                  "GROUP BY a, str ORDER BY a, str LIMIT 100000")
    exp = O.execute(q, [O.build_segment("rt", cols)])
    exp_rows = reduce_groups(q, exp.keys, exp.aggs).rows
    for d in ("v3seg", "v1seg"):
        seg, _ = SD.read_dir(str(tmp_path / d))
        e = O.execute(q, [seg])
        assert reduce_groups(q, e.keys, e.aggs).rows == exp_rows, d


# ------------------------------------------------------------------ index_map pinned by the reference's own file
REF_INDEX_MAP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "startree_segment", "index_map")


def _expected_index_map(path):
    """ColumnIndexUtils.parseIndexMapKeys restated (split from the right) over java.util.Properties lines."""
    out = {}
    for line in open(path, encoding="utf-8"):
        t = line.strip()
        if not t or t[0] in "#!":
            continue
        k, v = [x.strip() for x in t.split("=", 1)]
        a = k.rindex(".")
        b = k.rindex(".", 0, a)
        e = out.setdefault((k[:b], k[b + 1:a]), [0, 0])
        e[0 if k[a + 1:] == "startOffset" else 1] = int(v)
    return out


def _lookup(path, col, idx):
    import ctypes
    from pinot_amd import native as N
    start, size = ctypes.c_int64(-1), ctypes.c_int64(-1)
    rc = N.lib().ph_index_map_lookup(path.encode(), col.encode(), idx.encode(), ctypes.byref(start), ctypes.byref(size))
    return rc, start.value, size.value


def test_index_map_reference_file():
    # pinot-segment-local/src/test/resources/data/startree/segment/index_map (a reference-written V3 index_map,
    # committed as tests/golden/startree_segment/index_map): every (column, index) entry the loader resolves
    exp = _expected_index_map(REF_INDEX_MAP)
    assert len(exp) == 172 and ("$ts$DAY", "range_index") in exp
    for (col, idx), (start, size) in exp.items():
        assert _lookup(REF_INDEX_MAP, col, idx) == (0, start, size), (col, idx)
    assert _lookup(REF_INDEX_MAP, "$ts$DAY", "inverted_index")[0] == 2  # PH_ERR_BAD_QUERY: no such entry


def test_index_map_dotted_column_and_malformed_keys(tmp_path):
    p = tmp_path / "index_map"
    p.write_text("# comment\ncol.with.dots.dictionary.startOffset = 8\ncol.with.dots.dictionary.size : 24\n"
                 "plain.forward_index.startOffset=32\nplain.forward_index.size=100\n")
    assert _lookup(str(p), "col.with.dots", "dictionary") == (0, 8, 24)
    assert _lookup(str(p), "plain", "forward_index") == (0, 32, 100)
    for bad in ("nodots = 3\n", "one.dot = 3\n", "c.i.startOffset = 12x\n"):
        p.write_text(bad)
        assert _lookup(str(p), "c", "i")[0] == 1  # PH_ERR_INVALID_ARGUMENT (Preconditions.checkState / bad number)
    assert _lookup(str(tmp_path / "missing"), "c", "i")[0] == 1
