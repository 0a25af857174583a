"""GPU: ph_segment_load_dir (segment directories pinned straight from disk) against the CPU oracle.

* the reference's own V1 segment (tests/golden/v1_paddingNull, written by the reference's segment creator);
* V3 (columns.psf + index_map, a column name with a dot) and V1 directories written from create_segment output
  (tests/segment_dirs.py), including sorted and inverted-index columns -- results equal to pinning the same
  buffers through ph_segment_pin and to the oracle over an independent reader of the directory;
* a segment without zero string padding (tests/golden/v1_paddingOld, as the reference) and missing columns are
  refused.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import create_segment
from tests import segment_dirs as SD

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _rows(ctx, segs, q):
    r = ctx.execute(q, segs)
    return reduce_groups(q, r.keys, r.aggs).rows, r


def test_reference_v1_segment(ctx):
    path = os.path.join(GOLD, "v1_paddingNull")
    seg = ctx.load_segment_dir(path)
    assert seg.num_docs == 5
    ora, _ = SD.read_dir(path)
    for sql in ("SELECT name, COUNT(*), SUM(age), MIN(outgoingName1), MAX(percent) FROM t GROUP BY name "
                "ORDER BY name LIMIT 10",
                "SELECT COUNT(*), SUM(age), MAX(outgoingName1) FROM t WHERE name = 'lynda 2.0'",
                "SELECT age, COUNT(*) FROM t WHERE percent > 400 GROUP BY age ORDER BY age LIMIT 10"):
        q = parse_sql(sql)
        got, _ = _rows(ctx, [seg], q)
        e = O.execute(q, [ora])
        assert got == reduce_groups(q, e.keys, e.aggs).rows, sql


def test_legacy_padding_refused(ctx):
    # no segment.padding.character: a pre-2016 '%'-padded segment, which the reference refuses to load
    # (ColumnMetadataImpl.java:297-300)
    from pinot_amd.native import PinotHipError
    with pytest.raises(PinotHipError, match="non-zero string padding"):
        ctx.load_segment_dir(os.path.join(GOLD, "v1_paddingOld"))


@pytest.mark.parametrize("layout", ["v3", "v1"])
def test_written_directories(ctx, tmp_path, layout):
    rng = np.random.default_rng(17)
    n = 400_000
    cols = {"a": (rng.integers(0, 50, n).astype(np.int32), "INT"),
            "s": (np.sort(rng.integers(0, 30, n)).astype(np.int32), "INT"),
            "x.y": (rng.integers(-10**12, 10**12, n).astype(np.int64), "LONG"),
            "m": (rng.integers(0, 1 << 20, n).astype(np.int32), "INT"),
            "d": (np.round(rng.normal(0, 10, n), 2), "DOUBLE"),
            "str": (np.array(["p", "qq", "", "zzz"])[rng.integers(0, 4, n)], "STRING")}
    buf = create_segment("dirseg", cols, inverted=("a", "str"))
    path = str(tmp_path / layout)
    (SD.write_v3 if layout == "v3" else SD.write_v1)(buf, path)
    from_dir = ctx.load_segment_dir(path)
    pinned = ctx.pin(buf)
    assert from_dir.num_docs == n
    ora, _ = SD.read_dir(path)
    for sql in ("SELECT a, str, COUNT(*), SUM(x.y), MIN(d), MAX(s) FROM t WHERE s BETWEEN 3 AND 20 "
                "GROUP BY a, str ORDER BY a, str LIMIT 100000",
                "SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t WHERE a IN (1, 7, 30) AND str <> 'qq'",
                "SELECT COUNT(*) FROM t WHERE s = 4",
                "SELECT DISTINCTCOUNTHLL(m) FROM t WHERE a < 10"):
        q = parse_sql(sql)
        got, _ = _rows(ctx, [from_dir], q)
        ref, _ = _rows(ctx, [pinned], q)
        e = O.execute(q, [ora])
        exp = reduce_groups(q, e.keys, e.aggs).rows
        assert got == ref, sql
        for g, x in zip(got, exp):
            for a, b in zip(g, x):
                assert a == b or (isinstance(b, float) and abs(a - b) <= 1e-9 * abs(b)), (sql, g, x)
    # a subset of the columns only
    part = ctx.load_segment_dir(path, ["a", "m"])
    q = parse_sql("SELECT a, SUM(m) FROM t GROUP BY a ORDER BY a LIMIT 100")
    assert _rows(ctx, [part], q)[0] == _rows(ctx, [pinned], q)[0]
    from pinot_amd.native import PinotHipError
    with pytest.raises(PinotHipError):
        ctx.load_segment_dir(path, ["nope"])
