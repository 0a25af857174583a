"""GPU: the lean kernels' own decode (LaneStream / lds_value, scan_kernel.h) swept over every stream width 1..31
against the oracle, each query asserting which kernel ran (ph_exec_stats.scan_kernel):

  k_count_reg         COUNT(*) over the filter stream, register-direct decode (filter streams of 1..24 bits)
  k_agg_lean          aggregation only, one packed integer column (value streams of 1..26 bits)
  k_group_reg         LDS group table, register-direct decode, lane-interleaved slots (value streams of 1..31 bits;
                      32 slots per key for 37 keys, 4 for 740 keys, COUNT-only)
  k_group_lds_lean    LDS-private group table (value streams of 1..31 bits)
  k_part_reg          partitioned group-by, register-direct decode (filter streams <= 16 bits; 32-bit records), with
                      one and with two ring sets (part_sets)
  k_part_scan(2)      partitioned group-by, 90 000 keys (value streams of 1..31 bits; 32- and 64-bit records)

The aggregated column's frame-of-reference stream is `w` bits wide (values base + [0, 2^w - 1], both extremes
present) and the filter column's dictId stream min(w, 24) bits wide (a dictionary of 2^(b-1) + 1 values of which
the rows reference a subset), so both the value and the filter decode of every lean kernel see width w.  Segment
lengths are not multiples of a tile.  Bar: bit-exact (COUNT, integer SUM, MIN, MAX, keys)."""
import numpy as np
import pytest

from oracle import oracle as O
from pinot_amd.engine import SCAN_KERNEL_NAMES
from pinot_amd.query import parse_sql
from pinot_amd.reduce import reduce_groups
from pinot_amd.segment import SegmentBuffers, create_column, create_column_from_dict_ids
from tests.seeds import seed_of

pytestmark = pytest.mark.gpu

PH_KERNEL_AGG_LEAN, PH_KERNEL_GROUP_LDS_LEAN, PH_KERNEL_PART_LEAN, PH_KERNEL_PART_LEAN2, PH_KERNEL_PART_REG = 2, 4, 5, 6, 8
PH_KERNEL_COUNT_REG, PH_KERNEL_GROUP_REG = 9, 11


@pytest.fixture(scope="module")
def ctx():
    from pinot_amd.engine import GpuContext
    c = GpuContext(0)
    yield c
    c.close()


def _tables(w):
    rng = np.random.default_rng(seed_of(f"lean-width-{w}"))
    bf = min(w, 24)
    fcard = (1 << (bf - 1)) + 1 if bf > 1 else 2
    out = []
    for n in (70_001, 33_333):
        off = rng.integers(0, 1 << w, n, dtype=np.int64)
        off[:2] = [0, (1 << w) - 1]  # FOR width exactly w
        m = (off - (1 << 30)).astype(np.int64)  # negative and positive values
        fid = rng.integers(0, fcard, n).astype(np.int32)
        fid[:2] = [0, fcard - 1]
        out.append({"m": m, "fid": fid, "fcard": fcard,
                    "g": rng.integers(0, 37, n).astype(np.int32),
                    "g1": rng.integers(0, 300, n).astype(np.int32), "g2": rng.integers(0, 300, n).astype(np.int32),
                    "g3": rng.integers(0, 20, n).astype(np.int32)})
    return out


def _segments(ctx, w):
    gpu, ora = [], []
    for i, t in enumerate(_tables(w)):
        n = len(t["m"])
        seg = SegmentBuffers(f"lw{w}_{i}", n)
        seg.columns["m"] = create_column("m", t["m"], "LONG")
        fdict = np.arange(t["fcard"], dtype=np.int32)
        seg.columns["f"] = create_column_from_dict_ids("f", fdict, t["fid"], "INT", allow_sorted=False)
        for c, card in (("g", 37), ("g1", 300), ("g2", 300), ("g3", 20)):
            t[c][:card] = np.arange(card)  # complete dictionaries
            seg.columns[c] = create_column(c, t[c], "INT")
        gpu.append(ctx.pin(seg))
        ora.append(O.build_segment(seg.name, {"m": (t["m"], "LONG"), "f": (fdict[t["fid"]], "INT"),
                                              "g": (t["g"], "INT"), "g1": (t["g1"], "INT"),
                                              "g2": (t["g2"], "INT"), "g3": (t["g3"], "INT")}))
    return gpu, ora, _tables(w)[0]["fcard"]


def _check(ctx, gpu, ora, sql, kernel):
    q = parse_sql(sql)
    r = ctx.execute(q, gpu)
    e = O.execute(q, ora)
    assert reduce_groups(q, r.keys, r.aggs).rows == reduce_groups(q, e.keys, e.aggs).rows, sql
    assert r.stats.num_docs_scanned == e.stats.num_docs_scanned
    assert r.stats.scan_kernel == kernel, (sql, SCAN_KERNEL_NAMES.get(r.stats.scan_kernel))


@pytest.mark.parametrize("w", list(range(1, 32)))
def test_lean_kernels_every_width(ctx, w, monkeypatch):
    gpu, ora, fcard = _segments(ctx, w)
    where = f" WHERE f BETWEEN {fcard // 5} AND {fcard - 1 - fcard // 7}" if fcard > 2 else " WHERE f = 1"
    # k_count_reg: the register-direct COUNT over the filter stream (width min(w, 24))
    all_docs = fcard > 2 and fcard // 5 == 0 and fcard // 7 == 0  # the range covers the dictionary: no scan
    _check(ctx, gpu, ora, f"SELECT COUNT(*) FROM t{where}", 0 if all_docs else PH_KERNEL_COUNT_REG)
    # k_agg_lean: 32-bit tile sums need value offsets below 2^26; wider streams run k_scan<MODE_AGG>
    agg = f"SELECT COUNT(*), SUM(m), MIN(m), MAX(m) FROM t{where}"
    _check(ctx, gpu, ora, agg, PH_KERNEL_AGG_LEAN if w <= 26 else 1)  # the LDS-staged k_agg_lean (default)
    grp = f"SELECT g, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t{where} GROUP BY g ORDER BY g LIMIT 100"
    # k_group_reg keeps COUNT << 40 | SUM in one slot word: value ranges that could carry past 2^40 inside one
    # workgroup (w >= 29 here) run k_group_lds_lean's unpacked table
    packed = PH_KERNEL_GROUP_REG if w <= 28 else PH_KERNEL_GROUP_LDS_LEAN
    _check(ctx, gpu, ora, grp, packed)
    _check(ctx, gpu, ora, f"SELECT g, g3, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t{where} GROUP BY g, g3 "
           f"ORDER BY g, g3 LIMIT 1000", packed)
    _check(ctx, gpu, ora, f"SELECT g, COUNT(*) FROM t{where} GROUP BY g ORDER BY g LIMIT 100", PH_KERNEL_GROUP_REG)
    monkeypatch.setenv("PH_LDS_LEAN", "1")  # the LDS-staged k_group_lds_lean
    _check(ctx, gpu, ora, grp, PH_KERNEL_GROUP_LDS_LEAN)
    monkeypatch.delenv("PH_LDS_LEAN")
    part = (f"SET numGroupsLimit=2000000; SELECT g1, g2, COUNT(*), SUM(m), MIN(m), MAX(m) FROM t{where} "
            f"GROUP BY g1, g2 ORDER BY g1, g2 LIMIT 200000")
    # k_part_reg decodes from registers (its own per-width switch): filter / key streams <= 16 bits
    _check(ctx, gpu, ora, part, PH_KERNEL_PART_REG if min(w, 24) <= 16 else PH_KERNEL_PART_LEAN)
    for sets in ("1", "2"):  # one ring set (flush, barrier, append, barrier) / two (append beside the flush)
        monkeypatch.setenv("PH_PART_SETS", sets)
        _check(ctx, gpu, ora, part, PH_KERNEL_PART_REG if min(w, 24) <= 16 else PH_KERNEL_PART_LEAN)
        monkeypatch.setenv("PH_PART_RING_LOG2", "4")  # 16-slot rings: skewed rounds take the overflow path
        _check(ctx, gpu, ora, part, PH_KERNEL_PART_REG if min(w, 24) <= 16 else PH_KERNEL_PART_LEAN)
        monkeypatch.delenv("PH_PART_RING_LOG2")
    monkeypatch.delenv("PH_PART_SETS")
    monkeypatch.setenv("PH_PART_LDS", "1")  # the LDS-staged forms
    _check(ctx, gpu, ora, part, PH_KERNEL_PART_LEAN)
    monkeypatch.setenv("PH_PART_DEPTH", "2")
    _check(ctx, gpu, ora, part, PH_KERNEL_PART_LEAN2)
    for s in gpu:
        s.unpin()
