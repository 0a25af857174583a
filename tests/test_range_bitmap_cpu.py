"""CPU: the exact range index's RangeBitmap bytes (BitSlicedRangeIndexCreator.seal + RoaringBitmap 0.9.38 RangeBitmap,
restated -- parity unpinned for the byte format, the reference holds no range-index file).  The product-side writer
(pinot_amd.segment.range_index_bytes, used by the GPU tests' segments) against the oracle's independent reader:
decoded values round-trip, and the slice-by-slice evaluation of BitSlicedRangeIndexReader.queryRangeBitmap
(:184-211: lte / gte / between / eq / all) equals lo <= v <= hi on every interval tried.  All three container kinds
appear (random values: bitmaps; skewed values: arrays; sorted values: runs) over ragged key counts."""
import struct

import numpy as np
import pytest

from oracle import range_bitmap as RB
from pinot_amd.segment import range_index_bytes


def _kinds(blob):
    b = bytes(blob)
    _, _, S, K, _ = struct.unpack("<HBBHI", b[12:22])
    bpm = (S + 7) // 8
    masks = np.frombuffer(b[22:22 + K * bpm], np.uint8).reshape(K, bpm)
    at, kinds = 22 + K * bpm, set()
    for k in range(K):
        for i in range(S):
            if (masks[k, i >> 3] >> (i & 7)) & 1:
                kind, size = struct.unpack("<BH", b[at:at + 3])
                kinds.add(kind)
                at += 3 + (8192 if kind == RB.BITMAP else 4 * size if kind == RB.RUN else 2 * size)
    assert at == len(b)
    return kinds


def _cases():
    rng = np.random.default_rng(11)
    n = 2 * 65536 + 17
    yield "random", rng.integers(0, 1000, n), 999
    skew = np.full(n, 1023)
    skew[rng.integers(0, n, 300)] = rng.integers(0, 1023, 300)
    yield "skewed", skew, 1023
    yield "sorted", np.sort(rng.integers(0, 50_000, n)), 49_999
    yield "single", np.zeros(1000, np.int64), 0
    yield "tiny", rng.integers(0, 3, 5), 2


@pytest.mark.parametrize("name,ids,cmax", list(_cases()), ids=[c[0] for c in _cases()])
def test_round_trip_and_queries(name, ids, cmax):
    blob = range_index_bytes(ids, cmax)
    assert np.array_equal(RB.values(blob), ids.astype(np.uint64))
    rng = np.random.default_rng(3)
    probes = [(0, cmax), (0, 0), (cmax, cmax), (0, cmax // 2), (cmax // 2, cmax), (cmax + 1, cmax + 5)]
    probes += [tuple(sorted(rng.integers(0, cmax + 1, 2))) for _ in range(20)]
    for lo, hi in probes:
        lo, hi = int(lo), int(hi)
        got = RB.matching_docs(blob, lo, hi, cmax)
        assert np.array_equal(got, (ids >= lo) & (ids <= hi)), (name, lo, hi)
    assert not RB.matching_docs(blob, 5, 4, cmax).any()


def test_every_container_kind_is_written():
    kinds = set()
    for _, ids, cmax in _cases():
        kinds |= _kinds(range_index_bytes(ids, cmax))
    assert kinds == {RB.BITMAP, RB.RUN, RB.ARRAY}
