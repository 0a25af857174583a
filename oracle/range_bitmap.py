"""Range-index reader of the CPU oracle -- TEST INFRASTRUCTURE ONLY (tests/ may import it; the product never does).

Restates BitSlicedRangeIndexReader (pinot-segment-local/.../readers/BitSlicedRangeIndexReader.java) over the bytes
BitSlicedRangeIndexCreator.seal writes (BitSlicedRangeIndexCreator.java:123-133: int32 BE version 2, int64 BE min,
then RoaringBitmap's serialized RangeBitmap).  RangeBitmap belongs to org.roaringbitmap:RoaringBitmap 0.9.38
(/root/reference/pom.xml:405-407), which the reference does not vendor; its layout and its evaluation are restated from
the library's published RangeBitmap (map / Appender.serialize / lte / gte / between / eq):

  LE u16 cookie 0xF00D, u8 base 2, u8 slice count S, u16 key count K, u32 row count;
  K masks of ceil(S/8) bytes (bit i: slice i has a container for that 65536-row key);
  the containers key-major, slices ascending -- u8 kind (0 bitmap, 1 run, 2 array), u16 size, payload;
  slice i of a key = its rows whose value has bit i CLEAR.

The query is evaluated slice by slice (O'Neil's bit-sliced comparison), not from decoded values, so a decoder
round trip and the evaluation check each other.  The reference holds no range-index file, so the byte format is
parity unpinned: pinned here only against this restatement and the product-side writer.
"""
from __future__ import annotations

import struct

import numpy as np

COOKIE, BITMAP, RUN, ARRAY = 0xF00D, 0, 1, 2


def parse(blob: bytes):
    """-> (min, S, rows, slices): slices[i] = bool[rows], True where the value's bit i is clear."""
    b = bytes(blob)
    version, vmin = struct.unpack(">iq", b[:12])
    if version != 2:
        raise ValueError("not an exact (version 2) range index")
    cookie, base, S, K, rows = struct.unpack("<HBBHI", b[12:22])
    if cookie != COOKIE or base != 2:
        raise ValueError("not a RangeBitmap")
    bpm = (S + 7) // 8
    masks = np.frombuffer(b[22:22 + K * bpm], np.uint8).reshape(K, bpm) if K else np.zeros((0, bpm), np.uint8)
    at = 22 + K * bpm
    slices = np.zeros((S, K * 65536), bool)
    for k in range(K):
        for i in range(S):
            if not (masks[k, i >> 3] >> (i & 7)) & 1:
                continue
            kind, size = struct.unpack("<BH", b[at:at + 3])
            at += 3
            z = slices[i, k * 65536:(k + 1) * 65536]
            if kind == BITMAP:
                z[:] = np.unpackbits(np.frombuffer(b[at:at + 8192], np.uint8), bitorder="little").astype(bool)
                at += 8192
            elif kind == ARRAY:
                z[np.frombuffer(b[at:at + 2 * size], "<u2")] = True
                at += 2 * size
            elif kind == RUN:
                pr = np.frombuffer(b[at:at + 4 * size], "<u2").reshape(-1, 2).astype(np.int64)
                for s, ln in pr:
                    z[s:s + ln + 1] = True
                at += 4 * size
            else:
                raise ValueError("bad container kind")
    return vmin, S, rows, slices[:, :rows]


def values(blob: bytes) -> np.ndarray:
    """The indexed values (relative to min): bit i set where the row is absent from slice i."""
    _, S, rows, slices = parse(blob)
    v = np.zeros(rows, np.uint64)
    for i in range(S):
        v |= (~slices[i]).astype(np.uint64) << np.uint64(i)
    return v


def _lte(slices, S, c: int) -> np.ndarray:
    """RangeBitmap.lte: state = c_i ? state | Z_i : state & Z_i, low bit to high."""
    st = np.ones(slices.shape[1], bool)
    for i in range(S):
        st = (st | slices[i]) if (c >> i) & 1 else (st & slices[i])
    return st


def matching_docs(blob: bytes, lo: int, hi: int, column_max: int) -> np.ndarray:
    """BitSlicedRangeIndexReader.getMatchingDocIds(min, max) over dictIds (:131-138, queryRangeBitmap :184-202)."""
    vmin, S, rows, slices = parse(blob)
    if lo > hi or lo > column_max or hi < vmin:
        return np.zeros(rows, bool)
    lo, hi = max(lo, vmin) - vmin, hi - vmin
    cmax = column_max - vmin
    if hi < cmax:
        if lo > 0:
            if lo == hi:  # RangeBitmap.eq
                st = np.ones(rows, bool)
                for i in range(S):
                    st &= ~slices[i] if (lo >> i) & 1 else slices[i]
                return st
            return _lte(slices, S, hi) & ~_lte(slices, S, lo - 1)  # between
        return _lte(slices, S, hi)
    if lo > 0:
        return ~_lte(slices, S, lo - 1)  # gte
    return np.ones(rows, bool)
