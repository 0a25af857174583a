"""Segment creation (the writer side of the on-disk format) and HBM pinning.

``create_segment`` produces, for each dictionary-encoded single-value column, the exact byte buffers a
V3 Pinot segment holds in ``columns.psf`` (all big-endian):

* dictionary       sorted unique values, fixed width (SegmentDictionaryCreator.java:100-276)
* forward index    unsorted: dictIds packed MSB-first with bitsPerElement = getNumBitsPerValue(card-1)
                   (FixedBitSVForwardIndexWriter.java:39-50, packed by ph_fixed_bit_pack);
                   sorted: int32 (startDocId, endDocId) per dictId (SingleValueSortedForwardIndexCreator)
* inverted index   uint32 offsets[card+1] then one portable-format RoaringBitmap per dictId
                   (BitmapInvertedIndexWriter.java:33-96; RoaringFormatSpec, RoaringBitmap 0.9.38 serialize())

``pin`` hands those buffers to ``ph_segment_pin`` (the GPU side of ImmutableSegmentLoader.load).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Dict, Optional, Sequence

import struct

import numpy as np

from . import native as N


def num_bits_per_value(max_value: int) -> int:
    """PinotDataBitSet.getNumBitsPerValue (PinotDataBitSet.java:59-70)."""
    if max_value <= 1:
        return 1
    return int(max_value).bit_length()


def fixed_bit_pack(dict_ids: np.ndarray, bits: int) -> np.ndarray:
    ids = np.ascontiguousarray(dict_ids, dtype=np.int32)
    out = np.zeros((len(ids) * bits + 7) // 8, dtype=np.uint8)
    N.check(N.lib().ph_fixed_bit_pack(ids.ctypes.data, len(ids), bits, out.ctypes.data, out.nbytes))
    return out


# --------------------------------------------------------------------------- roaring (portable format)
SERIAL_COOKIE_NO_RUNCONTAINER = 12346
SERIAL_COOKIE = 12347
NO_OFFSET_THRESHOLD = 4


def roaring_serialize(docs: np.ndarray, run_optimize: bool = False) -> bytes:
    """Serialize a sorted set of doc ids in RoaringBitmap's portable format.  With ``run_optimize`` each
    container takes the smallest of array / bitmap / run encodings (RoaringBitmap.runOptimize)."""
    docs = np.asarray(docs, dtype=np.uint32)
    if len(docs) == 0:
        return np.array([SERIAL_COOKIE_NO_RUNCONTAINER, 0], dtype="<u4").tobytes()
    keys, starts = np.unique(docs >> 16, return_index=True)
    ends = np.append(starts[1:], len(docs))
    size = len(keys)
    kinds, payloads, cards = [], [], []
    for k, s, e in zip(keys, starts, ends):
        low = (docs[s:e] & 0xFFFF).astype(np.uint16)
        card = e - s
        nruns = 1 + int(np.count_nonzero(np.diff(low.astype(np.int32)) != 1))
        arr_bytes = 2 * card if card <= 4096 else 1 << 30
        bmp_bytes = 8192
        run_bytes = 2 + 4 * nruns if run_optimize else 1 << 30
        best = min(arr_bytes, bmp_bytes, run_bytes)
        if best == run_bytes:
            brk = np.flatnonzero(np.diff(low.astype(np.int32)) != 1)
            rs = np.concatenate([[0], brk + 1])
            re = np.concatenate([brk, [card - 1]])
            runs = np.empty(2 * nruns, dtype="<u2")
            runs[0::2] = low[rs]
            runs[1::2] = low[re] - low[rs]
            payloads.append(np.array([nruns], "<u2").tobytes() + runs.tobytes())
            kinds.append(2)
        elif best == arr_bytes:
            payloads.append(low.astype("<u2").tobytes())
            kinds.append(0)
        else:
            words = np.zeros(1024, dtype=np.uint64)
            np.bitwise_or.at(words, low >> 6, np.left_shift(np.uint64(1), (low & 63).astype(np.uint64)))
            payloads.append(words.astype("<u8").tobytes())
            kinds.append(1)
        cards.append(card)
    has_runs = any(k == 2 for k in kinds)
    head = bytearray()
    if has_runs:
        head += np.array([SERIAL_COOKIE | ((size - 1) << 16)], "<u4").tobytes()
        flags = np.zeros((size + 7) // 8, np.uint8)
        for i, k in enumerate(kinds):
            if k == 2:
                flags[i // 8] |= 1 << (i % 8)
        head += flags.tobytes()
        with_offsets = size >= NO_OFFSET_THRESHOLD
    else:
        head += np.array([SERIAL_COOKIE_NO_RUNCONTAINER, size], "<u4").tobytes()
        with_offsets = True
    desc = np.empty(2 * size, "<u2")
    desc[0::2] = keys
    desc[1::2] = np.array(cards) - 1
    head += desc.tobytes()
    pos = len(head) + (4 * size if with_offsets else 0)
    offs = []
    for p in payloads:
        offs.append(pos)
        pos += len(p)
    if with_offsets:
        head += np.array(offs, "<u4").tobytes()
    return bytes(head) + b"".join(payloads)


def build_inverted_index(dict_ids: np.ndarray, card: int, run_optimize: bool = False) -> np.ndarray:
    order = np.argsort(dict_ids, kind="stable")
    bounds = np.searchsorted(dict_ids[order], np.arange(card + 1), side="left")
    blobs = [roaring_serialize(order[bounds[i]:bounds[i + 1]], run_optimize) for i in range(card)]
    base = 4 * (card + 1)
    offsets = np.empty(card + 1, dtype=np.int64)
    offsets[0] = base
    offsets[1:] = base + np.cumsum([len(b) for b in blobs])
    return np.frombuffer(offsets.astype(">u4").tobytes() + b"".join(blobs), dtype=np.uint8)


# --------------------------------------------------------------------------- column / segment buffers
_NP = {"INT": ">i4", "LONG": ">i8", "FLOAT": ">f4", "DOUBLE": ">f8"}
_NATIVE = {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}


@dataclass
class ColumnBuffers:
    name: str
    data_type: str
    cardinality: int
    bits: int
    is_sorted: bool
    forward_index: np.ndarray
    dictionary: np.ndarray          # big-endian bytes
    entry_size: int
    dictionary_values: np.ndarray   # native values (for tests / reduce)
    inverted_index: Optional[np.ndarray] = None
    raw: bool = False               # forward_index is a raw chunk forward index (no dictionary)
    range_index: Optional[np.ndarray] = None  # bit-sliced range index bytes (header: version 2, min)


def range_index_header(min_value: int = 0) -> np.ndarray:
    """The BitSlicedRangeIndexCreator header (BitSlicedRangeIndexCreator.java:125-131: int32 BE version 2, int64 BE
    min -- 0 for a dictionary column, whose index is built over dictIds)."""
    return np.frombuffer(np.array([2], ">i4").tobytes() + np.array([min_value], ">i8").tobytes(), np.uint8).copy()


RB_COOKIE, RB_BITMAP, RB_RUN, RB_ARRAY = 0xF00D, 0, 1, 2


def _rb_container(rows: np.ndarray) -> bytes:
    """One RangeBitmap container of a key's sorted rows (u16): the smallest of run / array / bitmap."""
    card = int(rows.size)
    brk = np.flatnonzero(np.diff(rows.astype(np.int32)) != 1) + 1
    starts = np.concatenate(([0], brk))
    ends = np.concatenate((brk, [card]))
    nruns = int(starts.size)
    if 4 * nruns < min(2 * card, 8192):
        pairs = np.empty(2 * nruns, "<u2")
        pairs[0::2] = rows[starts]
        pairs[1::2] = ends - starts - 1
        return struct.pack("<BH", RB_RUN, nruns) + pairs.tobytes()
    if card <= 4096:
        return struct.pack("<BH", RB_ARRAY, card) + rows.astype("<u2").tobytes()
    bits = np.zeros(65536, np.uint8)
    bits[rows] = 1
    return struct.pack("<BH", RB_BITMAP, (card - 1) & 0xFFFF) + np.packbits(bits, bitorder="little").tobytes()


def range_index_bytes(values: np.ndarray, max_value: int, min_value: int = 0) -> np.ndarray:
    """An exact range index as BitSlicedRangeIndexCreator writes it (dictionary column: values = dictIds, max =
    cardinality - 1): the header, then RoaringBitmap 0.9.38's RangeBitmap (Appender.serialize; the dependency is not
    vendored in the reference, its layout is restated in pinot_amd/csrc/roaring.cpp parse_range_bitmap): LE u16
    cookie 0xF00D, u8 base 2, u8 slice count S, u16 key count, u32 rows; per 65536-row key a ceil(S/8)-byte mask of
    the slices present; the containers (key-major, slices ascending), slice i = the key's rows whose value has bit i
    clear."""
    v = np.asarray(values).astype(np.uint64) - np.uint64(min_value)
    n = int(v.size)
    S = max(1, int(max_value - min_value).bit_length())
    nkeys = (n + 65535) >> 16
    bpm = (S + 7) >> 3
    masks = np.zeros((nkeys, bpm), np.uint8)
    parts = []
    for k in range(nkeys):
        chunk = v[k << 16:(k + 1) << 16]
        for i in range(S):
            rows = np.flatnonzero(((chunk >> np.uint64(i)) & np.uint64(1)) == 0).astype(np.uint16)
            if rows.size == 0:
                continue
            masks[k, i >> 3] |= np.uint8(1 << (i & 7))
            parts.append(_rb_container(rows))
    body = struct.pack("<HBBHI", RB_COOKIE, 2, S, nkeys, n) + masks.tobytes() + b"".join(parts)
    return np.concatenate([range_index_header(min_value), np.frombuffer(body, np.uint8)])


def legacy_range_index_bytes(ids: np.ndarray, num_ranges: int = 20, value_type: str = "INT") -> tuple:
    """A legacy version-1 range index as RangeIndexCreator.seal lays it out (RangeIndexCreator.java:283-410): ranges of
    about ceil(n / num_ranges) sorted values that never split a value, then int32 BE version 1, the value type's name,
    the range count, the ranges' first values + the last range's end (in the value type: int32 / int64 / float32 /
    float64 BE), (R + 1) int64 BE absolute offsets and each range's doc bitmap (portable roaring).  ``ids``: the
    dictIds of a dictionary column (value_type "INT"), or the raw values of a no-dictionary column of that type.
    -> (bytes, starts + [last end]) -- the second for the oracle."""
    dt = {"INT": (">i4", np.int64), "LONG": (">i8", np.int64), "FLOAT": (">f4", np.float64),
          "DOUBLE": (">f8", np.float64)}[value_type]
    ids = np.asarray(ids)
    ids = ids.astype(np.float32 if value_type == "FLOAT" else np.float64) if value_type in ("FLOAT", "DOUBLE") \
        else ids.astype(np.int64)
    n = int(ids.size)
    order = np.argsort(ids, kind="stable")
    sv = ids[order]
    per = (n + num_ranges - 1) // num_ranges
    change = np.flatnonzero(sv[1:] != sv[:-1]) + 1  # i with sv[i] != sv[i - 1]
    ranges, start = [], 0
    while True:
        j = int(np.searchsorted(change, start + per, side="right"))  # first change i > start + per
        if j >= change.size:
            break
        i = int(change[j])
        ranges.append((start, i - 1))
        start = i
    ranges.append((start, n - 1))
    bitmaps = [roaring_serialize(np.sort(order[a:b + 1]).astype(np.uint32)) for a, b in ranges]
    R = len(ranges)
    name = value_type.encode()
    head = struct.pack(">ii", 1, len(name)) + name + struct.pack(">i", R)
    head += np.array([sv[a] for a, _ in ranges] + [sv[-1]], dt[0]).tobytes()
    off = len(head) + 8 * (R + 1)
    offs = [off]
    for bm in bitmaps:
        off += len(bm)
        offs.append(off)
    blob = head + np.array(offs, ">i8").tobytes() + b"".join(bitmaps)
    return np.frombuffer(blob, np.uint8).copy(), np.array([sv[a] for a, _ in ranges] + [sv[-1]], dt[1])


@dataclass
class SegmentBuffers:
    name: str
    num_docs: int
    columns: Dict[str, ColumnBuffers] = field(default_factory=dict)


def encode_dictionary(values: np.ndarray, data_type: str):
    if data_type == "STRING":
        enc = [str(v).encode("utf-8") for v in values]
        width = max([len(e) for e in enc] + [1])
        buf = np.zeros((len(enc), width), dtype=np.uint8)
        for i, e in enumerate(enc):
            buf[i, :len(e)] = np.frombuffer(e, dtype=np.uint8)
        return buf.reshape(-1), width
    arr = np.asarray(values, dtype=_NP[data_type])
    return np.frombuffer(arr.tobytes(), dtype=np.uint8), arr.dtype.itemsize


def create_column_from_dict_ids(name: str, dictionary: np.ndarray, dict_ids: np.ndarray, data_type: str,
                                inverted: bool = False, allow_sorted: bool = True,
                                run_optimize: bool = False) -> ColumnBuffers:
    card = len(dictionary)
    dict_ids = np.ascontiguousarray(dict_ids, dtype=np.int32)
    bits = num_bits_per_value(card - 1)
    is_sorted = allow_sorted and bool(len(dict_ids) == 0 or np.all(dict_ids[1:] >= dict_ids[:-1]))
    if is_sorted:
        starts = np.searchsorted(dict_ids, np.arange(card), side="left")
        ends = np.searchsorted(dict_ids, np.arange(card), side="right") - 1
        pairs = np.stack([starts, ends], axis=1).astype(">i4")
        fwd = np.frombuffer(pairs.tobytes(), dtype=np.uint8)
    else:
        fwd = fixed_bit_pack(dict_ids, bits)
    dbytes, width = encode_dictionary(dictionary, data_type)
    inv = build_inverted_index(dict_ids, card, run_optimize) if inverted else None
    return ColumnBuffers(name, data_type, card, bits, is_sorted, fwd, dbytes, width, np.asarray(dictionary), inv)


def create_column(name: str, values, data_type: str, inverted: bool = False, run_optimize: bool = False):
    if data_type == "STRING":
        values = np.asarray(values).astype(str)
    else:
        values = np.asarray(values, dtype=_NATIVE[data_type])
    dictionary, ids = np.unique(values, return_inverse=True)
    return create_column_from_dict_ids(name, dictionary, ids.reshape(-1), data_type, inverted,
                                       run_optimize=run_optimize)


# --------------------------------------------------------------------------- raw (no-dictionary) columns
COMPRESSION = {"PASS_THROUGH": 0, "SNAPPY": 1, "ZSTANDARD": 2, "LZ4": 3, "LZ4_LENGTH_PREFIXED": 4}


def _lz4_block(data: bytes) -> bytes:
    """LZ4 block format (greedy 4-byte hash matches; the last 5 bytes stay literals, as the format requires)."""
    n, out, anchor, i, table = len(data), bytearray(), 0, 0, {}

    def lengths(v):
        b = bytearray()
        while v >= 255:
            b.append(255)
            v -= 255
        b.append(v)
        return b
    while i + 12 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is None or i - j > 65535:
            i += 1
            continue
        m = 4
        while i + m < n - 5 and data[j + m] == data[i + m]:
            m += 1
        lit = i - anchor
        out.append((min(lit, 15) << 4) | min(m - 4, 15))
        if lit >= 15:
            out += lengths(lit - 15)
        out += data[anchor:i]
        out += (i - j).to_bytes(2, "little")
        if m - 4 >= 15:
            out += lengths(m - 4 - 15)
        i += m
        anchor = i
    lit = n - anchor
    out.append(min(lit, 15) << 4)
    if lit >= 15:
        out += lengths(lit - 15)
    out += data[anchor:]
    return bytes(out)


def _zstd(data: bytes) -> bytes:
    """ZstandardCompressor (zstd-jni Zstd.compress, level 3): one standard zstd frame, through the system's
    libzstd.so.1 (test data writer; the library decodes with the same libzstd)."""
    import ctypes
    z = ctypes.CDLL("libzstd.so.1")
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    z.ZSTD_isError.restype = ctypes.c_uint
    z.ZSTD_isError.argtypes = [ctypes.c_size_t]
    cap = z.ZSTD_compressBound(len(data))
    out = ctypes.create_string_buffer(cap)
    src = ctypes.create_string_buffer(bytes(data), len(data))
    n = z.ZSTD_compress(out, cap, src, len(data), 3)
    if z.ZSTD_isError(n):
        raise RuntimeError("zstd compression failed")
    return out.raw[:n]


def _snappy(data: bytes) -> bytes:
    """Snappy raw format: varint length, then literals and 2-byte-offset copies (greedy 4-byte hash matches)."""
    n, out = len(data), bytearray()
    v = n
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)

    def literal(a, b):
        ln = b - a - 1
        if ln < 60:
            out.append(ln << 2)
        else:
            nb = (ln.bit_length() + 7) // 8
            out.append((59 + nb) << 2)
            out.extend(ln.to_bytes(nb, "little"))
        out.extend(data[a:b])
    anchor, i, table = 0, 0, {}
    while i + 4 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is None or i - j > 65535:
            i += 1
            continue
        m = 4
        while i + m < n and m < 64 and data[j + m] == data[i + m]:
            m += 1
        if anchor < i:
            literal(anchor, i)
        out.append(((m - 1) << 2) | 2)
        out.extend((i - j).to_bytes(2, "little"))
        i += m
        anchor = i
    if anchor < n:
        literal(anchor, n)
    return bytes(out)


def write_raw_forward_index(values, data_type: str, compression: str = "PASS_THROUGH", version: int = 2,
                            docs_per_chunk: int = 1000) -> np.ndarray:
    """FixedByteChunkForwardIndexWriter / BaseChunkForwardIndexWriter (SingleValueFixedByteRawIndexCreator:
    NUM_DOCS_PER_CHUNK 1000; version 4 rounds docs per chunk up to a power of 2): header, chunk offsets, chunks."""
    vals = np.asarray(values, dtype=_NP[data_type])
    width = vals.dtype.itemsize
    if version >= 4 and docs_per_chunk & (docs_per_chunk - 1):
        docs_per_chunk = 1 << (docs_per_chunk - 1).bit_length()
    n = len(vals)
    nchunks = (n + docs_per_chunk - 1) // docs_per_chunk
    off_size = 4 if version == 2 else 8
    header = 7 * 4 + nchunks * off_size
    raw = vals.tobytes()
    chunks, offsets, pos = [], [], header
    for c in range(nchunks):
        body = raw[c * docs_per_chunk * width:(c + 1) * docs_per_chunk * width]
        if compression == "LZ4":
            body = _lz4_block(body)
        elif compression == "LZ4_LENGTH_PREFIXED":
            body = len(body).to_bytes(4, "little") + _lz4_block(body)
        elif compression == "SNAPPY":
            body = _snappy(body)
        elif compression == "ZSTANDARD":
            body = _zstd(body)
        elif compression != "PASS_THROUGH":
            raise ValueError(compression)
        offsets.append(pos)
        chunks.append(body)
        pos += len(body)
    head = np.array([version, nchunks, docs_per_chunk, width, n, COMPRESSION[compression], 28], ">i4").tobytes()
    head += np.array(offsets, ">i4" if off_size == 4 else ">i8").tobytes()
    return np.frombuffer(head + b"".join(chunks), dtype=np.uint8)


def read_raw_forward_index(buf: np.ndarray, data_type: str, num_docs: int) -> np.ndarray:
    """ph_raw_forward_index_read: the library's host decoder of a raw forward index (native-endian values)."""
    out = np.empty(num_docs, dtype=_NATIVE[data_type])
    b = np.ascontiguousarray(buf, dtype=np.uint8)
    N.check(N.lib().ph_raw_forward_index_read(b.ctypes.data, b.nbytes, N.DATA_TYPES[data_type], num_docs,
                                              out.ctypes.data))
    return out


def create_raw_column(name: str, values, data_type: str, compression: str = "PASS_THROUGH", version: int = 2):
    """A no-dictionary SV column (SingleValueFixedByteRawIndexCreator); dictionary_values keeps the sorted distinct
    values for tests."""
    vals = np.asarray(values, dtype=_NATIVE[data_type])
    fwd = write_raw_forward_index(vals, data_type, compression, version)
    uniq = np.unique(vals)
    return ColumnBuffers(name, data_type, len(uniq), num_bits_per_value(len(uniq) - 1), False, fwd,
                         np.zeros(0, np.uint8), vals.dtype.itemsize, uniq, None, True)


def create_segment(name: str, columns: Dict[str, tuple], inverted: Sequence[str] = (),
                   run_optimize: bool = False, raw: Sequence[str] = (), raw_compression: str = "PASS_THROUGH",
                   raw_version: int = 2, range_index: Sequence[str] = ()) -> SegmentBuffers:
    """columns: name -> (values, data_type) -- SegmentIndexCreationDriverImpl for SV columns (dictionary-encoded, or
    raw for the names in ``raw``: noDictionaryColumns; ``range_index``: rangeIndexColumns, see range_index_header)."""
    seg = SegmentBuffers(name, 0)
    n = None
    for c, (vals, dt) in columns.items():
        if c in raw:
            seg.columns[c] = create_raw_column(c, vals, dt, raw_compression, raw_version)
        else:
            seg.columns[c] = create_column(c, vals, dt, c in inverted, run_optimize)
        if c in range_index:
            cb = seg.columns[c]
            if cb.raw:
                seg.columns[c].range_index = range_index_header()  # raw columns: the leaf scans (header only)
            else:
                ids = np.searchsorted(np.asarray(cb.dictionary_values), np.asarray(vals))
                seg.columns[c].range_index = range_index_bytes(ids, max(len(cb.dictionary_values) - 1, 0))
        n = len(vals) if n is None else n
        if n != len(vals):
            raise ValueError("columns of different lengths")
    seg.num_docs = n or 0
    return seg


# --------------------------------------------------------------------------- pinning
class PinnedSegment:
    """An immutable segment resident in HBM (ph_segment)."""

    @classmethod
    def from_dir(cls, ctx, path: str, columns=None) -> "PinnedSegment":
        """ph_segment_load_dir: pin a V3 / V1 segment directory (columns: names to pin, None = every single-value
        dictionary column)."""
        self = cls.__new__(cls)
        self.ctx = ctx
        self.buffers = None
        self.handle = None
        cols = list(columns or [])
        arr = (ctypes.c_char_p * max(1, len(cols)))(*[c.encode() for c in cols])
        h = ctypes.c_void_p()
        N.check(N.lib().ph_segment_load_dir(ctx.handle, path.encode(), arr, len(cols), ctypes.byref(h)))
        self.handle = h
        self.num_docs = N.lib().ph_segment_num_docs(h)
        self.name = path
        return self

    def __init__(self, ctx, buffers: SegmentBuffers, hll_columns=(), log2m: int = 8):
        """hll_columns: columns whose DISTINCTCOUNTHLL table (for log2m) is built at pin (ph_column_desc.hll_log2m)."""
        self.ctx = ctx
        self.name = buffers.name
        self.num_docs = buffers.num_docs
        self.buffers = buffers
        cols = (N.ColumnDesc * max(1, len(buffers.columns)))()
        keep = []
        for i, cb in enumerate(buffers.columns.values()):
            d = cols[i]
            nm = cb.name.encode()
            keep.append(nm)
            d.name = nm
            d.data_type = N.DATA_TYPES[cb.data_type]
            d.cardinality = cb.cardinality
            d.bits_per_element = cb.bits
            d.is_sorted = int(cb.is_sorted)
            fwd = np.ascontiguousarray(cb.forward_index)
            dic = np.ascontiguousarray(cb.dictionary)
            keep += [fwd, dic]
            d.forward_index = fwd.ctypes.data
            d.forward_index_size = fwd.nbytes
            d.dictionary = dic.ctypes.data
            d.dictionary_size = dic.nbytes
            d.dictionary_entry_size = cb.entry_size
            d.raw_forward_index = int(cb.raw)
            d.hll_log2m = log2m if cb.name in hll_columns else 0
            if cb.inverted_index is not None:
                inv = np.ascontiguousarray(cb.inverted_index)
                keep.append(inv)
                d.inverted_index = inv.ctypes.data
                d.inverted_index_size = inv.nbytes
            if cb.range_index is not None:
                ri = np.ascontiguousarray(cb.range_index)
                keep.append(ri)
                d.range_index = ri.ctypes.data
                d.range_index_size = ri.nbytes
        desc = N.SegmentDesc(buffers.name.encode(), buffers.num_docs, len(buffers.columns), cols)
        h = ctypes.c_void_p()
        N.check(N.lib().ph_segment_pin(ctx.handle, ctypes.byref(desc), ctypes.byref(h)))
        self.handle = h

    @property
    def device_bytes(self) -> int:
        return N.lib().ph_segment_device_bytes(self.handle)

    def unpin(self):
        if self.handle:
            N.check(N.lib().ph_segment_unpin(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.unpin()
        except Exception:
            pass
