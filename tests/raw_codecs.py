"""Independent Python reader of raw (no-dictionary) chunk forward indexes (test infrastructure): the checker for
the library's ph_raw_forward_index_read.  Follows BaseChunkForwardIndexReader.java:57-105 (header, chunk offsets)
and FixedByteChunkSVForwardIndexReader (values big-endian, chunk = numDocsPerChunk values), with the LZ4 block
and Snappy raw formats restated from their published specifications (lz4-java 1.8 / snappy-java 1.1 are not in
/root/reference)."""
import numpy as np

_NP = {"INT": ">i4", "LONG": ">i8", "FLOAT": ">f4", "DOUBLE": ">f8"}


def lz4_decompress(src: bytes) -> bytes:
    out, i = bytearray(), 0
    while i < len(src):
        tok = src[i]
        i += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                b = src[i]
                i += 1
                lit += b
                if b != 255:
                    break
        out += src[i:i + lit]
        i += lit
        if i >= len(src):
            break
        off = src[i] | (src[i + 1] << 8)
        i += 2
        m = tok & 15
        if m == 15:
            while True:
                b = src[i]
                i += 1
                m += b
                if b != 255:
                    break
        for _ in range(m + 4):
            out.append(out[-off])
    return bytes(out)


def snappy_decompress(src: bytes) -> bytes:
    n, shift, i = 0, 0, 0
    while True:
        b = src[i]
        i += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if not b & 0x80:
            break
    out = bytearray()
    while i < len(src):
        tag = src[i]
        i += 1
        kind = tag & 3
        if kind == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(src[i:i + nb], "little")
                i += nb
            out += src[i:i + ln + 1]
            i += ln + 1
            continue
        if kind == 1:
            ln, off = ((tag >> 2) & 7) + 4, ((tag >> 5) << 8) | src[i]
            i += 1
        elif kind == 2:
            ln, off = (tag >> 2) + 1, int.from_bytes(src[i:i + 2], "little")
            i += 2
        else:
            ln, off = (tag >> 2) + 1, int.from_bytes(src[i:i + 4], "little")
            i += 4
        for _ in range(ln):
            out.append(out[-off])
    assert len(out) == n
    return bytes(out)


def zstd_decompress(src: bytes, cap: int) -> bytes:
    """zstd frame -> bytes through the system's libzstd.so.1 (ZstandardDecompressor: Zstd.decompress)."""
    import ctypes
    z = ctypes.CDLL("libzstd.so.1")
    z.ZSTD_decompress.restype = ctypes.c_size_t
    z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    z.ZSTD_isError.restype = ctypes.c_uint
    z.ZSTD_isError.argtypes = [ctypes.c_size_t]
    out = ctypes.create_string_buffer(max(1, cap))
    s = ctypes.create_string_buffer(bytes(src), len(src))
    n = z.ZSTD_decompress(out, cap, s, len(src))
    assert not z.ZSTD_isError(n)
    return out.raw[:n]


def read_raw(buf: bytes, data_type: str, num_docs: int) -> np.ndarray:
    h = np.frombuffer(buf[:28], ">i4")
    version, nchunks, per, width = (int(x) for x in h[:4])
    comp, start = (int(h[5]), int(h[6])) if version > 1 else (1, 16)
    osz = 4 if version <= 2 else 8
    offs = [int(x) for x in np.frombuffer(buf[start:start + nchunks * osz], ">i4" if osz == 4 else ">i8")]
    body = bytearray()
    for c in range(nchunks):
        chunk = buf[offs[c]:offs[c + 1] if c + 1 < nchunks else len(buf)]
        if comp == 1:
            chunk = snappy_decompress(chunk)
        elif comp == 3:
            chunk = lz4_decompress(chunk)
        elif comp == 2:
            chunk = zstd_decompress(chunk, per * width)
        elif comp == 4:
            want = int.from_bytes(chunk[:4], "little")
            chunk = lz4_decompress(chunk[4:])
            assert len(chunk) == want
        body += chunk[:per * width]
    return np.frombuffer(bytes(body[:num_docs * width]), _NP[data_type]).astype(_NP[data_type][1:])
