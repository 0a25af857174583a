"""CPU: raw (no-dictionary) forward indexes -- the library's host reader (ph_raw_forward_index_read, what
ph_segment_pin runs on a raw column) against an independent Python reader (tests/raw_codecs.py) and the source
values, for every fixed-width stored type, every chunk compression (ZSTANDARD through the system's libzstd.so.1, as
zstd-jni) and writer versions 2 / 3 / 4
(BaseChunkForwardIndexWriter.java, FixedByteChunkForwardIndexWriter.java; FixedByteChunkSVForwardIndexReader)."""
import numpy as np
import pytest

from pinot_amd import native as N
from pinot_amd.segment import read_raw_forward_index, write_raw_forward_index
from tests import raw_codecs as RC
from tests.seeds import seed_of

TYPES = {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64}


def _values(dt, n, seed):
    rng = np.random.default_rng(seed)
    if dt in ("INT", "LONG"):
        v = rng.integers(-1000, 1000, n) * (10**9 if dt == "LONG" else 7)
    else:
        v = np.round(rng.normal(0, 100, n), 1)
    v = v.astype(TYPES[dt])
    v[: n // 10] = v[0]  # long runs: LZ4 / Snappy overlapping copies
    return v


@pytest.mark.parametrize("dt", list(TYPES))
@pytest.mark.parametrize("comp", ["PASS_THROUGH", "LZ4", "LZ4_LENGTH_PREFIXED", "SNAPPY", "ZSTANDARD"])
@pytest.mark.parametrize("version", [2, 3, 4])
def test_raw_reader_round_trip(dt, comp, version):
    v = _values(dt, 4321, seed_of(f"{dt}/{comp}/{version}") & 0xFFFF)
    buf = write_raw_forward_index(v, dt, comp, version)
    got = read_raw_forward_index(buf, dt, len(v))
    ind = RC.read_raw(buf.tobytes(), dt, len(v))
    assert np.array_equal(got.view(np.uint8), v.view(np.uint8))
    assert np.array_equal(ind.view(np.uint8), v.view(np.uint8))


def test_hand_built_codec_vectors():
    # LZ4: literals "abcd", then a match at offset 4 of length 8 (overlapping), then the 5 literal tail bytes
    lz4 = bytes([0x44]) + b"abcd" + (4).to_bytes(2, "little") + bytes([0x50]) + b"efghi"
    assert RC.lz4_decompress(lz4) == b"abcdabcdabcdefghi"
    # Snappy: length 12, literal "abcd", copy-1 (len 8, offset 4)
    snap = bytes([12, (3 << 2) | 0]) + b"abcd" + bytes([((8 - 4) << 2) | 1, 4])
    assert RC.snappy_decompress(snap) == b"abcdabcdabcd"
    # the same bytes as INT chunks through the library (one chunk of 4 docs + header)
    for comp, code, body in (("LZ4", 3, lz4[:-6] + bytes([0x00])), ("SNAPPY", 1, snap)):
        raw = b"abcdabcdabcd"
        hdr = np.array([2, 1, 3, 4, 3, code, 28, 32], ">i4").tobytes()
        buf = np.frombuffer(hdr + body, np.uint8)
        got = read_raw_forward_index(buf, "INT", 3)
        assert got.tolist() == np.frombuffer(raw, ">i4").tolist(), comp


def test_corrupt_and_unsupported():
    v = _values("INT", 3000, 3)
    buf = write_raw_forward_index(v, "INT", "LZ4")
    bad = buf[:-3]  # the last chunk's literals cut short
    with pytest.raises(N.PinotHipError):
        read_raw_forward_index(bad, "INT", len(v))
    z = write_raw_forward_index(v, "INT", "PASS_THROUGH").copy()
    z[20:24] = np.frombuffer(np.array([2], ">i4").tobytes(), np.uint8)  # ZSTANDARD over bytes that are no zstd frame
    with pytest.raises(N.PinotHipError):
        read_raw_forward_index(z, "INT", len(v))
    z = write_raw_forward_index(v, "INT", "PASS_THROUGH").copy()
    z[20:24] = np.frombuffer(np.array([7], ">i4").tobytes(), np.uint8)  # no such ChunkCompressionType
    with pytest.raises(N.PinotHipError):
        read_raw_forward_index(z, "INT", len(v))
    with pytest.raises(N.PinotHipError):  # lengthOfLongestEntry != the stored type's size
        read_raw_forward_index(write_raw_forward_index(v, "INT"), "LONG", len(v))
