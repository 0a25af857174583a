// rawfwd.cpp -- raw (no-dictionary) single-value forward indexes.
//
// On disk (BaseChunkForwardIndexWriter.java / FixedByteChunkForwardIndexWriter.java, read by
// BaseChunkForwardIndexReader.java:57-105 and FixedByteChunkSVForwardIndexReader.java; all BIG_ENDIAN):
//   int32 version (2: int32 chunk offsets, 3 / 4: int64), numChunks, numDocsPerChunk, lengthOfLongestEntry
//   (== the stored type's size), [version > 1: totalDocs, compressionType, dataHeaderStart], then numChunks
//   absolute chunk offsets, then the chunks.  A chunk holds numDocsPerChunk values (the last one fewer), each
//   compressed on its own: PASS_THROUGH (0), SNAPPY (1), ZSTANDARD (2), LZ4 (3), LZ4_LENGTH_PREFIXED (4)
//   (ChunkCompressionType.java:22).  Version 1 has no compression field and is SNAPPY.
//
// The GPU path keeps ONE column format: at pin time a raw column is decoded once on the host and dictionary-
// encoded (sorted distinct values = the dictionary SegmentDictionaryCreator would write, dictIds packed with
// getNumBitsPerValue(card - 1) bits), so the same fused scan kernels filter, group and aggregate it.  Every
// result equals the reference's raw-value operators': predicates on raw values select the same docs as the
// dictId ranges / sets of the same literals (RangePredicateEvaluatorFactory raw evaluators vs the sorted-
// dictionary ones), NoDictionary*GroupKeyGenerator keys are the values (DefaultGroupByExecutor.java:94-104,
// first-seen group ids, as the dictionary generator), SUM/MIN/MAX read the same values, DISTINCTCOUNTHLL
// offers the value itself (DistinctCountHLLAggregationFunction.java:118-143), which is what it offers for a
// dictionary column's ids too.  The HBM image is b bits per doc instead of 32 / 64 -- fewer bytes per scan.
//
// Decompressors (the codecs are third-party libraries absent from /root/reference; restated from their
// published block formats): LZ4 block format (lz4-java 1.8, LZ4Decompressor.java's safeDecompressor), the
// LZ4_LENGTH_PREFIXED frame of lz4-java's LZ4CompressorWithLength (4-byte little-endian original length, then
// one LZ4 block; LZ4WithLengthDecompressor.java), and the Snappy raw format (snappy-java 1.1,
// SnappyDecompressor.java).  ZSTANDARD chunks are standard zstd frames (ZstandardCompressor.java:
// Zstd.compress, ZstandardDecompressor.java: Zstd.decompress -- zstd-jni over libzstd): decoded by the system's
// libzstd.so.1, dlopen'ed on first use (no link-time dependency; without it ZSTANDARD stays PH_ERR_UNSUPPORTED).
#include <dlfcn.h>

#include <algorithm>
#include <cstring>
#include <limits>
#include <thread>

#include "ph_internal.h"

namespace ph {

namespace {

// libzstd.so.1's one-shot frame decoder (thread-safe: each call owns its context)
struct Zstd {
  size_t (*decompress)(void*, size_t, const void*, size_t) = nullptr;
  unsigned (*is_error)(size_t) = nullptr;
};
const Zstd& zstd() {
  static Zstd z = [] {
    Zstd x;
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.decompress = reinterpret_cast<size_t (*)(void*, size_t, const void*, size_t)>(dlsym(h, "ZSTD_decompress"));
    x.is_error = reinterpret_cast<unsigned (*)(size_t)>(dlsym(h, "ZSTD_isError"));
    if (!x.decompress || !x.is_error) x.decompress = nullptr;
    return x;
  }();
  return z;
}

inline uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
inline uint64_t rd_be64(const uint8_t* p) { return ((uint64_t)rd_be32(p) << 32) | rd_be32(p + 4); }

[[noreturn]] void corrupt(const char* what) { fail(PH_ERR_INVALID_ARGUMENT, std::string("raw forward index: ") + what); }

// LZ4 block: sequences of (token, literal-length bytes, literals, LE16 offset, match-length bytes); the last
// sequence carries literals only.  Returns the decompressed size.
size_t lz4_block_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  size_t ip = 0, op = 0;
  while (ip < n) {
    const uint8_t token = src[ip++];
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= n) corrupt("truncated LZ4 literal length");
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > n || op + lit > cap) corrupt("LZ4 literals out of bounds");
    memcpy(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    if (ip == n) break;  // last sequence
    if (ip + 2 > n) corrupt("truncated LZ4 offset");
    const size_t off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) corrupt("bad LZ4 match offset");
    size_t len = (token & 15u);
    if (len == 15) {
      uint8_t b;
      do {
        if (ip >= n) corrupt("truncated LZ4 match length");
        b = src[ip++];
        len += b;
      } while (b == 255);
    }
    len += 4;
    if (op + len > cap) corrupt("LZ4 match out of bounds");
    for (size_t k = 0; k < len; ++k, ++op) dst[op] = dst[op - off];  // overlapping copies repeat the pattern
  }
  return op;
}

// Snappy raw format: varint32 uncompressed length, then literal / copy elements (tag low 2 bits).
size_t snappy_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  size_t ip = 0;
  uint64_t ulen = 0;
  for (int shift = 0;; shift += 7) {
    if (ip >= n || shift > 28) corrupt("bad Snappy length varint");
    const uint8_t b = src[ip++];
    ulen |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
  }
  if (ulen > cap) corrupt("Snappy chunk larger than the chunk size");
  size_t op = 0;
  while (ip < n) {
    const uint8_t tag = src[ip++];
    const int kind = tag & 3;
    if (kind == 0) {
      size_t len = tag >> 2;
      if (len >= 60) {
        const int nb = (int)len - 59;
        if (ip + nb > n) corrupt("truncated Snappy literal length");
        len = 0;
        for (int k = 0; k < nb; ++k) len |= (size_t)src[ip + k] << (8 * k);
        ip += nb;
      }
      len += 1;
      if (ip + len > n || op + len > ulen) corrupt("Snappy literal out of bounds");
      memcpy(dst + op, src + ip, len);
      ip += len;
      op += len;
      continue;
    }
    size_t len, off;
    if (kind == 1) {
      if (ip + 1 > n) corrupt("truncated Snappy copy");
      len = ((tag >> 2) & 7u) + 4;
      off = ((size_t)(tag >> 5) << 8) | src[ip];
      ip += 1;
    } else if (kind == 2) {
      if (ip + 2 > n) corrupt("truncated Snappy copy");
      len = (size_t)(tag >> 2) + 1;
      off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
      ip += 2;
    } else {
      if (ip + 4 > n) corrupt("truncated Snappy copy");
      len = (size_t)(tag >> 2) + 1;
      off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8) | ((size_t)src[ip + 2] << 16) | ((size_t)src[ip + 3] << 24);
      ip += 4;
    }
    if (off == 0 || off > op || op + len > ulen) corrupt("bad Snappy copy");
    for (size_t k = 0; k < len; ++k, ++op) dst[op] = dst[op - off];
  }
  if (op != ulen) corrupt("Snappy chunk shorter than its declared length");
  return op;
}

int type_size(int32_t t) {
  switch (t) {
    case PH_INT: case PH_FLOAT: return 4;
    case PH_LONG: case PH_DOUBLE: return 8;
    default: fail(PH_ERR_UNSUPPORTED, "raw forward index: only fixed-width INT / LONG / FLOAT / DOUBLE columns");
  }
}

// Java's Double.compare / Float.compare order (what Arrays.sort gives the dictionary creator): -0.0 < 0.0,
// NaN last; equality by bits (Double.equals), NaNs canonical.
inline uint64_t double_key(double v) {
  uint64_t u;
  if (v != v) return ~0ull;
  memcpy(&u, &v, 8);
  return (u >> 63) ? ~u : (u | (1ull << 63));
}

}  // namespace

void raw_forward_index_decode(const uint8_t* buf, uint64_t size, int32_t data_type, int64_t num_docs, void* out) {
  const int w = type_size(data_type);
  if (size < 16) corrupt("header too small");
  const int32_t version = (int32_t)rd_be32(buf);
  const int64_t nchunks = (int32_t)rd_be32(buf + 4);
  const int64_t per_chunk = (int32_t)rd_be32(buf + 8);
  const int32_t entry = (int32_t)rd_be32(buf + 12);
  if (version < 1 || version > 4) corrupt("unknown version");
  if (entry != w) corrupt("lengthOfLongestEntry differs from the stored type's size");
  if (nchunks < 0 || per_chunk <= 0 || nchunks * per_chunk < num_docs) corrupt("chunks do not cover the docs");
  int32_t comp = 1;  // version 1: SNAPPY
  uint64_t data_header = 16;
  if (version > 1) {
    if (size < 28) corrupt("header too small");
    comp = (int32_t)rd_be32(buf + 20);
    data_header = rd_be32(buf + 24);
  }
  const int off_size = version <= 2 ? 4 : 8;
  if (data_header + (uint64_t)nchunks * off_size > size) corrupt("chunk offsets beyond the buffer");
  if (comp == 2 && !zstd().decompress) fail(PH_ERR_UNSUPPORTED, "raw forward index: ZSTANDARD needs libzstd.so.1");
  if (comp < 0 || comp > 4) corrupt("unknown compression type");
  auto chunk_pos = [&](int64_t c) -> uint64_t {
    const uint8_t* p = buf + data_header + (uint64_t)c * off_size;
    return off_size == 4 ? rd_be32(p) : rd_be64(p);
  };
  const size_t chunk_bytes = (size_t)per_chunk * w;
  auto work = [&](int64_t c0, int64_t c1) {
    std::vector<uint8_t> tmp(comp == 0 ? 0 : chunk_bytes);
    for (int64_t c = c0; c < c1; ++c) {
      const int64_t d0 = c * per_chunk;
      if (d0 >= num_docs) break;
      const int64_t nd = std::min<int64_t>(per_chunk, num_docs - d0);
      const uint64_t pos = chunk_pos(c);
      const uint64_t end = c + 1 < nchunks ? chunk_pos(c + 1) : size;
      if (pos > end || end > size) corrupt("chunk out of the buffer");
      const uint8_t* src;
      if (comp == 0) {
        if (end - pos < (uint64_t)nd * w) corrupt("short PASS_THROUGH chunk");
        src = buf + pos;
      } else {
        size_t got;
        if (comp == 1) {
          got = snappy_decompress(buf + pos, end - pos, tmp.data(), chunk_bytes);
        } else if (comp == 2) {
          got = zstd().decompress(tmp.data(), chunk_bytes, buf + pos, end - pos);
          if (zstd().is_error(got)) corrupt("bad ZSTANDARD chunk");
        } else if (comp == 3) {
          got = lz4_block_decompress(buf + pos, end - pos, tmp.data(), chunk_bytes);
        } else {  // LZ4_LENGTH_PREFIXED
          if (end - pos < 4) corrupt("short LZ4 length prefix");
          const uint8_t* p = buf + pos;
          const size_t want = (size_t)p[0] | ((size_t)p[1] << 8) | ((size_t)p[2] << 16) | ((size_t)p[3] << 24);
          got = lz4_block_decompress(p + 4, end - pos - 4, tmp.data(), chunk_bytes);
          if (got != want) corrupt("LZ4 chunk length differs from its prefix");
        }
        if (got < (size_t)nd * w) corrupt("short decompressed chunk");
        src = tmp.data();
      }
      uint8_t* dst = static_cast<uint8_t*>(out) + (size_t)d0 * w;
      if (w == 4) {
        for (int64_t i = 0; i < nd; ++i) {
          const uint32_t u = rd_be32(src + 4 * i);
          memcpy(dst + 4 * i, &u, 4);
        }
      } else {
        for (int64_t i = 0; i < nd; ++i) {
          const uint64_t u = rd_be64(src + 8 * i);
          memcpy(dst + 8 * i, &u, 8);
        }
      }
    }
  };
  const int64_t nthreads = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  if (nchunks < 64 || nthreads <= 1) {
    work(0, nchunks);
    return;
  }
  std::vector<std::thread> th;
  std::vector<std::exception_ptr> errs(nthreads);
  const int64_t per = (nchunks + nthreads - 1) / nthreads;
  for (int64_t t = 0; t < nthreads; ++t) {
    const int64_t a = t * per, b = std::min(nchunks, a + per);
    if (a < b) th.emplace_back([&, t, a, b] {
      try {
        work(a, b);
      } catch (...) {
        errs[t] = std::current_exception();
      }
    });
  }
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
}

void raw_dictionary_encode(int32_t data_type, const void* values, int64_t n, Dictionary* dict, std::vector<int32_t>* ids) {
  dict->type = data_type;
  ids->resize((size_t)n);
  // sorted distinct values (the dictionary SegmentDictionaryCreator writes), then each doc's id by binary search
  auto encode = [&](auto key_of, auto& sorted) {
    using K = decltype(key_of(0));
    std::vector<K> keys((size_t)n);
    for (int64_t i = 0; i < n; ++i) keys[i] = key_of(i);
    std::vector<K> uniq(keys);
    std::sort(uniq.begin(), uniq.end());
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    sorted = uniq;
    const int64_t nthreads = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
    auto look = [&](int64_t a, int64_t b) {
      for (int64_t i = a; i < b; ++i)
        (*ids)[i] = (int32_t)(std::lower_bound(uniq.begin(), uniq.end(), keys[i]) - uniq.begin());
    };
    if (n < (1 << 16) || nthreads <= 1) {
      look(0, n);
      return;
    }
    std::vector<std::thread> th;
    const int64_t per = (n + nthreads - 1) / nthreads;
    for (int64_t t = 0; t < nthreads; ++t) {
      const int64_t a = t * per, b = std::min(n, a + per);
      if (a < b) th.emplace_back(look, a, b);
    }
    for (auto& t : th) t.join();
  };
  if (data_type == PH_INT || data_type == PH_LONG) {
    std::vector<int64_t> s;
    if (data_type == PH_INT)
      encode([&](int64_t i) { return (int64_t) static_cast<const int32_t*>(values)[i]; }, s);
    else
      encode([&](int64_t i) { return static_cast<const int64_t*>(values)[i]; }, s);
    dict->ints = std::move(s);
    dict->size = (int64_t)dict->ints.size();
  } else {
    std::vector<uint64_t> s;
    if (data_type == PH_FLOAT)
      encode([&](int64_t i) { return double_key((double) static_cast<const float*>(values)[i]); }, s);
    else
      encode([&](int64_t i) { return double_key(static_cast<const double*>(values)[i]); }, s);
    dict->reals.resize(s.size());
    for (size_t k = 0; k < s.size(); ++k) {
      uint64_t u = s[k];
      if (u == ~0ull) {
        dict->reals[k] = std::numeric_limits<double>::quiet_NaN();
        continue;
      }
      u = (u >> 63) ? (u & ~(1ull << 63)) : ~u;
      memcpy(&dict->reals[k], &u, 8);
    }
    dict->size = (int64_t)dict->reals.size();
  }
}

}  // namespace ph
