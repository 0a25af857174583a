// roaring.cpp -- host-side parsing of bitmap inverted indexes: the per-dictId offset table of
// BitmapInvertedIndexWriter (uint32 BE offsets[C + 1], BitmapInvertedIndexWriter.java:33-50,89-96, normalised by the
// first offset as BitmapInvertedIndexReader.java:40-61 does) and the portable-format RoaringBitmap blobs behind it
// (RoaringBitmap 0.9.38 serialize(), RoaringFormatSpec), parsed ONCE at pin into a container directory that stays
// on the device; a query then names only (dictId -> directory range) items.  Every length and offset read from the
// untrusted bytes is bounds-checked here (the CPU sanitizer harness tests/sanitize/ feeds it corrupted buffers).
#include <cstring>
#include <string>
#include <vector>

#include "ph_internal.h"

namespace ph {

namespace {

// ------------------------------------------------------------------ roaring container directory
uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }
uint16_t le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
uint32_t be32u(const uint8_t* p) { return ((uint32_t)p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3]; }

// Parse one portable-format RoaringBitmap (RoaringFormatSpec; RoaringBitmap 0.9.38 serialize()).
void parse_roaring(const uint8_t* blob, uint64_t len, uint64_t blob_offset, std::vector<RoaringContainer>& out) {
  if (len < 8) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated bitmap");  // cookie + size / first key
  const uint32_t cookie = le32(blob);
  uint64_t pos = 4;
  uint32_t size;
  const uint8_t* run_flags = nullptr;
  bool has_offsets;
  if ((cookie & 0xFFFF) == 12347) {  // SERIAL_COOKIE: run containers present
    size = (cookie >> 16) + 1;
    run_flags = blob + pos;
    pos += (size + 7) / 8;
    has_offsets = size >= 4;  // NO_OFFSET_THRESHOLD
  } else if (cookie == 12346) {  // SERIAL_COOKIE_NO_RUNCONTAINER
    size = le32(blob + pos);
    pos += 4;
    has_offsets = true;
  } else {
    fail(PH_ERR_INVALID_ARGUMENT, "inverted index: bad roaring cookie");
  }
  const uint8_t* desc = blob + pos;
  pos += 4ull * size;
  const uint8_t* offs = nullptr;
  if (has_offsets) {
    offs = blob + pos;
    pos += 4ull * size;
  }
  if (pos > len) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated roaring header");
  uint64_t cur = pos;
  int32_t prev_key = -1;
  for (uint32_t i = 0; i < size; ++i) {
    RoaringContainer c{};
    c.key = le16(desc + 4 * i);
    // keys strictly ascending (RoaringFormatSpec): the chunked device build takes a dictId's container for a chunk
    // by its key
    if (c.key <= prev_key) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: roaring keys not ascending");
    prev_key = c.key;
    const uint32_t card = (uint32_t)le16(desc + 4 * i + 2) + 1;
    const bool is_run = run_flags && ((run_flags[i / 8] >> (i % 8)) & 1);
    uint64_t at = has_offsets ? le32(offs + 4 * i) : cur;
    uint64_t bytes;
    if (is_run) {
      c.type = 2;
      if (at + 2 > len) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated run container");
      c.card = le16(blob + at);
      bytes = 2 + 4ull * c.card;
    } else if (card <= 4096) {
      c.type = 0;
      c.card = (int32_t)card;
      bytes = 2ull * card;
    } else {
      c.type = 1;
      c.card = (int32_t)card;
      bytes = 8192;
    }
    if (at + bytes > len) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated container");
    c.offset = blob_offset + at;
    cur = at + bytes;
    out.push_back(c);
  }
}

}  // namespace

void build_bitmap_directory(Column& c) {
  // BitmapInvertedIndexReader.getDocIds: offsets are uint32 BE; normalise by the first offset
  // (absolute or relative formats, BitmapInvertedIndexReader.java:40-61)
  const uint8_t* b = c.inverted.data();
  if (c.cardinality < 0) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: negative cardinality");
  const uint64_t off_end = 4ull * ((uint64_t)c.cardinality + 1);
  if (c.inverted.size() < off_end) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: truncated offset table");
  const uint64_t first = be32u(b);
  c.dir.clear();
  c.dir_begin.assign(1, 0);
  c.id_docs.assign(c.cardinality, 0);
  for (int32_t id = 0; id < c.cardinality; ++id) {
    uint64_t s = be32u(b + 4ull * id) - first, e = be32u(b + 4ull * (id + 1)) - first;
    if (off_end + e > c.inverted.size() || e < s) fail(PH_ERR_INVALID_ARGUMENT, "inverted index: bad offsets");
    const size_t k0 = c.dir.size();
    parse_roaring(b + off_end + s, e - s, off_end + s, c.dir);
    int64_t docs = 0;
    for (size_t k = k0; k < c.dir.size(); ++k) {
      const RoaringContainer& rc = c.dir[k];
      if (rc.type != 2) {
        docs += rc.card;
      } else {  // run container: (start, length - 1) pairs after the run count
        const uint8_t* r = b + rc.offset + 2;
        for (int32_t j = 0; j < rc.card; ++j) docs += (int64_t)le16(r + 4 * j + 2) + 1;
      }
    }
    c.id_docs[id] = docs;
    c.dir_begin.push_back((int64_t)c.dir.size());
  }
}


// A legacy version-1 range index (RangeIndexCreator.seal :300-380; RangeIndexReaderImpl :46-88): int32 BE version 1,
// int32 BE type-name length + the name ("INT": a dictionary column's index over dictIds), int32 BE range count R,
// R + 1 values (the ranges' first values, then the last range's end), R + 1 int64 BE absolute offsets of the ranges'
// portable roaring bitmaps.  Kept: the starts, the end and each range's doc count -- the leaf's doc set is exact
// from the dictIds; its statistic is the docs of its boundary ranges (getPartialMatchesInRange :300-308)
void parse_legacy_range_index_typed(const uint8_t* b, uint64_t size, std::string* type, std::vector<int64_t>* starts,
                                    int64_t* last_end, std::vector<double>* rstarts, double* rlast_end,
                                    std::vector<int64_t>* cards) {
  auto need = [&](uint64_t at) {
    if (at > size) fail(PH_ERR_INVALID_ARGUMENT, "legacy range index: truncated");
  };
  need(8);
  const uint32_t tl = be32u(b + 4);
  need(8 + (uint64_t)tl + 4);
  type->assign(reinterpret_cast<const char*>(b + 8), tl);
  const int w = *type == "INT" || *type == "FLOAT" ? 4 : (*type == "LONG" || *type == "DOUBLE" ? 8 : 0);
  if (!w) fail(PH_ERR_UNSUPPORTED, "legacy range index over " + *type + " values");
  uint64_t at = 8 + tl;
  const uint32_t R = be32u(b + at);
  at += 4;
  if (R == 0 || R > (1u << 24)) fail(PH_ERR_INVALID_ARGUMENT, "legacy range index: bad range count");
  need(at + (uint64_t)w * (R + 1) + 8ull * (R + 1));
  // the R + 1 values in the index's type (DataType.size(): 4 for INT / FLOAT, 8 for LONG / DOUBLE)
  auto value = [&](uint32_t r, int64_t* iv, double* dv) {
    const uint8_t* q = b + at + (uint64_t)w * r;
    const uint64_t u = w == 4 ? (uint64_t)be32u(q) : ((uint64_t)be32u(q) << 32) | be32u(q + 4);
    if (*type == "INT") *iv = (int32_t)(uint32_t)u;
    else if (*type == "LONG") *iv = (int64_t)u;
    else if (*type == "FLOAT") {
      const uint32_t x = (uint32_t)u;
      float f;
      memcpy(&f, &x, 4);
      *dv = f;
    } else {
      memcpy(dv, &u, 8);
    }
  };
  starts->assign(R, 0);
  rstarts->assign(R, 0.0);
  for (uint32_t r = 0; r < R; ++r) value(r, &(*starts)[r], &(*rstarts)[r]);
  *last_end = 0;
  *rlast_end = 0.0;
  value(R, last_end, rlast_end);
  at += (uint64_t)w * (R + 1);
  auto off = [&](uint32_t r) {
    return ((uint64_t)be32u(b + at + 8ull * r) << 32) | be32u(b + at + 8ull * r + 4);
  };
  if (off(R) != size) fail(PH_ERR_INVALID_ARGUMENT, "legacy range index: last offset differs from the size");
  cards->assign(R, 0);
  std::vector<RoaringContainer> dir;
  for (uint32_t r = 0; r < R; ++r) {
    const uint64_t s0 = off(r), s1 = off(r + 1);
    if (s1 < s0 || s1 > size) fail(PH_ERR_INVALID_ARGUMENT, "legacy range index: bad offsets");
    dir.clear();
    parse_roaring(b + s0, s1 - s0, s0, dir);
    int64_t docs = 0;
    for (const RoaringContainer& rc : dir) {
      if (rc.type != 2) {
        docs += rc.card;
      } else {
        const uint8_t* q = b + rc.offset + 2;
        for (int32_t j = 0; j < rc.card; ++j) docs += (int64_t)le16(q + 4 * j + 2) + 1;
      }
    }
    (*cards)[r] = docs;
  }
}

// a dictionary column's index is over dictIds ("INT")
void parse_legacy_range_index(const uint8_t* b, uint64_t size, std::vector<int64_t>* starts, int64_t* last_end,
                              std::vector<int64_t>* cards) {
  std::string type;
  std::vector<double> rs;
  double rl = 0;
  parse_legacy_range_index_typed(b, size, &type, starts, last_end, &rs, &rl, cards);
  if (type != "INT") fail(PH_ERR_UNSUPPORTED, "legacy range index over " + type + " values on a dictionary column");
}

// RoaringBitmap's RangeBitmap as BitSlicedRangeIndexCreator.seal writes it after its header (int32 BE version 2,
// int64 BE min; BitSlicedRangeIndexCreator.java:123-133) and BitSlicedRangeIndexReader maps it (:240-244).  The format
// belongs to org.roaringbitmap:RoaringBitmap 0.9.38 (pom.xml), which /root/reference does not vendor; restated from
// its published RangeBitmap.map / Appender.serialize (little-endian throughout):
//   u16 cookie 0xF00D, u8 base (2), u8 slice count S, u16 key count K, u32 row count
//   K masks of ceil(S / 8) bytes: bit i of key k's mask = slice i has a container for key k
//   the containers, key-major, slices ascending: u8 kind (0 bitmap, 1 run, 2 array), u16 size, then 8192 bytes of
//   bitmap / size (start, length - 1) u16 pairs / size u16 values; slice i of key k = the key's rows with bit i CLEAR
// Returns dir[k * S + i] = byte offset (from b) of that container, or -1.  The bytes are pinned by this restatement
// and the test writer only: the reference holds no range-index file (parity unpinned for the byte format).
std::vector<int32_t> parse_range_bitmap(const uint8_t* b, uint64_t size, int64_t num_docs, int32_t* nkeys,
                                        int32_t* nslices, bool* stageable) {
  *stageable = true;
  const uint64_t h = 12;  // Pinot's header
  if (size < h + 10) fail(PH_ERR_INVALID_ARGUMENT, "range index: truncated RangeBitmap header");
  if (size > (uint64_t)INT32_MAX) fail(PH_ERR_UNSUPPORTED, "range index past 2 GiB");
  const uint8_t* r = b + h;
  if (le16(r) != 0xF00D) fail(PH_ERR_INVALID_ARGUMENT, "range index: bad RangeBitmap cookie");
  if (r[2] != 2) fail(PH_ERR_INVALID_ARGUMENT, "range index: unsupported RangeBitmap base");
  const int32_t S = r[3], K = le16(r + 4);
  const uint64_t rows = (uint64_t)r[6] | (uint64_t)r[7] << 8 | (uint64_t)r[8] << 16 | (uint64_t)r[9] << 24;
  if (S < 1 || S > 64) fail(PH_ERR_INVALID_ARGUMENT, "range index: bad slice count");
  if ((int64_t)rows != num_docs || (int64_t)K != (num_docs + 65535) / 65536)
    fail(PH_ERR_INVALID_ARGUMENT, "range index: row / key count differs from the segment's");
  const int32_t bpm = (S + 7) / 8;
  uint64_t at = h + 10 + (uint64_t)K * bpm;
  if (at > size) fail(PH_ERR_INVALID_ARGUMENT, "range index: truncated slice masks");
  std::vector<int32_t> dir((size_t)K * S, -1);
  for (int32_t k = 0; k < K; ++k) {
    const uint8_t* m = r + 10 + (size_t)k * bpm;
    for (int32_t i = 0; i < S; ++i) {
      if (!((m[i >> 3] >> (i & 7)) & 1)) continue;
      if (at + 3 > size) fail(PH_ERR_INVALID_ARGUMENT, "range index: truncated container");
      const int kind = b[at];
      const uint64_t n = le16(b + at + 1);
      const uint64_t body = kind == 0 ? 8192 : kind == 1 ? 4 * n : kind == 2 ? 2 * n : ~0ull;
      if (body == ~0ull) fail(PH_ERR_INVALID_ARGUMENT, "range index: bad container kind");
      if ((kind == 2 && n > 4096) || (kind == 1 && n > 2048))  // k_range_slices stages <= 8 KB of u16 payload
        *stageable = false;
      if (at + 3 + body > size) fail(PH_ERR_INVALID_ARGUMENT, "range index: truncated container");
      dir[(size_t)k * S + i] = (int32_t)at;
      at += 3 + body;
    }
  }
  *nkeys = K;
  *nslices = S;
  return dir;
}

}  // namespace ph
