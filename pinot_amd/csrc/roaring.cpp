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


}  // namespace ph
