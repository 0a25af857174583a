// segment.cpp -- pinning immutable segments in HBM (the GPU side of ImmutableSegmentLoader.load).
//
// Input buffers are the column slices of the V3 columns.psf exactly as Pinot maps them
// (SingleFileIndexDirectory.java:279-305, all BIG_ENDIAN):
//   forward index  FixedBitSVForwardIndexWriter.java:39-50 (unsorted) / SortedIndexReaderImpl.java:37-42 (sorted)
//   dictionary     SegmentDictionaryCreator.java:100-276 (sorted, fixed width; STRING zero padded)
//   inverted index BitmapInvertedIndexWriter.java:33-96 (uint32 offsets + portable RoaringBitmap blobs)
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>

#include "ph_internal.h"

namespace ph {

// ------------------------------------------------------------------ device buffer
DeviceBuffer::~DeviceBuffer() {
  if (ptr) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != device) (void)hipSetDevice(device);
    (void)hipFree(ptr);
    if (cur != device) (void)hipSetDevice(cur);
  }
}

void DeviceBuffer::alloc(size_t n, int dev) {
  device = dev;
  bytes = n;
  if (n == 0) n = 16;
  hipError_t e = hipMalloc(&ptr, n);
  if (e != hipSuccess) {
    ptr = nullptr;
    fail(e == hipErrorOutOfMemory ? PH_ERR_OUT_OF_MEMORY : PH_ERR_DEVICE,
         std::string("hipMalloc(") + std::to_string(n) + "): " + hipGetErrorString(e));
  }
}

std::unique_ptr<DeviceBuffer> Context::scratch_acquire(size_t n) {
  n = std::max<size_t>(256, (n + 255) / 256 * 256);
  {
    std::lock_guard<std::mutex> lk(scratch_mu);
    auto it = scratch_free.lower_bound(n);
    if (it != scratch_free.end() && it->first <= n + n / 2 + (1 << 20)) {
      auto b = std::move(it->second);
      scratch_free_bytes -= it->first;
      scratch_free.erase(it);
      return b;
    }
  }
  auto b = std::make_unique<DeviceBuffer>();
  try {
    b->alloc(n, device);
  } catch (const Error&) {
    {
      std::lock_guard<std::mutex> lk(scratch_mu);  // give cached scratch back to the allocator and retry once
      scratch_free.clear();
      scratch_free_bytes = 0;
    }
    b->alloc(n, device);
  }
  return b;
}

void Context::scratch_release(std::unique_ptr<DeviceBuffer> b) {
  if (!b || !b->ptr) return;
  constexpr size_t kMaxCached = size_t(32) << 30;  // keep at most 32 GiB of idle scratch per context (of 288)
  if (b->bytes > kMaxCached) return;
  std::lock_guard<std::mutex> lk(scratch_mu);
  while (scratch_free_bytes + b->bytes > kMaxCached && !scratch_free.empty()) {
    auto it = scratch_free.begin();
    scratch_free_bytes -= it->first;
    scratch_free.erase(it);
  }
  scratch_free_bytes += b->bytes;
  const size_t k = b->bytes;
  scratch_free.emplace(k, std::move(b));
}

// ------------------------------------------------------------------ execution lanes
Lane::Lane(int dev) : device(dev) {
  PH_HIP_CHECK(hipSetDevice(dev));
  PH_HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  PH_HIP_CHECK(hipStreamCreateWithFlags(&stream_b, hipStreamNonBlocking));
  PH_HIP_CHECK(hipEventCreate(&ev_start));
  PH_HIP_CHECK(hipEventCreate(&ev_stop));
  PH_HIP_CHECK(hipEventCreate(&ev_bm0));
  PH_HIP_CHECK(hipEventCreate(&ev_bm1));
  PH_HIP_CHECK(hipEventCreateWithFlags(&ev_uploaded, hipEventDisableTiming));
}

Lane::~Lane() {
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  if (stream_b) (void)hipStreamSynchronize(stream_b);
  if (ev_start) (void)hipEventDestroy(ev_start);
  if (ev_stop) (void)hipEventDestroy(ev_stop);
  if (ev_bm0) (void)hipEventDestroy(ev_bm0);
  if (ev_bm1) (void)hipEventDestroy(ev_bm1);
  if (ev_uploaded) (void)hipEventDestroy(ev_uploaded);
  for (auto e : ev_pool) (void)hipEventDestroy(e);
  if (stream) (void)hipStreamDestroy(stream);
  if (stream_b) (void)hipStreamDestroy(stream_b);
  for (void* p : staging)
    if (p) (void)hipHostFree(p);
}

void* Lane::host_staging(size_t n, int slot) {
  if (n > staging_bytes[slot]) {
    // a pending upload may still read the old block: drain the lane before freeing it
    PH_HIP_CHECK(hipStreamSynchronize(stream));
    if (staging[slot]) PH_HIP_CHECK(hipHostFree(staging[slot]));
    staging[slot] = nullptr;
    size_t sz = std::max<size_t>(n, 1 << 20);
    PH_HIP_CHECK(hipHostMalloc(&staging[slot], sz, hipHostMallocDefault));
    staging_bytes[slot] = sz;
  }
  return staging[slot];
}

hipEvent_t Lane::event(size_t i) {
  while (ev_pool.size() <= i) {
    hipEvent_t e;
    PH_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev_pool.push_back(e);
  }
  return ev_pool[i];
}

std::unique_ptr<Lane> Context::lane_acquire() {
  {
    std::lock_guard<std::mutex> lk(lane_mu);
    if (!lanes_free.empty()) {
      auto l = std::move(lanes_free.back());
      lanes_free.pop_back();
      return l;
    }
  }
  return std::make_unique<Lane>(device);
}

void Context::lane_release(std::unique_ptr<Lane> l) {
  if (!l) return;
  std::lock_guard<std::mutex> lk(lane_mu);
  lanes_free.push_back(std::move(l));
}

Context::~Context() {
  lanes_free.clear();
  for (auto& kv : pinned_free) (void)hipHostFree(kv.second);
}

void* Context::pinned_acquire(size_t n, size_t* cap) {
  n = std::max<size_t>(n, 4096);
  {
    std::lock_guard<std::mutex> lk(pool_mu);
    auto it = pinned_free.lower_bound(n);
    if (it != pinned_free.end() && it->first <= 2 * n) {
      void* p = it->second;
      *cap = it->first;
      pinned_free.erase(it);
      return p;
    }
  }
  void* p = nullptr;
  PH_HIP_CHECK(hipHostMalloc(&p, n, hipHostMallocDefault));
  *cap = n;
  return p;
}

void Context::pinned_release(void* p, size_t cap) {
  std::lock_guard<std::mutex> lk(pool_mu);
  pinned_free.emplace(cap, p);
  size_t total = 0;
  for (auto& kv : pinned_free) total += kv.first;
  while (total > ((size_t)1 << 31) && !pinned_free.empty()) {  // keep at most 2 GiB cached
    auto it = pinned_free.begin();
    total -= it->first;
    (void)hipHostFree(it->second);
    pinned_free.erase(it);
  }
}

// ------------------------------------------------------------------ big-endian readers
static inline uint32_t be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
static inline uint64_t be64(const uint8_t* p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }

// ------------------------------------------------------------------ fixed-bit pack (FixedBitSVForwardIndexWriter)
void fixed_bit_pack_host(const int32_t* ids, int64_t n, int bits, uint8_t* out) {
  // Values are written MSB-first into a big-endian bit stream (PinotDataBitSet.writeInt,
  // PinotDataBitSet.java:138-165).  Parallel over 32-value groups: a group of 32 values occupies
  // exactly `bits` 32-bit words, so threads never share an output byte.
  const int64_t groups = (n + 31) / 32;
  const int64_t nbytes = (n * bits + 7) / 8;
  auto work = [&](int64_t g0, int64_t g1) {
    for (int64_t g = g0; g < g1; ++g) {
      uint64_t acc = 0;
      int nacc = 0;
      int64_t byte = g * 4 * bits;
      const int64_t i1 = std::min<int64_t>(n, (g + 1) * 32);
      for (int64_t i = g * 32; i < i1; ++i) {
        acc = (acc << bits) | ((uint32_t)ids[i] & ((bits == 32) ? 0xffffffffu : ((1u << bits) - 1u)));
        nacc += bits;
        while (nacc >= 8) {
          nacc -= 8;
          if (byte < nbytes) out[byte] = (uint8_t)(acc >> nacc);
          byte++;
        }
      }
      if (nacc > 0 && byte < nbytes) out[byte] = (uint8_t)(acc << (8 - nacc));
    }
  };
  const int64_t nthreads = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  if (groups < 65536 || nthreads <= 1) {
    work(0, groups);
    return;
  }
  std::vector<std::thread> th;
  const int64_t per = (groups + nthreads - 1) / nthreads;
  for (int64_t t = 0; t < nthreads; ++t) {
    const int64_t a = t * per, b = std::min(groups, a + per);
    if (a < b) th.emplace_back(work, a, b);
  }
  for (auto& t : th) t.join();
}

// clearspring MurmurHash.hash(byte[] data, int length, int seed); Java bytes are signed
int32_t murmur_hash_bytes(const uint8_t* data, int32_t length, int32_t seed) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = (uint32_t)(seed ^ length);
  const int32_t len4 = length >> 2;
  for (int32_t i = 0; i < len4; i++) {
    const int32_t i4 = i << 2;
    uint32_t k = (uint32_t)(int32_t)(int8_t)data[i4 + 3];
    k = (k << 8) | data[i4 + 2];
    k = (k << 8) | data[i4 + 1];
    k = (k << 8) | data[i4 + 0];
    k *= m;
    k ^= k >> 24;
    k *= m;
    h *= m;
    h ^= k;
  }
  const int32_t left = length - (len4 << 2);
  if (left != 0) {
    if (left >= 3) h ^= (uint32_t)((int32_t)(int8_t)data[length - 3] << 16);
    if (left >= 2) h ^= (uint32_t)((int32_t)(int8_t)data[length - 2] << 8);
    if (left >= 1) h ^= (uint32_t)(int32_t)(int8_t)data[length - 1];
    h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

// ------------------------------------------------------------------ dictionary
static bool parse_int64(const std::string& s, int64_t* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  errno = 0;
  long long v = strtoll(s.c_str(), &end, 10);
  if (errno != 0 || end != s.c_str() + s.size()) return false;
  *out = v;
  return true;
}

static bool parse_double(const std::string& s, double* out) {
  if (s.empty()) return false;
  char* end = nullptr;
  double v = strtod(s.c_str(), &end);
  if (end != s.c_str() + s.size()) return false;
  *out = v;
  return true;
}

int64_t Dictionary::insertion_index_of(const std::string& literal) const {
  // BaseImmutableDictionary.insertionIndexOf / binarySearch (BaseImmutableDictionary.java:124-245):
  // index when present, else -(insertionPoint) - 1.  Literals are parsed with the column's stored type
  // (PredicateUtils.getStoredValue).
  int64_t lo = 0, hi = size - 1;
  if (type == PH_INT || type == PH_LONG) {
    int64_t iv;
    double dv;
    if (parse_int64(literal, &iv)) {
      while (lo <= hi) {
        int64_t mid = (lo + hi) >> 1;
        if (ints[mid] < iv) lo = mid + 1;
        else if (ints[mid] > iv) hi = mid - 1;
        else return mid;
      }
      return -(lo + 1);
    }
    if (!parse_double(literal, &dv)) fail(PH_ERR_BAD_QUERY, "Cannot convert value: '" + literal + "' to type: INT/LONG");
    while (lo <= hi) {  // non-integral literal: never equal, insertion point by numeric order
      int64_t mid = (lo + hi) >> 1;
      if ((double)ints[mid] < dv) lo = mid + 1;
      else if ((double)ints[mid] > dv) hi = mid - 1;
      else return mid;
    }
    return -(lo + 1);
  }
  if (type == PH_FLOAT || type == PH_DOUBLE) {
    double dv;
    if (!parse_double(literal, &dv)) fail(PH_ERR_BAD_QUERY, "Cannot convert value: '" + literal + "' to type: DOUBLE");
    if (type == PH_FLOAT) dv = (double)(float)dv;
    while (lo <= hi) {
      int64_t mid = (lo + hi) >> 1;
      if (reals[mid] < dv) lo = mid + 1;
      else if (reals[mid] > dv) hi = mid - 1;
      else return mid;
    }
    return -(lo + 1);
  }
  while (lo <= hi) {  // STRING: byte order == code point order for UTF-8
    int64_t mid = (lo + hi) >> 1;
    int c = strings[mid].compare(literal);
    if (c < 0) lo = mid + 1;
    else if (c > 0) hi = mid - 1;
    else return mid;
  }
  return -(lo + 1);
}

int Dictionary::compare(int64_t i, const Dictionary& o, int64_t j) const {
  if (type == PH_STRING) return strings[i].compare(o.strings[j]);
  if (type == PH_INT || type == PH_LONG) return ints[i] < o.ints[j] ? -1 : (ints[i] > o.ints[j] ? 1 : 0);
  return reals[i] < o.reals[j] ? -1 : (reals[i] > o.reals[j] ? 1 : 0);
}

static void parse_dictionary(const ph_column_desc& d, Dictionary* out) {
  const uint8_t* b = static_cast<const uint8_t*>(d.dictionary);
  const int64_t card = d.cardinality;
  out->type = d.data_type;
  out->size = card;
  int width = 0;
  switch (d.data_type) {
    case PH_INT: width = 4; break;
    case PH_LONG: width = 8; break;
    case PH_FLOAT: width = 4; break;
    case PH_DOUBLE: width = 8; break;
    case PH_STRING: width = d.dictionary_entry_size; break;
    default: fail(PH_ERR_INVALID_ARGUMENT, "unknown data type for column " + std::string(d.name));
  }
  if (width <= 0 || (uint64_t)width * card > d.dictionary_size)
    fail(PH_ERR_INVALID_ARGUMENT, "dictionary buffer too small for column " + std::string(d.name));
  switch (d.data_type) {
    case PH_INT:
      out->ints.resize(card);
      for (int64_t i = 0; i < card; ++i) out->ints[i] = (int32_t)be32(b + 4 * i);
      break;
    case PH_LONG:
      out->ints.resize(card);
      for (int64_t i = 0; i < card; ++i) out->ints[i] = (int64_t)be64(b + 8 * i);
      break;
    case PH_FLOAT:
      out->reals.resize(card);
      for (int64_t i = 0; i < card; ++i) {
        uint32_t u = be32(b + 4 * i);
        float f;
        memcpy(&f, &u, 4);
        out->reals[i] = f;
      }
      break;
    case PH_DOUBLE:
      out->reals.resize(card);
      for (int64_t i = 0; i < card; ++i) {
        uint64_t u = be64(b + 8 * i);
        memcpy(&out->reals[i], &u, 8);
      }
      break;
    case PH_STRING:
      out->strings.resize(card);
      for (int64_t i = 0; i < card; ++i) {
        const char* s = reinterpret_cast<const char*>(b + (int64_t)width * i);
        size_t len = strnlen(s, width);  // FixedByteValueReaderWriter: value ends at the first 0 byte
        out->strings[i].assign(s, len);
        out->max_string_len = std::max<int32_t>(out->max_string_len, (int32_t)len);
      }
      break;
  }
}

// ------------------------------------------------------------------ pin
uint64_t next_object_id() {
  static std::atomic<uint64_t> next{1};
  return next++;
}

// The kernels address a packed stream with 32-bit buffer offsets (reg_decode.h reg_load, scan_kernel.h tile loads):
// a stream plus its pad must stay below 2 GiB, else loads past it would read zeros and answer wrongly.
constexpr uint64_t kMaxStreamBytes = 0x7fffffffull - kFwdPadBytes - 4096;

static int bits_for_card(int64_t card) {  // PinotDataBitSet.getNumBitsPerValue(cardinality - 1)
  int bits = 1;
  while (bits < 31 && ((int64_t)1 << bits) < card) bits++;
  return bits;
}

// what ph_segment_pin refuses before touching the device (sizes only: no buffer is read beyond its declared size)
void segment_check_impl(const ph_segment_desc* desc) {
  if (!desc || desc->num_docs < 0 || desc->num_columns < 0 || (desc->num_columns && !desc->columns))
    fail(PH_ERR_INVALID_ARGUMENT, "bad segment descriptor");
  const int64_t n = desc->num_docs;
  for (int ci = 0; ci < desc->num_columns; ++ci) {
    const ph_column_desc& d = desc->columns[ci];
    if (!d.name) fail(PH_ERR_INVALID_ARGUMENT, "column without a name");
    const std::string name = d.name;
    if (!d.forward_index) fail(PH_ERR_INVALID_ARGUMENT, "column " + name + ": missing forward index");
    if (d.hll_log2m < 0 || d.hll_log2m > 16) fail(PH_ERR_INVALID_ARGUMENT, "column " + name + ": hll_log2m");
    // a raw column is dictionary-encoded at pin, where its real cardinality is known: its stream is checked there
    // (a bound from num_docs distinct values would refuse large raw columns whose encoded stream is small)
    if (d.raw_forward_index) continue;
    const int64_t card = d.cardinality;
    if (d.cardinality <= 0 && n > 0) fail(PH_ERR_INVALID_ARGUMENT, "column " + name + ": cardinality <= 0");
    const int bits = bits_for_card(card);
    const uint64_t packed = ((uint64_t)n * (uint64_t)bits + 7) / 8;
    if (packed > kMaxStreamBytes)
      fail(PH_ERR_UNSUPPORTED, "column " + name + ": packed stream of " + std::to_string(packed) +
                                   " bytes is past the 2 GiB range of the kernels' buffer offsets");
    if (!d.is_sorted && d.forward_index_size < packed)
      fail(PH_ERR_INVALID_ARGUMENT, "column " + name + ": forward index too small");
  }
}

// The frame-of-reference value stream of an INT / LONG column (VK_PACKED: value - min in bits(max - min) per doc),
// encoded from the packed dictIds on the pin stream; not built when the range needs 32 bits or more, or when the
// stream would pass the buffer-offset limit (the kernels then gather from the dictionary)
static void build_value_stream(Context* ctx, ph_segment* seg, Column& c, hipStream_t st) {
  c.vpacked_ready = true;
  if (c.data_type != PH_INT && c.data_type != PH_LONG) return;
  if (c.cardinality <= 0 || seg->num_docs == 0) return;
  const int64_t lo = c.dict.ints.front(), hi = c.dict.ints.back();
  const uint64_t range = (uint64_t)hi - (uint64_t)lo;
  int vb = 1;
  while (vb < 64 && (range >> vb) != 0) ++vb;
  if (vb > 31) return;
  const int64_t n = seg->num_docs;
  const size_t bytes = (size_t)((n * vb + 7) / 8);
  if (bytes > kMaxStreamBytes) return;
  const size_t alloc = ((bytes + kFwdPadBytes + 255) / 256) * 256;
  auto buf = std::make_unique<DeviceBuffer>();
  buf->alloc(alloc, ctx->device);
  PH_HIP_CHECK(hipMemsetAsync(buf->ptr, 0, alloc, st));
  launch_encode_values(c.d_fwd.as<uint32_t>(), c.bits, c.d_values.as<int64_t>(), lo, vb, n, buf->as<uint32_t>(), st);
  c.vbase = lo;
  c.vbits = vb;
  seg->device_bytes += (int64_t)alloc;
  c.d_vpacked = std::move(buf);
}

// The column's DISTINCTCOUNTHLL table for log2m: per dictId the (register << 8 | rank) pair clearspring
// HyperLogLog.offer would update for the dictionary value (DistinctCountHLLAggregationFunction.java:438-447), on `st`
// (the caller synchronises)
void build_hll_table(Context* ctx, Column& c, int log2m, hipStream_t st) {
  if (c.hll_tables.count(log2m)) return;
  HllTable t;
  t.buf = std::make_unique<DeviceBuffer>();
  t.buf->alloc(sizeof(uint32_t) * std::max(1, c.cardinality), ctx->device);
  if (c.data_type == PH_STRING) {
    // MurmurHash.hash(String.getBytes()) = hash(bytes, len, -1)
    std::vector<uint32_t> h(c.cardinality);
    for (int32_t i = 0; i < c.cardinality; ++i) {
      const std::string& s = c.dict.strings[i];
      h[i] = hll_entry(murmur_hash_bytes(reinterpret_cast<const uint8_t*>(s.data()), (int32_t)s.size(), -1), log2m);
    }
    copy_h2d_sync(t.buf->ptr, h.data(), sizeof(uint32_t) * h.size());
  } else {
    // INT / LONG -> hashLong((long) value); DOUBLE -> hashLong(doubleToRawLongBits); FLOAT ->
    // hashLong(floatToRawIntBits) (DistinctCountHLLAggregationFunction.java:127-131 offers the Float itself)
    const int32_t kind = c.data_type == PH_DOUBLE ? PH_HLL_HASH_DOUBLE
                         : c.data_type == PH_FLOAT ? PH_HLL_HASH_FLOAT : PH_HLL_HASH_INT;
    launch_hll_table(c.d_values.ptr, kind, c.cardinality, log2m, t.buf->as<uint32_t>(), st);
  }
  c.hll_tables[log2m] = std::move(t);
}

ph_segment* segment_pin_impl(Context* ctx, const ph_segment_desc* desc) {
  segment_check_impl(desc);
  PH_HIP_CHECK(hipSetDevice(ctx->device));
  LaneGuard lg(ctx);
  const hipStream_t st = lg.lane->stream;  // a pin never runs on the caller's external stream
  auto seg = std::make_unique<ph_segment>();
  seg->ctx = ctx;
  seg->name = desc->name ? desc->name : "";
  seg->num_docs = desc->num_docs;
  const int64_t n = desc->num_docs;
  std::vector<int32_t> ids;
  for (int ci = 0; ci < desc->num_columns; ++ci) {
    const ph_column_desc& d = desc->columns[ci];
    if (!d.name) fail(PH_ERR_INVALID_ARGUMENT, "column without a name");
    auto col = std::make_unique<Column>();
    col->name = d.name;
    col->data_type = d.data_type;
    col->cardinality = d.cardinality;
    col->is_sorted = d.is_sorted != 0;
    col->is_raw = d.raw_forward_index != 0;
    if (d.range_index) {
      // BitSlicedRangeIndexReader header: int32 BE version, int64 BE min.  Version 2 (BitSlicedRangeIndexCreator) is
      // exact; a legacy version-1 index (RangeIndexCreator: ranges + a partial scan) is ignored -- the leaf then
      // scans, with the same doc set and that form's own entry count
      if (d.range_index_size < 12) fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": truncated range index");
      const uint8_t* h = static_cast<const uint8_t*>(d.range_index);
      const uint32_t version = (uint32_t)h[0] << 24 | (uint32_t)h[1] << 16 | (uint32_t)h[2] << 8 | h[3];
      col->has_range_index = version == 2;
      col->has_inexact_range_index = version != 2;
      if (version == 1 && !col->is_raw) {
        parse_legacy_range_index(h, d.range_index_size, &col->legacy_starts, &col->legacy_last_end, &col->legacy_cards);
        col->legacy_range = true;
      } else if (version == 1) {  // over the raw values, in the column's stored type
        std::string type;
        parse_legacy_range_index_typed(h, d.range_index_size, &type, &col->legacy_starts, &col->legacy_last_end,
                                       &col->legacy_rstarts, &col->legacy_rlast_end, &col->legacy_cards);
        static const char* const kTypeNames[] = {"INT", "LONG", "FLOAT", "DOUBLE", "STRING"};
        if (d.data_type < PH_INT || d.data_type > PH_DOUBLE || type != kTypeNames[d.data_type])
          fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": legacy range index of type " + type +
                                            " on a column of another stored type");
        col->legacy_raw = true;
      }
    }
    const uint8_t* fwd = static_cast<const uint8_t*>(d.forward_index);
    if (!fwd) fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": missing forward index");
    std::vector<uint8_t> packed;
    const uint8_t* src = fwd;
    uint64_t src_bytes = d.forward_index_size;
    int64_t card = d.cardinality;
    if (col->is_raw) {
      // raw (no-dictionary) column: decode the chunks once, dictionary-encode (rawfwd.cpp) and pin the packed form
      if (d.inverted_index) fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": raw column with an inverted index");
      col->is_sorted = false;
      const int w = (d.data_type == PH_LONG || d.data_type == PH_DOUBLE) ? 8 : 4;
      std::vector<uint8_t> vals((size_t)n * w);
      raw_forward_index_decode(fwd, d.forward_index_size, d.data_type, n, vals.data());
      raw_dictionary_encode(d.data_type, vals.data(), n, &col->dict, &ids);
      card = col->dict.size;
      col->cardinality = (int32_t)card;
    } else {
      if (d.cardinality <= 0 && n > 0) fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": cardinality <= 0");
      if (!d.dictionary) fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": no dictionary and not marked raw");
      parse_dictionary(d, &col->dict);
    }
    const int bits = bits_for_card(card);  // PinotDataBitSet.getNumBitsPerValue(cardinality - 1)
    if (col->is_raw) {
      if (((uint64_t)n * (uint64_t)bits + 7) / 8 > kMaxStreamBytes)
        fail(PH_ERR_UNSUPPORTED, "column " + col->name + ": dictionary-encoded raw stream past the 2 GiB range of the "
                                 "kernels' buffer offsets");
      packed.assign((size_t)((n * bits + 7) / 8), 0);
      fixed_bit_pack_host(ids.data(), n, bits, packed.data());
      src = packed.data();
      src_bytes = packed.size();
    } else if (col->is_sorted) {
      // SortedIndexReaderImpl: int32 BE (start, end) per dictId; expand to the packed fixed-bit form
      if (d.forward_index_size < (uint64_t)8 * d.cardinality)
        fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": sorted index too small");
      col->sorted_ranges.resize(2 * (size_t)d.cardinality);
      ids.assign(n, 0);
      for (int64_t k = 0; k < d.cardinality; ++k) {
        int32_t s = (int32_t)be32(fwd + 8 * k), e = (int32_t)be32(fwd + 8 * k + 4);
        col->sorted_ranges[2 * k] = s;
        col->sorted_ranges[2 * k + 1] = e;
        for (int64_t doc = std::max<int64_t>(s, 0); doc <= e && doc < n; ++doc) ids[doc] = (int32_t)k;
      }
      packed.assign((size_t)((n * bits + 7) / 8), 0);
      fixed_bit_pack_host(ids.data(), n, bits, packed.data());
      src = packed.data();
      src_bytes = packed.size();
    } else {
      if (d.bits_per_element != bits)
        fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": bitsPerElement " + std::to_string(d.bits_per_element) +
                                          " != getNumBitsPerValue(cardinality - 1) = " + std::to_string(bits));
      if (src_bytes < (uint64_t)((n * bits + 7) / 8))
        fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": forward index too small");
    }
    col->bits = bits;
    const size_t fwd_bytes = (size_t)((n * bits + 7) / 8);
    const size_t alloc = ((fwd_bytes + kFwdPadBytes + 255) / 256) * 256;
    col->d_fwd.alloc(alloc, ctx->device);
    PH_HIP_CHECK(hipMemsetAsync(col->d_fwd.ptr, 0, alloc, st));
    PH_HIP_CHECK(hipMemcpyAsync(col->d_fwd.ptr, src, fwd_bytes, hipMemcpyHostToDevice, st));
    seg->device_bytes += alloc;
    // dictionary values widened for arithmetic
    if (d.data_type != PH_STRING) {
      col->d_values.alloc(sizeof(int64_t) * std::max<int64_t>(1, card), ctx->device);
      const void* vsrc = (d.data_type == PH_INT || d.data_type == PH_LONG) ? (const void*)col->dict.ints.data()
                                                                           : (const void*)col->dict.reals.data();
      PH_HIP_CHECK(hipMemcpyAsync(col->d_values.ptr, vsrc, sizeof(int64_t) * card, hipMemcpyHostToDevice,
                                  st));
      seg->device_bytes += col->d_values.bytes;
    }
    if (d.inverted_index && d.inverted_index_size) {
      const uint8_t* inv = static_cast<const uint8_t*>(d.inverted_index);
      if (d.inverted_index_size < (uint64_t)4 * (card + 1))
        fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": inverted index too small");
      col->inverted.assign(inv, inv + d.inverted_index_size);
      build_bitmap_directory(*col);
      col->d_inverted.alloc(d.inverted_index_size + 16, ctx->device);  // + the dword past a bitmap container's end
      PH_HIP_CHECK(hipMemcpyAsync(col->d_inverted.ptr, inv, d.inverted_index_size, hipMemcpyHostToDevice, st));
      seg->device_bytes += d.inverted_index_size;
      // the container directory too, so a query's inverted leaves upload only (dictId -> container range) items
      col->d_dir.alloc(sizeof(RoaringContainer) * std::max<size_t>(1, col->dir.size()), ctx->device);
      if (!col->dir.empty())
        PH_HIP_CHECK(hipMemcpyAsync(col->d_dir.ptr, col->dir.data(), sizeof(RoaringContainer) * col->dir.size(),
                                    hipMemcpyHostToDevice, st));
      seg->device_bytes += col->d_dir.bytes;
    }
    // an exact range index over dictIds: its RangeBitmap pinned with the (key, slice) container directory, so its
    // leaves are evaluated from the bit slices (k_range_slices).  A raw column's index is over raw values (minus the
    // header's min), not the dictIds it is pinned as: its leaves scan the dictIds (same doc set)
    std::vector<int32_t> range_dir;
    bool range_stageable = false;
    if (col->has_range_index && !col->is_raw && d.range_index_size > 12) {
      const uint8_t* ri = static_cast<const uint8_t*>(d.range_index);
      for (int j = 4; j < 12; ++j)
        if (ri[j]) fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": dictionary range index with min != 0");
      range_dir = parse_range_bitmap(ri, d.range_index_size, n, &col->range_nkeys, &col->range_nslices,
                                     &range_stageable);
      if (card > 0 && (uint64_t)(card - 1) >> (col->range_nslices - 1) >> 1)
        fail(PH_ERR_INVALID_ARGUMENT, "column " + col->name + ": range index slices narrower than the dictionary");
    }
    // (an array / run container wider than a bitmap one, which RoaringBitmap never writes: the leaf scans instead)
    if (col->has_range_index && !col->is_raw && d.range_index_size > 12 && !range_dir.empty() &&
        range_stageable) {
      const uint8_t* ri = static_cast<const uint8_t*>(d.range_index);
      col->d_range.alloc(d.range_index_size + 16, ctx->device);  // + the padding k_range_slices' paired loads read
      PH_HIP_CHECK(hipMemcpyAsync(col->d_range.ptr, ri, d.range_index_size, hipMemcpyHostToDevice, st));
      col->d_range_dir.alloc(sizeof(int32_t) * std::max<size_t>(1, range_dir.size()), ctx->device);
      if (!range_dir.empty())
        PH_HIP_CHECK(hipMemcpyAsync(col->d_range_dir.ptr, range_dir.data(), sizeof(int32_t) * range_dir.size(),
                                    hipMemcpyHostToDevice, st));
      seg->device_bytes += col->d_range.bytes + col->d_range_dir.bytes;
      col->range_slices = true;
    }
    // derived streams, on the pin stream: no query builds them (nor waits for one another doing so)
    build_value_stream(ctx, seg.get(), *col, st);
    if (d.hll_log2m > 0) build_hll_table(ctx, *col, d.hll_log2m, st);
    // the caller's buffers may be released after pin returns
    PH_HIP_CHECK(hipStreamSynchronize(st));
    seg->columns[col->name] = std::move(col);
  }
  seg->id = next_object_id();
  ctx->pinned_rows += seg->num_docs;
  return seg.release();
}

}  // namespace ph
