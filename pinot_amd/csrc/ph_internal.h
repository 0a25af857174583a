// ph_internal.h -- internal types of libpinot_hip.so shared by the host runtime and the gfx950 kernels.
//
// Device-side layout (per pinned segment, per column):
//   fwd     packed dictIds exactly as FixedBitSVForwardIndexWriter writes them (MSB-first, big-endian),
//           copied verbatim into HBM, padded with 64 zero bytes so the 8-byte look-ahead of the unpack
//           never leaves the allocation.  Sorted columns (whose on-disk forward index is the sorted
//           index) are expanded to the same packed form at pin time so every kernel reads one format.
//   values  dictionary values widened for arithmetic: int64 for INT/LONG, float64 for FLOAT/DOUBLE
//           (the dictionary is sorted, so dictId order == value order).
//   inv     the bitmap inverted index bytes (offsets + portable roaring blobs), decoded on demand into
//           a per-query doc bitmap by k_roaring_or.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "pinot_hip.h"

namespace ph {

// ------------------------------------------------------------------ errors
struct Error {
  int code;
  std::string msg;
};
[[noreturn]] void fail(int code, const std::string& msg);

#define PH_HIP_CHECK(x)                                                                         \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) ::ph::fail(PH_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------ limits
constexpr int kMaxCols = 12;      // distinct columns referenced by one query
constexpr int kMaxAggs = 8;       // aggregation functions per query
constexpr int kMaxGroupCols = 4;  // group-by columns
constexpr int kMaxProg = 64;      // filter program length per segment
constexpr int kMaxStack = 30;     // filter evaluation stack depth (bits of a uint32)
constexpr int kFwdPadBytes = 64;

// ------------------------------------------------------------------ device structs
struct DevColumn {
  const uint32_t* fwd;   // packed big-endian 32-bit words
  const int32_t* remap;  // dictId -> table-level global id (group-by columns); nullptr = identity
  const void* values;    // int64_t* (INT/LONG) or double* (FLOAT/DOUBLE)
  const uint32_t* hll;   // dictId -> (register index << 8) | rank   (DISTINCTCOUNTHLL)
  int32_t bits;
  int32_t cardinality;
};

enum : int32_t {
  OP_RANGE = 0,      // dictId in [lo, lo + len)             (scan leaf, RANGE / EQ)
  OP_SET = 1,        // bit dictId of ptr                    (scan leaf, IN / NOT_IN / NOT_EQ)
  OP_DOCRANGES = 2,  // doc in one of lo (start,end) pairs    (sorted-index leaf)
  OP_BITMAP = 3,     // bit doc of ptr                       (inverted-index leaf)
  OP_AND = 4,
  OP_OR = 5,
  OP_NOT = 6,
  OP_ALL = 7,
  OP_NONE = 8,
};

struct FilterInsn {
  int32_t op;
  int32_t col;        // column slot (RANGE/SET); number of children (AND/OR)
  uint32_t lo;        // RANGE: first dictId; DOCRANGES: number of ranges
  uint32_t len;       // RANGE: number of dictIds
  const uint32_t* ptr;
};

struct DevSegment {
  int32_t num_docs;
  int32_t prog_off;
  int32_t prog_len;
  int32_t fast_range;  // 1: program is a single OP_RANGE on slot fast_col
  int32_t fast_col;
  uint32_t fast_lo, fast_len;
  int32_t pad;
  DevColumn cols[kMaxCols];
};

struct Chunk {
  int32_t seg;
  int32_t word_begin;  // 64-doc words
  int32_t word_end;
  int32_t pad;
};

enum : int32_t { AGG_COUNT = 0, AGG_SUM = 1, AGG_MIN = 2, AGG_MAX = 3, AGG_HLL = 4 };

enum : int32_t { MODE_COUNT = 0, MODE_AGG = 1, MODE_GROUP_LDS = 2, MODE_GROUP_GLOBAL = 3 };

struct KParams {
  const DevSegment* segs;
  const FilterInsn* prog;
  const Chunk* chunks;
  int32_t num_chunks;
  int32_t num_group_cols;
  int32_t group_slot[kMaxGroupCols];
  int64_t group_stride[kMaxGroupCols];
  int64_t num_groups;  // dense key space (1 for aggregation-only)
  int32_t num_aggs;
  int32_t num_hll;
  int32_t log2m;
  int32_t lds_bytes;
  int32_t agg_type[kMaxAggs];
  int32_t agg_slot[kMaxAggs];
  int32_t agg_is_int[kMaxAggs];   // value table is int64 (else double)
  int32_t agg_hll[kMaxAggs];      // HLL register-set index
  int32_t lds_off[kMaxAggs];      // MODE_GROUP_LDS: byte offset of the aggregation's table
  int32_t lds_hll_off;
  unsigned long long* out_count;  // [num_groups] matched docs per group
  void* out_agg[kMaxAggs];        // [num_groups]: int64 SUM / ordered MIN/MAX keys, or double SUM
  uint32_t* out_hll;              // [num_groups][num_hll][2^log2m]
};

// order-preserving int64 key of a double (MIN/MAX of FLOAT/DOUBLE columns)
__host__ __device__ inline int64_t double_order_key(double d) {
  int64_t b;
  __builtin_memcpy(&b, &d, 8);
  return b >= 0 ? b : (b ^ INT64_MAX);
}
__host__ __device__ inline double double_from_order_key(int64_t k) {
  int64_t b = k >= 0 ? k : (k ^ INT64_MAX);
  double d;
  __builtin_memcpy(&d, &b, 8);
  return d;
}

// ------------------------------------------------------------------ device memory
struct DeviceBuffer {
  void* ptr = nullptr;
  size_t bytes = 0;
  int device = 0;
  DeviceBuffer() = default;
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  ~DeviceBuffer();
  void alloc(size_t n, int dev);
  template <class T>
  T* as() const { return reinterpret_cast<T*>(ptr); }
};

// ------------------------------------------------------------------ host-side segment model
struct Dictionary {
  int32_t type = PH_INT;
  int64_t size = 0;
  std::vector<int64_t> ints;           // INT / LONG
  std::vector<double> reals;           // FLOAT (widened) / DOUBLE
  std::vector<std::string> strings;    // STRING
  int32_t max_string_len = 0;

  // BaseImmutableDictionary.indexOf / insertionIndexOf over a literal string
  int64_t insertion_index_of(const std::string& literal) const;
  int64_t index_of(const std::string& literal) const {
    int64_t i = insertion_index_of(literal);
    return i >= 0 ? i : -1;
  }
  int compare(int64_t i, const Dictionary& other, int64_t j) const;  // value order across dictionaries
};

struct HllTable {
  std::unique_ptr<DeviceBuffer> buf;  // uint32 per dictId
};

struct Column {
  std::string name;
  int32_t data_type = PH_INT;
  int32_t cardinality = 0;
  int32_t bits = 1;
  bool is_sorted = false;
  Dictionary dict;
  std::vector<int32_t> sorted_ranges;  // [card][2] (sorted columns)
  std::vector<uint8_t> inverted;       // host copy of the inverted index (offsets + roaring blobs)
  DeviceBuffer d_fwd;
  DeviceBuffer d_values;
  DeviceBuffer d_inverted;
  std::mutex cache_mu;
  std::map<int, HllTable> hll_tables;                                // by log2m
  std::map<uint64_t, std::shared_ptr<DeviceBuffer>> remaps;          // by global dictionary id
  bool has_inverted() const { return !inverted.empty(); }
};

struct Context;

}  // namespace ph

struct ph_segment {
  ph::Context* ctx = nullptr;
  std::string name;
  int32_t num_docs = 0;
  int64_t device_bytes = 0;
  uint64_t id = 0;
  std::map<std::string, std::unique_ptr<ph::Column>> columns;
};

namespace ph {

struct GlobalDict {
  uint64_t id;
  Dictionary dict;
};

struct Context {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  int num_cus = 256;
  std::mutex mu;  // serialises queries on this context
  std::map<std::string, std::shared_ptr<GlobalDict>> table_dicts;   // ph_table_set_dictionary
  std::map<std::string, std::shared_ptr<GlobalDict>> union_cache;   // column + segment-set -> union
  uint64_t next_id = 1;
  // scratch
  std::vector<std::unique_ptr<DeviceBuffer>> scratch;
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  void* host_staging(size_t n);
};

// kernels.hip
void launch_scan(const KParams& p, int mode, int grid, int block, size_t lds, hipStream_t s);
void launch_fill_i64(int64_t* p, int64_t v, int64_t n, hipStream_t s);
void launch_hll_table(const void* values, int32_t is_int, int64_t n, int log2m, uint32_t* out, hipStream_t s);
struct RoaringContainer {
  int32_t type;      // 0 array, 1 bitmap, 2 run
  int32_t key;       // high 16 bits
  int32_t card;      // array: cardinality; run: number of runs
  int32_t pad;
  uint64_t offset;   // byte offset of the payload in the device inverted buffer
};
void launch_roaring_or(const RoaringContainer* c, int n, const uint8_t* base, uint32_t* bitmap, int32_t num_docs,
                       hipStream_t s);
void launch_selftest_unpack(const uint32_t* fwd, int64_t n, int bits, int32_t* out, hipStream_t s);

// host helpers
int32_t murmur_hash_long(int64_t v);
int32_t murmur_hash_bytes(const uint8_t* data, int32_t len, int32_t seed);
uint32_t hll_entry(int32_t hash, int log2m);
void fixed_bit_pack_host(const int32_t* ids, int64_t n, int bits, uint8_t* out);

}  // namespace ph

struct ph_result {
  std::vector<int32_t> key_types;
  std::vector<int32_t> key_entry_size;
  std::vector<std::vector<uint8_t>> keys;   // per group-by column, num_groups * entry_size
  std::vector<int32_t> agg_types;
  std::vector<int32_t> agg_log2m;
  std::vector<std::vector<uint8_t>> aggs;   // per aggregation
  int64_t num_groups = 0;
  ph_exec_stats stats{};
};
