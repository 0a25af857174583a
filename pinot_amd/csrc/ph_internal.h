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

#include <atomic>
#include <exception>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <vector>

#include "pinot_hip.h"
#include "and_walk.h"

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

// a host -> device copy that has LANDED when this returns: the library's lanes are non-blocking streams, which do not
// order after work on the null stream, and a plain hipMemcpy may return once its source is staged
inline void copy_h2d_sync(void* dst, const void* src, size_t bytes) {
  PH_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, nullptr));
  PH_HIP_CHECK(hipStreamSynchronize(nullptr));
}

// ------------------------------------------------------------------ limits
constexpr int kMaxCols = 12;      // distinct columns referenced by one query
constexpr int kMaxAggs = 8;       // aggregation functions per query
constexpr int kMaxGroupCols = 4;  // group-by columns
constexpr int kMaxProg = 64;      // filter program length per segment
constexpr int kMaxStack = 30;     // filter evaluation stack depth (bits of a uint32)
constexpr int kFwdPadBytes = 1024;  // >= one staged span: the scan reads whole 64-doc words

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

// Single-leaf filters are specialised (the common shapes); anything else runs the postfix program.
enum : int32_t { FK_ALL = 0, FK_RANGE = 1, FK_SET = 2, FK_BITMAP = 3, FK_DOCRANGE = 4, FK_GENERIC = 5, FK_CONJ = 6 };
// FK_CONJ: an AND of up to kMaxConj scan leaves (dictId range or bitset), each on its own LDS-staged stream -- the
// FilterPlanNode shape of multi-predicate WHERE clauses (AndFilterOperator over ScanBasedFilterOperators), decoded
// from the staged tile like a single leaf instead of gathered per doc by the generic program
constexpr int kMaxConj = 4;
constexpr int kSparseBitmaps = 6;  // k_group_sparse: inverted-index doc bitmaps per segment filter
constexpr int kConjSetWords = 256;  // conj_reg.h: a set leaf of <= 8192 dictIds is staged in LDS per chunk

// How an aggregated numeric column is read:
//   VK_PACKED   frame-of-reference stream (value - base) in `bits`, built once per column in HBM from the
//               dictionary-encoded forward index (no per-row dictionary gather on the hot path)
//   VK_DICT_I64 dictId stream + int64 dictionary table      VK_DICT_F64 dictId stream + float64 table
enum : int32_t { VK_PACKED = 0, VK_DICT_I64 = 1, VK_DICT_F64 = 2 };
constexpr int kMaxVals = 4;
constexpr int kMaxHll = 4;

struct DevValCol {
  const uint32_t* fwd;
  const void* table;
  int64_t base;
  int32_t bits;
  int32_t kind;
};

// A packed bit stream the hot loop reads (dictId or frame-of-reference values).  The first `nstage`
// streams of a query are staged per wave through LDS: each wave works on tiles of kTileWords consecutive
// 64-doc words; a tile of a b-bit stream is one contiguous span of kTileWords * 8 * b bytes, moved with
// 16-byte-per-lane coalesced loads (prefetched into registers one tile ahead) and decoded from LDS.
constexpr int kMaxStreams = 8;
constexpr int kMaxStage = kMaxStreams;  // every stream of the hot loop is LDS-staged
constexpr int kMaxTileWords = 32;                    // <= 2048 docs per wave tile (host picks 4..32)
constexpr int kBlock = 256;                          // threads per scan workgroup (4 waves)
constexpr int kWaves = kBlock / 64;
// MODE_PARTITION workgroups are 8 waves sharing ONE set of partition rings (the rings, not the staging, are
// the big LDS item: 8 waves per ring set doubles the resident waves per CU at the same ring footprint)
constexpr int kPartBlock = 512;
constexpr int kPartWaves = kPartBlock / 64;
// k_part_reg (kernel A, register-direct): 4-wave workgroups; a wave tile is 32 words = 2048 docs, lane l owning the
// 32 consecutive docs [32 l, 32 l + 32) of it, whose b-bit values are exactly b dwords of every stream
constexpr int kRegBlock = 256;
constexpr int kRegWaves = kRegBlock / 64;
constexpr int kRegTileWords = 32;
constexpr int kSparseStepWords = 64;              // k_agg_sparse: bitmap words (4096 docs) per wave step
constexpr int kContWords = 1024;                      // k_group_sparse container mode: one 65536-doc container key
                                                      // per chunk (its leaf bitmaps built in LDS once per chunk)
constexpr int kChunkWords = 256;                     // 16384 docs per chunk (a multiple of every round)
constexpr int kInterruptChunks = 8192;               // an interruptible scan checks every 8192 chunks (~134M docs)
// 16-byte-per-lane loads (1 KiB per wave-instruction) a wave keeps in flight per tile, over all streams
constexpr int kPrefetchCount = 8;                    // MODE_COUNT: one stream
constexpr int kPrefetchOther = 12;
constexpr int kPrefetchPartition = 6;                // MODE_PARTITION prefetch pool (r2: 8-word tiles need 5 loads at 10+10+10+20 bits; 12 cost 24 VGPRs)
constexpr int stage_loads(int tile_words, int bits) { return (tile_words * 8 * bits + 8 + 1023) / 1024; }
// staged span of one stream: 16-byte front pad (the decode reads dword j-1 and j) + the tile's bytes.  (r2: staging
// whole 1 KiB pieces without exec branches measured slower -- config2 0.49 -> 0.55 ms -- from the extra LDS writes.)
constexpr int stage_stream_bytes(int tile_words, int bits) { return 16 + (tile_words * 8 * bits + 8 + 15) / 16 * 16; }
struct DevStream {
  const uint32_t* fwd;
  int32_t bits;
  int32_t pad;
};

// One 1 KiB wave-load of a full tile's staged data (precomputed per segment on the host): the piece
// covers bytes [off, off + 1024) of stream `stream`'s span; the span of word w0 starts at fwd + w0 * stride.
struct DevPiece {
  const uint8_t* fwd;  // stream base + off
  int32_t stride;      // bytes per 64-doc word (8 * bits)
  int32_t off;         // byte offset of the piece inside the span
  int32_t lds;         // LDS destination inside the wave's staging area (stage_soff + 16 + off)
  int32_t pad;
};
constexpr int kMaxPieces = 12;  // == kPrefetchOther >= kPrefetchCount

struct RoaringContainer;
struct RoaringRange;

struct DevSegment {
  int32_t num_docs;
  int32_t npieces;
  int32_t fkind;       // FK_*
  int32_t fslot;       // FK_RANGE / FK_SET column slot
  uint32_t flo, flen;  // FK_RANGE: [flo, flo + flen) ; FK_DOCRANGE: [flo, flo + flen) docs
  int32_t prog_off;
  int32_t prog_len;
  int32_t pad;
  const uint32_t* fptr;  // FK_SET bitset over dictIds ; FK_BITMAP doc bitmap
  const uint32_t* keep;  // numGroupsLimit: bitset over global keys this segment may aggregate (nullptr: all)
  int32_t nconj;                    // FK_CONJ leaves
  int32_t conj_nidx;                // FK_CONJ: > 0 when the AND is an applyAnd one -- its first conj_nidx leaves
                                    // are range-index leaves, the rest scans (filter-entry statistic)
  int32_t cstream[kMaxConj];        // FK_CONJ: staged stream of leaf k
  uint32_t clo[kMaxConj], clen[kMaxConj];  // FK_CONJ range leaf k: [clo, clo + clen)
  const uint32_t* cset[kMaxConj];   // FK_CONJ set leaf k: bitset over dictIds (nullptr: range leaf)
  uint32_t* first_doc;              // numGroupsLimit pass: this segment's [num_groups] first matching doc per key
  // k_group_sparse (KParams::group_sparse): the filter as an AND of sp_nbm inverted-index doc bitmaps (ORs of
  // consecutive ones where sp_or is set), then sp_nscan
  // scan leaves (dictId range [sp_lo, sp_lo + sp_len) or bitset sp_set) on column slot sp_slot, evaluated per
  // matched doc by gathers; sp_stats: the AND is an applyAnd one (numEntriesScannedInFilter).  The segment keeps
  // its generic program (fkind) for the numGroupsLimit passes.
  int32_t sp_nbm, sp_nscan, sp_stats;
  int32_t sp_reg;  // no bitmaps: the sp scan leaves are evaluated register-direct per wave step (conj_reg.h)
  const uint32_t* sp_bm[kSparseBitmaps];
  int32_t sp_or[kSparseBitmaps];     // bitmap k ORs into bitmap k - 1's group (an OR of inverted leaves)
  int32_t sp_slot[kMaxConj];
  uint32_t sp_lo[kMaxConj], sp_len[kMaxConj];
  const uint32_t* sp_set[kMaxConj];
  uint32_t* sp_lbits[kMaxConj];  // sp_reg: each scan leaf's doc bitmap (32-doc words), written by the front end for
                                 // the filter statistic's AND walk (null: not needed)
  // k_agg_sparse container mode (KParams::agg_cont): the FK_BITMAP leaf's dictIds as their roaring containers in
  // the column's device directory (the chunks name ranges of them) and the inverted buffer they point into
  const RoaringContainer* cdir;
  const uint8_t* cbase;
  // k_group_sparse container mode (KParams::group_cont): bitmap leaf k as its dictIds' container ranges sp_rng[k]
  // (sp_nrng[k] of them) in the column directory sp_cdir[k], payloads in the inverted buffer sp_cbase[k]
  const RoaringRange* sp_rng[kSparseBitmaps];
  int32_t sp_nrng[kSparseBitmaps];
  const RoaringContainer* sp_cdir[kSparseBitmaps];
  const uint8_t* sp_cbase[kSparseBitmaps];
  const int32_t* sp_ctab;  // [65536-doc key][sp_ntot]: the directory index of range t's container of that key, or -1
  int32_t sp_ntot;         // ranges over all leaves (sum of sp_nrng)
  int32_t pad2;
  // ph_filter_execute (KParams::docset): the segment's doc bitmap, ceil(num_docs / 64) 64-bit words (bit i of word w =
  // doc 64 w + i), written by the MODE_COUNT scans; words outside the scanned chunks stay as zeroed by the host
  uint32_t* docset;
  DevColumn cols[kMaxCols];
  DevValCol vals[kMaxVals];
  DevValCol vals2[kMaxVals];       // second operand of a 2-operand expression term (KParams::val_op)
  DevStream streams[kMaxStreams];  // packed bit streams read by the scan loop (staged ones first)
  DevPiece pieces[kMaxPieces];     // the tile's 1 KiB loads, all streams
};

struct Chunk {
  int32_t seg;
  int32_t word_begin;  // 64-doc words
  int32_t word_end;
  int32_t pad;
};

enum : int32_t { AGG_COUNT = 0, AGG_SUM = 1, AGG_MIN = 2, AGG_MAX = 3, AGG_HLL = 4 };

enum : int32_t {
  MODE_COUNT = 0,
  MODE_AGG = 1,
  MODE_GROUP_LDS = 2,
  MODE_GROUP_GLOBAL = 3,
  MODE_PARTITION = 4,
  MODE_GROUP_HASH = 5,  // key spaces beyond the dense budget: global open-addressing table keyed by the raw key
};
constexpr size_t kUnionCacheEntries = 64;  // segment-set dictionary unions kept per context
constexpr double kDenseTableBudget = 32e9;  // HBM bytes of dense (or hash) group tables one query may allocate
constexpr unsigned long long kHashEmpty = ~0ull;  // empty slot of the MODE_GROUP_HASH key table

constexpr int kPartUnroll = 4;     // 64-doc words per step of the partition append loop (independent LDS chains)
constexpr int kPartSlots = 2048;    // LDS record slots per workgroup (partition p owns slots [p*C, (p+1)*C)); swept r1: small
                                     // slot sets + more resident workgroups beat 8192 slots at 3 WG/CU
constexpr int kPartMaxParts = 1024;
constexpr int kPartKeysLog2 = 12;   // keys per partition = 4096: kernel B's LDS table <= 80 KiB

struct KParams {
  const DevSegment* segs;
  const FilterInsn* prog;
  const Chunk* chunks;
  int32_t chunk_begin;  // this launch covers chunks [chunk_begin, chunk_end)
  int32_t chunk_end;
  int32_t nstage;                 // streams staged through LDS (<= kMaxStage)
  int32_t f_stream;               // FK_RANGE / FK_SET filter column stream
  int32_t g_stream[kMaxGroupCols];
  int32_t v_stream[kMaxVals];
  int32_t v2_stream[kMaxVals];    // stream of an expression term's second operand
  int32_t val_op[kMaxVals];       // ph_expr_op of value term j (0: plain column)
  int32_t stage_off;              // byte offset of the per-wave staging areas in dynamic LDS
  int32_t stage_stride;           // bytes of one wave's staging area
  int32_t tile_words;             // 64-doc words per wave tile
  int32_t late_prefetch;          // decode gathers from HBM: issue the next tile's loads after it
  int32_t stage_soff[kMaxStage];  // byte offset of staged stream s inside a wave's area
  int32_t lds_cnt_off;            // MODE_GROUP_LDS: byte offset of the count table (MODE_GROUP_GLOBAL: cache counts)
  int32_t gc_slots;               // MODE_GROUP_GLOBAL: LDS group cache slots (power of 2; 0 = off)
  int32_t gc_key_off;             // MODE_GROUP_GLOBAL: byte offset of the cache's key array (uint32, ~0u = empty)
  int32_t num_group_cols;
  int32_t group_slot[kMaxGroupCols];
  int64_t group_stride[kMaxGroupCols];
  int64_t num_groups;  // dense key space (1 for aggregation-only)
  int32_t num_vals;               // distinct aggregated value columns
  int32_t num_hll;                // DISTINCTCOUNTHLL register sets
  int32_t log2m;
  int32_t lds_bytes;
  // value-column-centric aggregation state (SUM/MIN/MAX of one column share one decode)
  int32_t val_ops[kMaxVals];      // bit 0 SUM, bit 1 MIN, bit 2 MAX
  int32_t val_is_int[kMaxVals];   // int64 arithmetic (else float64 SUM, order-key MIN/MAX)
  void* out_sum[kMaxVals];        // [num_groups] int64 or double
  int64_t* out_min[kMaxVals];     // [num_groups] int64 order keys
  int64_t* out_max[kMaxVals];
  int32_t lds_sum_off[kMaxVals];  // MODE_GROUP_LDS byte offsets
  int32_t lds_min_off[kMaxVals];
  int32_t lds_max_off[kMaxVals];
  int32_t hll_slot[kMaxHll];      // column slot of each HLL register set
  int32_t lds_hll_off;
  unsigned long long* out_count;  // [num_groups] matched docs per group
  unsigned long long* matched_total;  // group-by plans: matched docs of the launch (numDocsScanned), or nullptr
  unsigned long long* filter_entries; // applyAnd filter entries of the launch (programs with flagged ANDs), or nullptr
  uint32_t* first_doc;            // non-null: this launch is the numGroupsLimit first-seen pass (DevSegment.first_doc)
  unsigned long long* hkeys;      // MODE_GROUP_HASH: [num_groups] slot keys (kHashEmpty = free); out_* by slot
  int64_t hmask;                  // MODE_GROUP_HASH: slots - 1 (a power of two >= 2x the distinct keys possible)
  // MODE_GROUP_HASH numGroupsLimit (one limit segment per launch): the segment's first-seen table -- raw key per slot
  // (lkeys, lmask) -- whose slots the segment's keep bitset (DevSegment.keep) indexes
  unsigned long long* lkeys;
  int64_t lmask;
  uint32_t* out_hll;              // [num_groups][num_hll][2^log2m]
  // MODE_PARTITION (kernel A) -- records to per-partition buffers
  int32_t part_klo;               // key bits kept in a record (keys per partition = 1 << part_klo)
  int32_t part_vbits;             // value-offset bits in a record (0: COUNT only)
  int32_t num_parts;
  int32_t part_load_first;        // lean kernel A: issue the next tile's loads before the flush (tuning)
  int32_t agg_fast;               // MODE_AGG: run k_agg_lean
  int32_t agg_sparse;             // MODE_AGG over selective bitmap leaves: run k_agg_sparse
  int32_t agg_cont;               // k_agg_sparse straight from each segment's roaring containers (no doc bitmaps):
                                  // chunks are container ranges of DevSegment::cdir
  int32_t group_cont;             // k_group_sparse builds each chunk's leaf bitmaps in LDS from the containers
                                  // (no doc bitmaps in HBM): chunks are kChunkWords-aligned, LDS at cont_bm_off
  int32_t cont_bm_off;
  int32_t sparse_c;               // sparse kernels over sp_reg segments: 16-byte loads per lane of a leaf (4 or 8)
  int32_t lds_fast;               // MODE_GROUP_LDS: run k_group_lds_lean
  int32_t lds_pack;               //   COUNT << 40 | SUM in one 64-bit LDS word
  int32_t lds_copies;             //   table copies (one per wave when they fit)
  int32_t lds_copy_bytes;         //   bytes per copy
  int32_t part_cap;               // records per (partition, workgroup) region
  int64_t part_vbase;             // record value = value - part_vbase
  void* part_buf;                 // [gridDim.x][num_parts][part_cap] records: one region per (workgroup, partition)
  uint32_t* part_count;           // [num_parts][gridDim.x] records written per region (may exceed part_cap)
  int32_t pl_slot_off, pl_lcnt_off, pl_bcnt_off, pl_misc_off;  // LDS layout
  int32_t part_slot_log2;         // C = 1 << part_slot_log2 LDS ring slots per partition
  int32_t part_ring_stride;       // k_part_reg: words between consecutive partitions' rings (C + 4: the flush's owner
                                  // threads read their rings at distinct bank offsets)
  int32_t part_set_words;         // k_part_reg: words between its two ring sets (slots; the pending words follow
                                  // pl_lcnt_off at a stride of num_parts + 64)
  int32_t part_fast;              // kernel A may run the lean k_part_scan (no gathers; ALL / RANGE / DOCRANGE leaves)
  int32_t part_depth;             // lean kernel A: tiles of loads in flight per wave (1: k_part_scan, 2: k_part_scan2)
  int32_t part_reg;               // kernel A = k_part_reg (register-direct decode; 0: the LDS-staged forms)
  int32_t part_ck, part_cv;       // k_part_reg: 16-byte loads per lane of a filter / key stream, of the value stream
  int32_t part_sets;              // k_part_reg: ring sets (2: append and flush overlap; 1: half the LDS, more workgroups)
  int32_t count_reg;              // MODE_COUNT: k_count_reg with this many 16-byte loads per lane (ceil(b / 4)); 0 off
  int32_t group_reg;              // MODE_GROUP_LDS: k_group_reg (register-direct, lane-interleaved LDS table)
  int32_t group_sparse;           // MODE_GROUP_LDS / GLOBAL: k_group_sparse (selective bitmap ANDs, DevSegment sp_*)
  int32_t group_reg_lanes_log2;   //   log2 of the slots per key (lane l updates slot key * L + (l & (L - 1)))
  int32_t group_reg_cf, group_reg_cg, group_reg_cv;  // 16-byte loads per lane: filter / each group / value stream
  int32_t docset;                 // MODE_COUNT: every segment's DevSegment::docset receives its doc bitmap
  unsigned long long* ovf_count;  // overflow table (same layout as out_*), merged at the end
  int64_t* ovf_sum;
  int64_t* ovf_min;
  int64_t* ovf_max;
};

// Kernel B of the partitioned group-by: aggregates one batch of records per partition in LDS, then merges
// the partition's key range into the dense result table (each key range has exactly one owner block).
struct PartAggParams {
  const void* part_buf;
  const uint32_t* part_count;  // [num_parts][regions]
  int32_t regions;             // kernel A's grid size
  int32_t num_parts;
  int32_t part_cap;
  int32_t part_klo;
  int32_t part_vbits;
  int32_t rec64;
  int32_t has_sum, has_min, has_max;
  int32_t pack_cs;        // count and value-offset sum share one 64-bit LDS word (count << 40 | sum)
  int32_t slices;         // workgroups per partition (each aggregates a contiguous range of the regions)
  int32_t dbg_unused;     // (layout pad)
  int32_t mm_blind;       // MIN / MAX as one atomic per record each (else read first, atomic only on improvement)
  int32_t pad;
  int64_t part_vbase;
  int64_t num_groups;
  unsigned long long* out_count;
  int64_t* out_sum;
  int64_t* out_min;
  int64_t* out_max;
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

// ------------------------------------------------------------------ dense partial tables (multi-GPU combine)
enum : int32_t { DENSE_LAYOUT = 1, DENSE_EXECUTE = 2, DENSE_FINALIZE = 3 };
struct GlobalDict;
struct DenseArgs {
  int32_t op;
  void* const* tables;     // DENSE_EXECUTE / DENSE_FINALIZE: caller-owned device tables (layout order)
  int64_t g0, g1;          // DENSE_FINALIZE: the key shard [g0, g1) the tables hold
  ph_dense_layout* layout; // DENSE_LAYOUT output
  // group-by dictionaries in group-by order, in place of the context's table dictionaries (the multi-device combine
  // builds one union over every device's segments, one copy per device)
  const std::vector<std::shared_ptr<GlobalDict>>* dicts = nullptr;
  // ph_filter_execute: the call is a COUNT(*) whose scan also writes each segment's doc bitmap into `words` (device
  // memory, zeroed here): segment i's ceil(num_docs / 64) words start at word_off[i]
  struct FilterDocset* docset = nullptr;
  // star-tree views in this call (startree.cpp): a view's filter is its traversal's documents AND the remaining
  // predicates, not the query's filter tree
  const std::map<const ph_segment*, struct StarSegPlan>* star = nullptr;
};
// One star-tree view of a query (StarTreeFilterOperator.getFilterOperator, StarTreeFilterOperator.java:157-199): the
// star-tree documents the traversal matched (sorted, disjoint, inclusive (start, end) pairs), the remaining predicate
// columns' composites in the order the AND receives them (each a list of predicate indices ORed), and whether a
// predicate column matched no dictId (EmptyFilterOperator).
struct StarSegPlan {
  std::vector<int32_t> ranges;
  std::vector<std::vector<int32_t>> composites;
  bool empty = false;
};
struct FilterDocset {
  unsigned long long* words;
  const int64_t* word_off;
  int64_t total_words;
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

struct RoaringContainer {
  int32_t type;      // 0 array, 1 bitmap, 2 run
  int32_t key;       // high 16 bits
  int32_t card;      // array: cardinality; run: number of runs
  int32_t target;    // launch time: index of the leaf's RoaringTarget (its inverted buffer and doc bitmap)
  uint64_t offset;   // byte offset of the payload in the device inverted buffer
};

// one inverted-index leaf of a query: the device inverted buffer its containers point into and its doc bitmap
struct RoaringTarget {
  const uint8_t* base;
  uint32_t* bitmap;
  int32_t num_docs;
  int32_t pad;
};

// one dictId of one inverted leaf: its containers dir[first, first + count) of the leaf's column directory
constexpr int64_t kRoaringWorkContainers = 16;  // containers per RoaringWork item (4 waves x 4)
struct RoaringWork {
  const RoaringContainer* dir;
  int32_t target;  // RoaringTarget index
  int32_t first;
  int32_t count;
  int32_t pad;
};

// chunked bitmap build (k_roaring_chunk): one leaf's target and its dictIds' directory ranges
struct RoaringRange {
  int32_t first;  // dir[first, first + count): one dictId's containers, ascending keys
  int32_t count;
};
struct RoaringLeaf {
  const uint8_t* base;            // device inverted buffer
  const RoaringContainer* dir;    // the column's device directory
  uint32_t* bitmap;               // doc bitmap, padded_words words
  int32_t num_docs;
  int32_t padded_words;
  int32_t ids_first;              // ranges[ids_first, ids_first + ids_count)
  int32_t ids_count;
};
// the chunked build applies when every dictId has at most this many containers (each wave scans them 256 at a time)
constexpr int64_t kRoaringChunkMaxContainers = 1024;

// k_range_slices: one exact bit-sliced range-index leaf (BitSlicedRangeIndexReader.getMatchingDocIds) -- docs whose
// value v has lo <= v <= hi, composed from the RangeBitmap's slices (slice i = the docs whose bit i is 0)
struct RangeSliceLeaf {
  const uint8_t* payload;  // the RangeBitmap bytes after its 12-byte header (device)
  const int32_t* dir;      // [nkeys][nslices]: byte offset in payload of the (key, slice) container, -1 = none
  uint32_t* bitmap;        // doc bitmap, padded_words words
  int32_t num_docs;
  int32_t padded_words;
  int32_t nkeys;
  int32_t nslices;
  uint64_t hi;             // v <= hi (hi < 2^nslices)
  uint64_t lo_m1;          // and, when use_lo, NOT v <= lo - 1
  int32_t use_lo;
  int32_t pad;
};

struct Column {
  std::string name;
  int32_t data_type = PH_INT;
  int32_t cardinality = 0;
  int32_t bits = 1;
  bool is_sorted = false;
  bool is_raw = false;                // pinned from a raw forward index (dictionary-encoded at pin)
  bool has_range_index = false;       // an exact (version 2) bit-sliced range index came with the column
  bool has_inexact_range_index = false;  // a legacy version-1 range index (ranges + a partial scan)
  // the exact index's RangeBitmap parsed at pin (dictionary columns; segment.cpp parse_range_bitmap): leaves are
  // evaluated from its slices by k_range_slices
  bool range_slices = false;
  int32_t range_nkeys = 0, range_nslices = 0;
  DeviceBuffer d_range;                // the RangeBitmap bytes (header + masks + containers)
  DeviceBuffer d_range_dir;            // [nkeys][nslices] container offsets into d_range's container area, -1 none
  // a legacy version-1 index over dictIds (parse_legacy_range_index): range starts, last end, docs per range
  bool legacy_range = false;
  std::vector<int64_t> legacy_starts, legacy_cards;
  int64_t legacy_last_end = 0;
  // ... or over a raw column's values (legacy_raw; RangeIndexCreator of the stored type): INT / LONG starts in
  // legacy_starts, FLOAT / DOUBLE in legacy_rstarts; a RANGE leaf's boundary ranges come from the predicate's raw
  // inclusive bounds (RangeIndexBasedFilterOperator.getPartiallyMatchingDocIds :143-166)
  bool legacy_raw = false;
  std::vector<double> legacy_rstarts;
  double legacy_rlast_end = 0.0;
  Dictionary dict;
  std::vector<int32_t> sorted_ranges;  // [card][2] (sorted columns)
  std::vector<uint8_t> inverted;       // host copy of the inverted index (offsets + roaring blobs)
  DeviceBuffer d_fwd;
  DeviceBuffer d_values;
  DeviceBuffer d_inverted;
  std::mutex cache_mu;
  std::map<int, HllTable> hll_tables;                                // by log2m
  bool vpacked_ready = false;                                        // VK_PACKED stream built
  std::unique_ptr<DeviceBuffer> d_vpacked;
  int64_t vbase = 0;
  int32_t vbits = 0;
  // container directory of the inverted index, parsed once at pin (not per query): the containers of dictId i
  // are dir[dir_begin[i] .. dir_begin[i + 1]); id_docs[i] = its bitmap's cardinality (FastFilteredCount)
  std::vector<RoaringContainer> dir;
  std::vector<int64_t> dir_begin;
  DeviceBuffer d_dir;                  // `dir` in HBM (uploaded at pin): queries name (dictId -> container range) only
  std::vector<int64_t> id_docs;
  bool has_inverted() const { return !inverted.empty(); }
};

struct Context;

// ------------------------------------------------------------------ per-context options (ph_ctx_set_option)
// Plan and kernel-form overrides for tests and tuning sweeps; unset (the default) = the planner's own choice.  The
// product reads no environment: a server process's environment cannot change a query plan.
enum Opt : int {
  OPT_ROARING_ATOMIC,
  OPT_AGG_CONT,
  OPT_GROUP_CONT,
  OPT_DISABLE_PARTITION,
  OPT_LDS_TABLE_MAX,
  OPT_NO_GROUP_CACHE,
  OPT_GROUP_SPARSE,
  OPT_AGG_SPARSE,
  OPT_TILE_WORDS,
  OPT_LIMIT_EAGER,
  OPT_PART_GENERIC,
  OPT_AGG_GENERIC,
  OPT_LDS_GENERIC,
  OPT_COUNT_GENERIC,
  OPT_LDS_LEAN,
  OPT_GROUP_REG_LG,
  OPT_STAT_FUSE,
  OPT_INTERRUPT_CHUNKS,
  OPT_PART_KLO,
  OPT_PART_BATCH_ROWS,
  OPT_PART_FLUSH_FIRST,
  OPT_PART_DEPTH,
  OPT_PART_LDS,
  OPT_PART_SETS,
  OPT_PART_WG_PER_CU,
  OPT_PART_SLICES,
  OPT_PART_MM_BLIND,
  OPT_PART_SERIAL,
  OPT_PART_RING_LOG2,
  OPT_MULTI_HOST_MERGE,
  OPT_SPARSE_C,
  OPT_COUNT
};
constexpr int64_t kOptUnset = INT64_MIN;
extern const char* const kOptNames[OPT_COUNT];

}  // namespace ph

namespace ph {
struct StarTree;
}
struct ph_segment {
  ph::Context* ctx = nullptr;
  std::string name;
  int32_t num_docs = 0;
  int64_t device_bytes = 0;
  uint64_t id = 0;
  std::map<std::string, std::unique_ptr<ph::Column>> columns;
  std::vector<std::unique_ptr<ph::StarTree>> star_trees;  // ph_segment_add_star_tree (startree.cpp)
  int32_t parent_docs = -1;  // a star-tree view: its segment's total docs (numTotalDocs of a star-tree plan)
  ~ph_segment();
};

namespace ph {
// A star-tree of a pinned segment (StarTreeV2): the tree on the host (OffHeapStarTree nodes, 7 ints each: dimension,
// value, start, end, aggregated doc, first child, last child) and its records pinned as a segment of their own -- the
// split-order dimensions with the segment's dictionaries, the count / sum / min / max pair columns as raw columns
struct StarTree {
  std::vector<std::string> dims;
  std::vector<int32_t> nodes;
  int32_t num_nodes = 0;
  std::vector<std::string> pairs;     // every function-column pair of the tree
  std::set<std::string> served;       // the pairs pinned in `view` (count / sum / min / max)
  ph_segment* view = nullptr;         // owned
  ~StarTree();
};
}  // namespace ph

namespace ph {

struct GlobalDict {
  uint64_t id;
  Dictionary dict;
  std::mutex mu;
  std::unique_ptr<DeviceBuffer> d_values;  // int64 (INT/LONG) or float64 (FLOAT/DOUBLE) values, on demand
  // dictId -> id remaps of the segments grouped over this dictionary, by segment id (nullptr = identity); they
  // live and die with the dictionary, and ph_segment_unpin drops a segment's entries (guarded by mu)
  std::map<uint64_t, std::shared_ptr<DeviceBuffer>> remaps;
};

// One execution lane = what a single call needs exclusively: a stream (and a second one for the partitioned
// plan's kernel B), timing events, hand-off events and a pinned host staging block.  Every call takes a lane
// from the context's pool and returns it, so concurrent queries on one context run on their own streams
// (SURVEY.md 8(b) Threading: per-call stream and scratch; operators run on many worker threads).
struct Lane {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream_b = nullptr;
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  hipEvent_t ev_bm0 = nullptr, ev_bm1 = nullptr;  // around the inverted-leaf bitmap build (part of device_ms)
  hipEvent_t ev_uploaded = nullptr;  // the call's segment descriptors and programs are in HBM (statistics pass)
  std::vector<hipEvent_t> ev_pool;
  // slot 0: launch parameters; slot 1: the bitmap build's work items; slot 2: predicate payloads (sets / ranges)
  void* staging[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t staging_bytes[4] = {0, 0, 0, 0};
  explicit Lane(int dev);
  ~Lane();
  void* host_staging(size_t n, int slot = 0);  // valid until the lane's stream passes this call's uploads
  hipEvent_t event(size_t i);  // hand-off event i (created on demand)
};

struct Context {
  Context() {
    for (auto& o : opts) o.store(kOptUnset, std::memory_order_relaxed);
  }
  int device = 0;
  int num_cus = 256;
  std::atomic<int64_t> opts[OPT_COUNT];  // ph_ctx_set_option
  bool has(Opt o) const { return opts[o].load(std::memory_order_relaxed) != kOptUnset; }
  int64_t opt(Opt o) const { return opts[o].load(std::memory_order_relaxed); }
  std::atomic<hipStream_t> ext_stream{nullptr};  // ph_ctx_set_stream: run calls on the caller's stream
  std::mutex mu;  // guards table_dicts and union_cache (held only around their lookups / inserts)
  std::map<std::string, std::shared_ptr<GlobalDict>> table_dicts;   // ph_table_set_dictionary
  std::map<std::string, int32_t> column_types;                      // ph_table_set_column_type (schema)
  std::map<std::string, std::shared_ptr<GlobalDict>> union_cache;   // column + segment-set -> union
  std::deque<std::string> union_order;                              // union_cache keys, oldest first
  // segment / dictionary ids come from one process-wide counter (next_object_id): a multi-device ph_ctx holds one
  // Context per device, and union-cache keys and remaps must not confuse segments of different devices
  std::atomic<int64_t> pinned_rows{0};  // docs of the segments pinned here (multi-device placement: greedy by rows)
  int32_t device_index = 0;             // position in its ph_ctx's device list
  // execution lanes
  std::mutex lane_mu;
  std::vector<std::unique_ptr<Lane>> lanes_free;
  std::unique_ptr<Lane> lane_acquire();
  void lane_release(std::unique_ptr<Lane> l);
  // pinned host blocks for result columns (D2H lands directly in the result; returned on destroy)
  std::mutex pool_mu;
  std::multimap<size_t, void*> pinned_free;
  void* pinned_acquire(size_t n, size_t* cap);
  void pinned_release(void* p, size_t cap);
  // device scratch pool: per-query work buffers (dense group tables, partition buffers, descriptors) are
  // recycled across queries instead of hipMalloc/hipFree per query
  std::mutex scratch_mu;
  std::multimap<size_t, std::unique_ptr<DeviceBuffer>> scratch_free;
  size_t scratch_free_bytes = 0;
  std::unique_ptr<DeviceBuffer> scratch_acquire(size_t n);
  void scratch_release(std::unique_ptr<DeviceBuffer> b);
  ~Context();
};

// A pinned host block of the context's pool held by one call, returned to the pool when the call's scope ends --
// also when it ends by a throw, after draining `st` so no copy into the block is still in flight
struct PinnedBlock {
  Context* ctx;
  hipStream_t st;
  void* p = nullptr;
  size_t cap = 0;
  PinnedBlock(Context* c, hipStream_t s, size_t n) : ctx(c), st(s) { p = c->pinned_acquire(n, &cap); }
  ~PinnedBlock() { release(); }
  void release() {
    if (!p) return;
    if (std::uncaught_exceptions() > 0) (void)hipStreamSynchronize(st);
    ctx->pinned_release(p, cap);
    p = nullptr;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
  PinnedBlock(const PinnedBlock&) = delete;
  PinnedBlock& operator=(const PinnedBlock&) = delete;
};

// RAII lane of one call; stream() is the caller's external stream when one is set (ph_ctx_set_stream)
struct LaneGuard {
  Context* ctx;
  std::unique_ptr<Lane> lane;
  explicit LaneGuard(Context* c) : ctx(c), lane(c->lane_acquire()) {}
  ~LaneGuard() { ctx->lane_release(std::move(lane)); }
  hipStream_t stream() const {
    hipStream_t e = ctx->ext_stream.load();
    return e ? e : lane->stream;
  }
  LaneGuard(const LaneGuard&) = delete;
  LaneGuard& operator=(const LaneGuard&) = delete;
};

// kernels.hip
void launch_scan(const KParams& p, int mode, int ngroup, int rec64, int grid, size_t lds, hipStream_t s);
void launch_part_agg(const PartAggParams& p, size_t lds, hipStream_t s);
size_t part_agg_lds_bytes(const PartAggParams& p);
size_t partition_lds_bytes(KParams& p, int ring_log2 = 5);  // fills the pl_* offsets, returns the dynamic LDS size
int part_reg_blocks_per_cu(const KParams& p, int ng, size_t lds);  // k_part_reg occupancy
void launch_part_reg(const KParams& p, int ng, int grid, size_t lds, hipStream_t s);  // scan_partition_reg.hip
void launch_count_reg(const KParams& p, int grid, hipStream_t s);                      // scan_count_reg.hip
void launch_group_reg(const KParams& p, int ng, int grid, size_t lds, hipStream_t s);   // scan_group_reg.hip
void launch_group_sparse(const KParams& p, int mode, int grid, size_t lds, hipStream_t s);  // scan_group_sparse.hip
struct MergeParams {
  unsigned long long* out_count;
  int64_t* out_sum;
  int64_t* out_min;
  int64_t* out_max;
  const unsigned long long* ovf_count;
  const int64_t* ovf_sum;
  const int64_t* ovf_min;
  const int64_t* ovf_max;
  int64_t n;
};
void launch_merge_overflow(const MergeParams& p, hipStream_t s);
void launch_encode_values(const uint32_t* fwd, int32_t bits, const int64_t* table, int64_t base, int32_t vbits,
                          int64_t n, uint32_t* out, hipStream_t s);
void launch_fill_i64(int64_t* p, int64_t v, int64_t n, hipStream_t s);
void launch_reduce_table(void* dst, const void* src, int64_t n, int32_t op, hipStream_t s);  // dst (op)= src
void launch_fill_identity(void* dst, int64_t n, int32_t op, hipStream_t s);                 // op's identity
enum : int32_t { PH_HLL_HASH_INT = 0, PH_HLL_HASH_DOUBLE = 1, PH_HLL_HASH_FLOAT = 2 };
void launch_hll_table(const void* values, int32_t kind, int64_t n, int log2m, uint32_t* out, hipStream_t s);

void build_bitmap_directory(Column& c);  // at pin, from c.inverted
// at pin: the (key, slice) container directory of an exact range index's RangeBitmap (after Pinot's 12-byte header)
void parse_legacy_range_index(const uint8_t* b, uint64_t size, std::vector<int64_t>* starts, int64_t* last_end,
                              std::vector<int64_t>* cards);
void parse_legacy_range_index_typed(const uint8_t* b, uint64_t size, std::string* type, std::vector<int64_t>* starts,
                                    int64_t* last_end, std::vector<double>* rstarts, double* rlast_end,
                                    std::vector<int64_t>* cards);
std::vector<int32_t> parse_range_bitmap(const uint8_t* b, uint64_t size, int64_t num_docs, int32_t* nkeys,
                                        int32_t* nslices, bool* stageable);
// (column, index id) -> (startOffset, size) of a V3 index_map file (loader.cpp)
typedef std::map<std::pair<std::string, std::string>, std::pair<int64_t, int64_t>> IndexMap;
IndexMap read_index_map(const std::string& path);
ph_segment* segment_pin_impl(Context* ctx, const ph_segment_desc* desc);
ph_segment* segment_load_dir_impl(Context* ctx, const char* dir, const char* const* columns, int32_t num_columns);
int64_t segment_dir_num_docs(const char* dir);  // metadata.properties segment.total.docs, 0 if unreadable
// every container of every (leaf, dictId) work item of a query in one launch (one wave per container)
void launch_roaring_or(const RoaringWork* w, int n, const RoaringTarget* targets, hipStream_t s);
void launch_range_slices(const RangeSliceLeaf* leaves, int nleaves, int max_chunks, hipStream_t s);
void launch_roaring_chunk(const RoaringLeaf* leaves, int nleaves, int max_chunks, const RoaringRange* ranges,
                          hipStream_t s);
void launch_selftest_unpack(const uint32_t* fwd, int64_t n, int bits, int32_t* out, hipStream_t s);
// numGroupsLimit: from each limit segment's first-doc-per-key table (nseg tables of G entries, back to back), the
// bitsets of the keys the reference keeps (nseg x ceil(G/32) words); docbits: nseg x dbw zeroed words; scal: 3 per
// segment (distinct, threshold, reached; zeroed)
void launch_limit_select(const uint32_t* first, int64_t G, int64_t limit, int nseg, int64_t dbw, uint32_t* docbits,
                         uint32_t* keep, unsigned long long* scal, hipStream_t s);
// number of non-zero entries of cnt[0, n) into *out (zeroed by the call)
void launch_count_nonzero(const unsigned long long* cnt, int64_t n, unsigned long long* out, hipStream_t s);
// filter-entry statistic of an AND with a remaining OR (AndDocIdIterator + OrDocIdIterator advance() semantics)
constexpr int kMaxFbProgs = 12;
struct FbJob {
  int32_t seg;                 // device segment
  int32_t nprog;
  int32_t off[kMaxFbProgs], len[kMaxFbProgs];  // sub-programs inside the query's program array
  int32_t row[kMaxFbProgs];    // output row of each sub-program
  int64_t nwords;              // 64-doc words of the segment
  unsigned long long* out;     // [rows][nwords] doc bitmaps
};
void launch_filter_bitmaps(const FilterInsn* prog, const DevSegment* segs, const FbJob& job, hipStream_t s);
// numEntriesScannedInFilter of ANDs of scans: the leap-frog as composed per-chunk transition tables (and_walk.h,
// scan_and_walk.hip); out[slot] = the job's sum of (calls - [match]) + [ends after a match]: entries = numDocs - 1 +
// out.  Each job needs (k + 1) x ngroups table entries, ngroups = ceil(nchunks / and_dfa_block(max_k)).
int and_dfa_block(int32_t max_k);
int and_dfa_chunk_words();  // words of 64 docs per k_and_dfa chunk
void launch_and_walk(const AndWalkJob* jobs, int32_t njobs, int64_t max_groups, int32_t max_k, unsigned long long* out,
                     hipStream_t s);
// the same tables on the host (CPU tests), chunks of 1 << shift docs composed in order: the entries
int64_t and_walk_entries_host(const uint64_t* bits, int k, int64_t num_docs, int shift);
// the doc bitmap of a dictId scan leaf (leaf_bitmaps.hip): RANGE [lo, lo + len) or, with `set`, a dictId bitset over
// `card` ids (<= kLeafSetWords * 32); `out` holds ceil(ndocs / 64) * 2 uint32 words (= the uint64 doc-bitmap words)
constexpr int kLeafSetWords = 4096;
struct LeafJob {
  const uint32_t* fwd;
  int64_t ndocs;
  int32_t bits;
  uint32_t lo, len;
  const uint32_t* set;
  int32_t set_words, card;
  uint32_t* out;
  int64_t out_words;
};
void launch_leaf_bitmaps(const LeafJob* jobs, int32_t njobs, int64_t max_docs, int32_t max_bits, int32_t set_words,
                         hipStream_t s);
// host iterator simulation of the statistic (filter_sim.cpp): the planned filter tree over per-leaf doc bitmaps
enum SimOp { SIM_LEAF = 0, SIM_AND = 1, SIM_OR = 2, SIM_NOT = 3 };
enum SimLeafKind { SIM_SCAN = 0, SIM_SORTED = 1, SIM_BITMAP = 2 };
struct SimLeaf {
  int32_t kind;          // SimLeafKind: which iterator the reference builds for the leaf
  const uint64_t* bits;  // the leaf's doc bitmap (ceil(num_docs / 64) words)
};
struct SimNode {
  int32_t op = SIM_LEAF;
  int32_t priority = 0;  // FilterOperatorUtils.reorderAndFilterChildOperators priority (AND children, stable order)
  int32_t leaf = -1;
  std::vector<SimNode> kids;
};
int64_t simulate_filter_entries(const SimNode& root, const std::vector<SimLeaf>& leaves, int64_t num_docs);
void launch_selftest_staged(const DevSegment* seg, int32_t tile_words, int32_t stage_stride, int64_t n, int32_t* out,
                            hipStream_t s);
// the 1 KiB wave-loads of a full tile of every staged stream of `d` (stage offsets per stream)
void fill_tile_pieces(DevSegment& d, int nstage, const int32_t* stage_soff, int tile_words);

// device-side result compaction of a dense group table (non-empty groups, keys decoded, values converted)
constexpr int kCompactBlocks = 2048;
enum : int32_t { CK_COUNT = 0, CK_INT = 1, CK_REAL_SUM = 2, CK_REAL_ORDER = 3 };
struct CompactParams {
  int64_t num_groups;
  int64_t chunk;  // groups per block
  const unsigned long long* count;
  int32_t num_aggs;
  int32_t num_keys;
  const int64_t* agg_src[kMaxAggs];
  int32_t agg_kind[kMaxAggs];
  double* agg_out[kMaxAggs];
  int64_t key_stride[kMaxGroupCols];
  int64_t key_size[kMaxGroupCols];
  const void* key_table[kMaxGroupCols];  // nullptr: emit the int32 global id (STRING keys)
  int32_t key_type[kMaxGroupCols];
  void* key_out[kMaxGroupCols];
  int64_t* count_out;
  int64_t key_base;          // group id of element 0 (finalizing one key shard of a dense table)
  const unsigned long long* hkeys;  // MODE_GROUP_HASH: slot -> raw key (the key of row g is hkeys[g])
  unsigned long long* blk;   // [kCompactBlocks + 2] counts -> offsets, total at [kCompactBlocks], matched docs
                             // (sum of the group counts = numDocsScanned) at [kCompactBlocks + 1], zeroed by the host
  int32_t* flags;            // bit 0: an integer SUM reached 2^53
};
void launch_compact(const CompactParams& p, hipStream_t s);

// host helpers
int32_t murmur_hash_long(int64_t v);
int32_t murmur_hash_bytes(const uint8_t* data, int32_t len, int32_t seed);
uint32_t hll_entry(int32_t hash, int log2m);
void segment_check_impl(const ph_segment_desc* desc);                    // segment.cpp
uint64_t next_object_id();                                               // segment.cpp
// trim.cpp: per-device results of one query merged keyed by group values (the multi-device host combine)
ph_result* merge_results_by_value(const ph_query* q, const std::vector<std::unique_ptr<ph_result>>& parts);
std::shared_ptr<GlobalDict> union_dictionary(const std::string& col, const std::vector<ph_segment*>& segs);
void build_hll_table(Context* ctx, Column& c, int log2m, hipStream_t st);  // into c.hll_tables (async on st)
void fixed_bit_pack_host(const int32_t* ids, int64_t n, int bits, uint8_t* out);
// raw (no-dictionary) forward indexes (rawfwd.cpp): decode a chunk forward index to native values, and
// dictionary-encode native values (sorted distinct values + per-doc ids)
void raw_forward_index_decode(const uint8_t* buf, uint64_t size, int32_t data_type, int64_t num_docs, void* out);
std::vector<uint8_t> result_to_datatable(const ph_result* r, const ph_query* q, const ph_metadata_entry* extra,
                                         int32_t num_extra);
void raw_dictionary_encode(int32_t data_type, const void* values, int64_t n, Dictionary* dict, std::vector<int32_t>* ids);
// star-trees (startree.cpp): a query whose segments a star-tree serves runs over their views and merges with the rest
// by group value; nullptr when no queried segment takes its star-tree.  `dense_op`: a dense-partials call refuses
// star-tree segments (PH_ERR_UNSUPPORTED) rather than mixing their tables.
ph_result* star_tree_execute(Context* ctx, const ph_query* q, ph_segment* const* segs, int32_t nseg, int dense_op);
bool star_tree_serves_any(const ph_query* q, ph_segment* const* segs, int32_t nseg);
void star_tree_forget(Context& c, ph_segment* seg);  // api.cpp: drop a view's remaps / unions before it is freed
// query.cpp helpers the star-tree planner shares with the scan planner: the dictIds a predicate matches on a column
// (bit per dictId; *always_true / *always_false as the evaluator reports them), and whether a segment's filter is
// answered by FastFilteredCountOperator (COUNT(*) over an index-countable filter, AggregationPlanNode.java:183-188)
std::vector<char> predicate_dict_ids(const ph_predicate& p, const Column& c, bool* always_true, bool* always_false);
bool filter_index_countable(const ph_query* q, ph_segment* seg);

}  // namespace ph

// A result column: small ones live in a host vector, large ones in a pinned block of the context's pool
// (device-compacted results are copied straight into it).
struct ResultBuf {
  std::vector<uint8_t> host;
  void* pinned = nullptr;
  size_t cap = 0;
  size_t n = 0;
  void assign(size_t bytes, uint8_t v) {
    host.assign(bytes, v);
    n = bytes;
  }
  uint8_t* data() { return pinned ? static_cast<uint8_t*>(pinned) : host.data(); }
  const uint8_t* data() const { return pinned ? static_cast<const uint8_t*>(pinned) : host.data(); }
  size_t size() const { return n; }
};

namespace ph {
struct MultiState;  // multi.cpp: placement lock, RCCL communicators
}

// One context per ph_ctx_create (one GPU) or ph_ctx_create_multi (a set of GPUs of one node: one Context each)
struct ph_ctx {
  ph::Context c;                                   // device 0 of the set (a single-device context: the only one)
  std::vector<std::unique_ptr<ph::Context>> more;  // devices 1.. of a multi-device context
  std::vector<ph::Context*> devs;                  // every device's context, devs[0] == &c
  std::vector<int32_t> ordinals;                   // their HIP device ordinals (may repeat: logical shards)
  std::shared_ptr<ph::MultiState> multi;
  int32_t transport = PH_TRANSPORT_PEER;           // merge of the devices' dense partials (ph_ctx_set_multi_transport)
  ~ph_ctx();
};

struct ph_result {
  ph::Context* ctx = nullptr;
  std::vector<int32_t> key_types;
  std::vector<int32_t> key_entry_size;
  std::vector<ResultBuf> keys;   // per group-by column, num_groups * entry_size
  std::vector<int32_t> agg_types;
  std::vector<int32_t> agg_log2m;
  std::vector<ResultBuf> aggs;   // per aggregation
  int64_t num_groups = 0;
  int32_t mode = 0;
  ph_exec_stats stats{};
  ~ph_result() {
    for (auto* v : {&keys, &aggs})
      for (auto& b : *v)
        if (b.pinned && ctx) ctx->pinned_release(b.pinned, b.cap);
  }
};
