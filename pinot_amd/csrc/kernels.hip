// kernels.hip -- gfx950 (CDNA4, wave64) kernels of the segment filter -> aggregation / group-by path.
//
// One launch covers every segment of a query on this GPU: the host cuts each segment into chunks of
// 64-doc "words" and the persistent grid strides over the chunk list.  Inside a wave, lane l owns doc
// 64*w + l of the current word w, so
//   * every column is decoded with the same doc -> lane mapping whatever its bit width: lane l reads the
//     two big-endian 32-bit words that contain bits [doc*b, doc*b + b) (the 64 lanes of a wave touch
//     one contiguous 8*b-byte span: coalesced, ~2-3 cache lines per column per word), and
//   * the filter result of the wave is a 64-bit ballot = exactly one word of the doc-id bitmap
//     (SVScanDocIdIterator's 256-doc batches become one ballot per 64 docs; popcount = COUNT).
// Aggregation state lives in registers (aggregation-only), in an LDS-private dense group table
// (DictionaryBasedGroupKeyGenerator ArrayBased regime, product of cardinalities small enough for LDS)
// or in an HBM dense table updated with device-scope atomics (large key spaces).
//
// Reference loops replaced (file:line in weixiangsun/pinot):
//   FixedBitIntReader.read32 / PinotDataBitSet.readInt     pinot-segment-local/.../io/util/PinotDataBitSet.java:78-100
//   SVScanDocIdIterator.next + PredicateEvaluator.applySV   pinot-core/.../dociditerators/SVScanDocIdIterator.java:76-98
//   AndDocIdSet / OrDocIdSet / NotDocIdSet                   pinot-core/.../docidsets/AndDocIdSet.java:71-185
//   DefaultGroupByExecutor.process + aggregateGroupBySV      pinot-core/.../groupby/DefaultGroupByExecutor.java:131-148
//   Sum/Count/Min/Max/DistinctCountHLL aggregate*            pinot-core/.../aggregation/function/*.java
//   BitmapInvertedIndexReader.getDocIds + roaring OR         pinot-segment-local/.../readers/BitmapInvertedIndexReader.java:45-62
#include <cstdlib>
#include <type_traits>

#include "ph_internal.h"

namespace ph {

// Segment data lives in HBM: address-space-1 loads emit global_load_* (flat_* would also tick lgkmcnt
// and serialise the LDS staging behind every memory load).
#define PH_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const PH_GLOBAL T*)(p);  // C-style cast = addrspacecast (generic -> global)
}
// Read-only per-query descriptors (segments, chunks, filter programs) are read through the constant address
// space: wave-uniform addresses become scalar loads (s_load, counted by lgkmcnt), so fetching a tile's
// metadata never waits behind the wave's in-flight vector loads (vmcnt is in-order).
#define PH_CONST __attribute__((address_space(4)))
typedef const PH_CONST DevSegment* SegPtr;
typedef const PH_CONST DevColumn& ColRef;
typedef const PH_CONST DevValCol& ValRef;

// Workgroup barrier for LDS hand-offs only.  __syncthreads() is a workgroup-scope fence on every address
// space and waits for all of the wave's outstanding vector loads (vmcnt(0)) -- including the next tile's
// prefetch -- before s_barrier; LDS visibility needs only lgkmcnt(0).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 16-byte load from an 8-byte aligned address (a 64-doc word of a b-bit stream is 8*b bytes)
typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));
__device__ __forceinline__ u32x4a8 gld16a8(const uint8_t* p) {
  return *(const PH_GLOBAL u32x4a8*)(p);
}

__device__ __forceinline__ uint32_t unpack_bits(const uint32_t* __restrict__ fwd, int32_t bits, uint32_t doc) {
  const uint64_t bit = (uint64_t)doc * (uint32_t)bits;
  const uint32_t w = (uint32_t)(bit >> 5);
  const uint32_t sh = (uint32_t)bit & 31u;
  const uint32_t hi = __builtin_bswap32(gld(fwd + w));
  const uint32_t lo = __builtin_bswap32(gld(fwd + w + 1));
  const uint64_t x = ((uint64_t)hi << 32) | lo;
  return (uint32_t)((x << sh) >> (64 - bits));
}

__device__ __forceinline__ uint32_t unpack_col(ColRef c, uint32_t doc) {
  return unpack_bits(c.fwd, c.bits, doc);
}

// Postfix filter program over a bit stack (bit 0 = top).  Control flow is wave-uniform: every lane of a
// wave runs the same instruction sequence on its own doc.
__device__ __forceinline__ bool eval_filter(const PH_CONST FilterInsn* prog, int32_t n, SegPtr S,
                                            uint32_t doc) {
  uint32_t st = 0;
  for (int32_t i = 0; i < n; ++i) {
    const PH_CONST FilterInsn* gi = prog + i;
    FilterInsn in;
    in.op = gi->op;
    in.col = gi->col;
    in.lo = gi->lo;
    in.len = gi->len;
    in.ptr = gi->ptr;
    uint32_t b = 0;
    switch (in.op) {
      case OP_RANGE: {
        const uint32_t v = unpack_col(S->cols[in.col], doc);
        b = (v - in.lo) < in.len;
        st = (st << 1) | b;
        break;
      }
      case OP_SET: {
        const uint32_t v = unpack_col(S->cols[in.col], doc);
        b = (gld(in.ptr + (v >> 5)) >> (v & 31u)) & 1u;
        st = (st << 1) | b;
        break;
      }
      case OP_DOCRANGES: {
        const int32_t* r = reinterpret_cast<const int32_t*>(in.ptr);
        for (uint32_t k = 0; k < in.lo; ++k) b |= (uint32_t)((int32_t)doc >= gld(r + 2 * k)) & (uint32_t)((int32_t)doc <= gld(r + 2 * k + 1));
        st = (st << 1) | b;
        break;
      }
      case OP_BITMAP:
        b = (gld(in.ptr + (doc >> 5)) >> (doc & 31u)) & 1u;
        st = (st << 1) | b;
        break;
      case OP_AND: {
        const uint32_t m = (1u << in.col) - 1u;
        b = (st & m) == m;
        st = ((st >> in.col) << 1) | b;
        break;
      }
      case OP_OR: {
        const uint32_t m = (1u << in.col) - 1u;
        b = (st & m) != 0;
        st = ((st >> in.col) << 1) | b;
        break;
      }
      case OP_NOT:
        st ^= 1u;
        break;
      case OP_ALL:
        st = (st << 1) | 1u;
        break;
      default:  // OP_NONE
        st = st << 1;
        break;
    }
  }
  return st & 1u;
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}

__device__ __forceinline__ uint32_t lanes_below(unsigned long long mask, int lane) {
  return (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
}

// compile-time loop: the body sees `i` as a constant expression, so register arrays never spill
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ tile staging
// A wave tile = p.tile_words consecutive 64-doc words of one chunk.  For each staged stream the tile is one
// contiguous span (a 64-doc word of a b-bit stream is exactly 8*b bytes, so the span starts 8-byte
// aligned) read with 16-byte-per-lane coalesced loads (1 KiB per wave-instruction).  The loads of all
// staged streams share one flat register pool of NL loads per lane, so narrow streams leave room for wide
// ones; the host sizes the tile so every segment's spans fit.  The loads of tile i+1 are issued before
// tile i is decoded (software pipelining), so every wave keeps a whole tile of HBM reads in flight.
template <int NL>
struct Prefetch {
  u32x4 r[NL];
};

template <int NL>
__device__ __forceinline__ void tile_load(SegPtr S, int32_t w0, int32_t nvalid, int lane, Prefetch<NL>& pf) {
  if (nvalid <= 0) return;
  const int np = S->npieces;
  // fixed trip count (no early exit), so the pool is fully unrolled and stays in VGPRs
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    if (k < np) {
      const uint8_t* fwd = S->pieces[k].fwd;
      const int32_t stride = S->pieces[k].stride, off = S->pieces[k].off;
      // bytes of this stream the tile needs (+8: the decode reads the dword after the last value)
      if (off + lane * 16 < nvalid * stride + 8) pf.r[k] = gld16a8(fwd + (size_t)w0 * stride + lane * 16);
    }
  }
}

template <int NL>
__device__ __forceinline__ void tile_store(SegPtr S, int32_t nvalid, uint8_t* wst, int lane, const Prefetch<NL>& pf) {
  if (nvalid > 0) {
    const int np = S->npieces;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const int32_t stride = S->pieces[k].stride, off = S->pieces[k].off, lds = S->pieces[k].lds;
      if (k < np && off + lane * 16 < nvalid * stride + 8) {
        // byte-swap once here (the stream is big-endian) so the decode is one funnel shift per value
        u32x4 v = pf.r[k];
        v.x = __builtin_bswap32(v.x);
        v.y = __builtin_bswap32(v.y);
        v.z = __builtin_bswap32(v.z);
        v.w = __builtin_bswap32(v.w);
        *reinterpret_cast<u32x4*>(wst + lds + lane * 16) = v;
      }
    }
  }
  // every load of this tile has been consumed; saying so explicitly keeps the waitcnt pass from
  // assuming a predicated-off load into the pool is still pending (it would then put vmcnt(0) before
  // each load of the next prefetch, serialising it)
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
}

// Per-lane decode cursor over a staged (byte-swapped) stream.  Doc `lane` of 64-doc word u ends at bit
// e = (64u + lane + 1) * b - 1 of the span; word u+1 starts exactly 2b dwords later, so the dword index
// advances by 2b per word and the in-dword position of the value's last bit never changes: the value is
// alignbit(dw[j-1], dw[j], 31 - (e & 31)) & mask, one funnel shift and one AND.
struct BitCursor {
  const uint32_t* dw;  // dword j of word 0 (dw[-1] is inside the 16-byte front pad for the first doc)
  uint32_t rsh;
  uint32_t mask;
  int32_t step;        // dwords per 64-doc word = 2b
};

__device__ __forceinline__ BitCursor bit_cursor(const uint8_t* stg, int32_t bits, int lane) {
  BitCursor c;
  const uint32_t e1 = (uint32_t)lane * (uint32_t)bits + (uint32_t)bits - 1u;
  c.dw = reinterpret_cast<const uint32_t*>(stg + 16) + (e1 >> 5);
  c.rsh = 31u - (e1 & 31u);
  c.mask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
  c.step = 2 * bits;
  return c;
}

__device__ __forceinline__ uint32_t cursor_value(const BitCursor& c, int u) {
  const uint32_t* w = c.dw + u * c.step;
  return __builtin_amdgcn_alignbit(w[-1], w[0], c.rsh) & c.mask;
}

// value of value-column j for a doc: int64 (integer columns) or float64 (real columns)
__device__ __forceinline__ void read_value(int kind, int64_t base, const void* table, uint32_t x, int64_t& iv,
                                           double& dv) {
  if (kind == VK_PACKED) {
    iv = base + (int64_t)x;
    dv = 0.0;
  } else if (kind == VK_DICT_I64) {
    iv = gld(reinterpret_cast<const int64_t*>(table) + x);
    dv = 0.0;
  } else {
    dv = gld(reinterpret_cast<const double*>(table) + x);
    iv = double_order_key(dv);
  }
}

// ------------------------------------------------------------------ partition slots (MODE_PARTITION)
// Each workgroup owns one region of every partition's buffer (region (partition, blockIdx) is written by
// exactly one workgroup: no global atomics, no cross-workgroup reservations).  Matched records are appended
// straight into per-partition LDS slots (C per partition; one returning LDS atomic per record); a flush
// copies every partition's slots to the end of its region in coalesced runs.  A record that finds its
// partition's slots full goes straight to its final region position (bcnt + rank), so the order of the
// region is exactly the LDS rank order either way; beyond the region capacity it spills to the overflow
// table.

template <int REC64>
__device__ __forceinline__ void part_store(const KParams& p, uint32_t b, uint32_t dst,
                                           typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type r) {
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  if (dst < (uint32_t)p.part_cap) {
    reinterpret_cast<Rec*>(p.part_buf)[((size_t)b * gridDim.x + blockIdx.x) * (size_t)p.part_cap + dst] = r;
  } else {
    // region overflow (skewed keys): aggregate straight into the overflow table
    const uint32_t klo = REC64 ? (uint32_t)((unsigned long long)r >> 32) : (uint32_t)r >> p.part_vbits;
    const uint32_t vo = REC64 ? (uint32_t)r : ((uint32_t)r & (p.part_vbits ? ((1u << p.part_vbits) - 1u) : 0u));
    const int64_t g = ((int64_t)b << p.part_klo) | klo;
    const int64_t v = p.part_vbase + (int64_t)vo;
    atomicAdd(&p.ovf_count[g], 1ull);
    if (p.ovf_sum) atomicAdd(reinterpret_cast<unsigned long long*>(p.ovf_sum) + g, (unsigned long long)v);
    if (p.ovf_min) atomicMin(reinterpret_cast<long long*>(p.ovf_min) + g, (long long)v);
    if (p.ovf_max) atomicMax(reinterpret_cast<long long*>(p.ovf_max) + g, (long long)v);
  }
}

template <int REC64>
__device__ void part_flush(const KParams& p, uint8_t* smem) {
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  const Rec* slots = reinterpret_cast<const Rec*>(smem + p.pl_slot_off);
  uint32_t* lcnt = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  uint32_t* bcnt = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
  const int P = p.num_parts;
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  const int total = P << cl;
#pragma unroll 4
  for (int s = threadIdx.x; s < total; s += kBlock) {
    const uint32_t b = (uint32_t)s >> cl, i = (uint32_t)s & (C - 1u);
    const uint32_t n = lcnt[b];
    if (i < n && i < C) part_store<REC64>(p, b, bcnt[b] + i, slots[s]);
  }
  lds_barrier();
  for (int b = threadIdx.x; b < P; b += kBlock) {
    bcnt[b] += lcnt[b];
    lcnt[b] = 0;
  }
  if (threadIdx.x == 0) *reinterpret_cast<uint32_t*>(smem + p.pl_misc_off) = 0;
  lds_barrier();
}

size_t partition_lds_bytes(KParams& p) {
  const size_t rec = p.part_vbits + p.part_klo > 32 ? 8 : 4;
  size_t o = 0;
  auto place = [&](int32_t& dst, size_t bytes) {
    dst = (int32_t)o;
    o = (o + bytes + 15) / 16 * 16;
  };
  int32_t stage_off = 0;
  place(stage_off, (size_t)kWaves * p.stage_stride);
  p.stage_off = stage_off;
  int slots = kPartSlots;
  if (const char* e = getenv("PH_PART_SLOTS")) slots = std::max(256, atoi(e));  // tuning knob
  int cl = 0;
  while ((p.num_parts << (cl + 1)) <= slots) ++cl;
  p.part_slot_log2 = cl;
  // flush before the next round (<= kWaves * tile_words * 64 records) could overrun the slots on average
  p.part_flush_at = std::max(1, (p.num_parts << cl) - kWaves * p.tile_words * 64);
  place(p.pl_slot_off, (size_t)(p.num_parts << cl) * rec);
  place(p.pl_lcnt_off, 4 * (size_t)p.num_parts);
  place(p.pl_bcnt_off, 4 * (size_t)p.num_parts);
  place(p.pl_misc_off, 64);
  return o;
}

// ------------------------------------------------------------------ the scan kernel
enum : int32_t { OPS_SUM = 1, OPS_MIN = 2, OPS_MAX = 4 };

template <int MODE>
struct NumLoads {
  static constexpr int value = MODE == MODE_COUNT ? kPrefetchCount : (MODE == MODE_PARTITION ? kPrefetchPartition : kPrefetchOther);
};

// Value columns the register state is sized for.  REC64 means 64-bit partition records in MODE_PARTITION; in
// every other mode it selects the single-value-column variant, so a one-column query does not carry the
// accumulators and cursors of kMaxVals columns (r1: 158 VGPRs / 3 waves per SIMD in MODE_AGG otherwise).
template <int MODE, int REC64>
struct ValCap {
  // MODE_PARTITION is only planned for <= 1 value column (query.cpp part_ok)
  static constexpr int value = (MODE == MODE_PARTITION || REC64) ? 1 : kMaxVals;
};

// Per-wave accumulation state of the scan (registers).
struct ScanAcc {
  unsigned long long matched;  // wave-uniform
  int64_t isum[kMaxVals], vmin[kMaxVals], vmax[kMaxVals];
  double dsum[kMaxVals];
};

// One staged tile of one segment: every parameter the inner loop needs is hoisted into (scalar) registers
// once per tile, and the filter kind is a template parameter, so the per-64-doc body is LDS reads + ALU.
template <int MODE, int NG, int REC64, int FK, int LATE>
__device__ __forceinline__ void process_tile(const KParams& p, SegPtr S, uint8_t* smem, const uint8_t* wst, int lane,
                                             int32_t w0, int32_t nvalid, ScanAcc& acc) {
  constexpr int VC = ValCap<MODE, REC64>::value;
  const uint32_t ndocs = (uint32_t)S->num_docs;
  const int m = 1 << p.log2m;
  // filter leaf
  const int fbits = (FK == FK_RANGE || FK == FK_SET) ? S->streams[p.f_stream].bits : 1;
  const BitCursor fcur = bit_cursor(wst + p.stage_soff[p.f_stream], fbits, lane);
  const uint32_t flo = S->flo, flen = S->flen;
  const uint32_t* fptr = S->fptr;
  // group-by key streams
  BitCursor gcur[NG > 0 ? NG : 1];
  const int32_t* gremap[NG > 0 ? NG : 1];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    gcur[g] = bit_cursor(wst + p.stage_soff[p.g_stream[g]], S->streams[p.g_stream[g]].bits, lane);
    gremap[g] = S->cols[p.group_slot[g]].remap;
  }
  // aggregated value streams
  int vkind[kMaxVals];
  int64_t vbase[kMaxVals];
  const void* vtab[kMaxVals];
  BitCursor vcur[kMaxVals];
#pragma unroll
  for (int j = 0; j < VC; ++j) {
    if (MODE == MODE_COUNT || j >= p.num_vals || (MODE == MODE_PARTITION && j > 0)) continue;
    vcur[j] = bit_cursor(wst + p.stage_soff[p.v_stream[j]], S->streams[p.v_stream[j]].bits, lane);
    vkind[j] = S->vals[j].kind;
    vbase[j] = S->vals[j].base;
    vtab[j] = S->vals[j].table;
  }
  uint32_t* lds_cnt = reinterpret_cast<uint32_t*>(smem + p.lds_cnt_off);
  uint32_t* lds_hll = reinterpret_cast<uint32_t*>(smem + p.lds_hll_off);
  uint32_t* pl_n = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off);

  // filter of one 64-doc word, branch-free (bitwise AND, no short-circuit: no exec-mask branches)
  auto filter_word = [&](int u) -> bool {
    const uint32_t doc = (uint32_t)(w0 + u) * 64u + (uint32_t)lane;
    bool hit = doc < ndocs;
    if constexpr (FK == FK_RANGE) {
      hit &= (cursor_value(fcur, u) - flo) < flen;
    } else if constexpr (FK == FK_SET && LATE) {
      const uint32_t v = cursor_value(fcur, u);
      hit &= (bool)((gld(fptr + (v >> 5)) >> (v & 31u)) & 1u);
    } else if constexpr (FK == FK_BITMAP && LATE) {
      hit &= (bool)((gld(fptr + (min(doc, ndocs - 1) >> 5)) >> (doc & 31u)) & 1u);
    } else if constexpr (FK == FK_DOCRANGE) {
      hit &= (doc - flo) < flen;
    } else if constexpr (FK == FK_GENERIC && LATE) {
      if (hit) hit = eval_filter((const PH_CONST FilterInsn*)p.prog + S->prog_off, S->prog_len, S, doc);
    }
    return hit;
  };

  // per-word aggregation of the matched docs
  auto aggregate_word = [&](int u, bool hit, unsigned long long bal) {
    const uint32_t doc = (uint32_t)(w0 + u) * 64u + (uint32_t)lane;
    int64_t vi[VC];
    double vd[VC];
    int64_t key = 0;
#pragma unroll
    for (int j = 0; j < VC; ++j) {
      vi[j] = 0;
      vd[j] = 0.0;
    }
    if (hit) {
#pragma unroll
      for (int j = 0; j < VC; ++j)
        if (j < p.num_vals) {
          if (LATE) read_value(vkind[j], vbase[j], vtab[j], cursor_value(vcur[j], u), vi[j], vd[j]);
          else vi[j] = vbase[j] + (int64_t)cursor_value(vcur[j], u);  // VK_PACKED: no gather
        }
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        uint32_t id = cursor_value(gcur[g], u);
        if (LATE && gremap[g]) id = (uint32_t)gld(gremap[g] + id);
        key += (int64_t)id * p.group_stride[g];
      }
    }

    if constexpr (MODE == MODE_PARTITION) {
      return;
    } else {
      if (!hit) return;
      const int64_t g = key;
      if (MODE == MODE_GROUP_LDS) atomicAdd(&lds_cnt[g], 1u);
      else if (MODE == MODE_GROUP_GLOBAL) atomicAdd(&p.out_count[g], 1ull);
#pragma unroll
      for (int j = 0; j < VC; ++j) {
        if (j >= p.num_vals) continue;
        const int ops = p.val_ops[j];
        const int64_t iv = vi[j];
        if (MODE == MODE_AGG) {
          if (ops & OPS_SUM) {
            if (p.val_is_int[j]) acc.isum[j] += iv; else acc.dsum[j] += vd[j];
          }
          if (ops & OPS_MIN) acc.vmin[j] = iv < acc.vmin[j] ? iv : acc.vmin[j];
          if (ops & OPS_MAX) acc.vmax[j] = iv > acc.vmax[j] ? iv : acc.vmax[j];
        } else {
          void* sb = MODE == MODE_GROUP_LDS ? (void*)(smem + p.lds_sum_off[j]) : p.out_sum[j];
          long long* mnb = MODE == MODE_GROUP_LDS ? reinterpret_cast<long long*>(smem + p.lds_min_off[j])
                                                  : reinterpret_cast<long long*>(p.out_min[j]);
          long long* mxb = MODE == MODE_GROUP_LDS ? reinterpret_cast<long long*>(smem + p.lds_max_off[j])
                                                  : reinterpret_cast<long long*>(p.out_max[j]);
          if (ops & OPS_SUM) {
            if (p.val_is_int[j]) atomicAdd(reinterpret_cast<unsigned long long*>(sb) + g, (unsigned long long)iv);
            else atomicAdd(reinterpret_cast<double*>(sb) + g, vd[j]);
          }
          if (ops & OPS_MIN) atomicMin(mnb + g, (long long)iv);
          if (ops & OPS_MAX) atomicMax(mxb + g, (long long)iv);
        }
      }
#pragma unroll
      for (int h = 0; h < kMaxHll; ++h) {
        if (!LATE || h >= p.num_hll) continue;
        ColRef col = S->cols[p.hll_slot[h]];
        const uint32_t e = gld(col.hll + unpack_col(col, doc));
        const int64_t ri = (g * p.num_hll + h) * m + (e >> 8);
        if (MODE == MODE_GROUP_GLOBAL) atomicMax(&p.out_hll[ri], e & 0xffu);
        else atomicMax(&lds_hll[ri], e & 0xffu);
      }
    }
  };

  // 4 words per step: their filter decodes are independent, so their LDS reads (and bitmap gathers) overlap
  constexpr int UB = 4;
  if constexpr (MODE == MODE_PARTITION) {
    constexpr int UB = kPartUnroll;
    // lean path: <= 1 value column (the host only plans MODE_PARTITION for that shape).  Records are
    // (key low bits << vbits | value - vbase); the partition (key high bits) picks the LDS slot run.
    using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
    const uint32_t kmask = (1u << p.part_klo) - 1u;
    Rec* slots = reinterpret_cast<Rec*>(smem + p.pl_slot_off);
    uint32_t* lcnt = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
    const uint32_t* bcnt = reinterpret_cast<const uint32_t*>(smem + p.pl_bcnt_off);
    const int cl = p.part_slot_log2;
    const uint32_t C = 1u << cl;
    for (int u = 0; u < nvalid; u += UB) {
      bool hit[UB];
      uint32_t tot = 0;
#pragma unroll
      for (int q = 0; q < UB; ++q) hit[q] = (u + q < nvalid) ? filter_word(u + q) : false;
#pragma unroll
      for (int q = 0; q < UB; ++q) tot += (uint32_t)__popcll(__ballot(hit[q]));
      acc.matched += tot;
      if (tot == 0 || (p.dbg_flags & 4)) continue;
      if (lane == 0) atomicAdd(pl_n, tot);
      uint32_t bk[UB], rk[UB];
      Rec rec[UB];
#pragma unroll
      for (int q = 0; q < UB; ++q) {
        // without gathers, keys and values are decoded for every lane (branch-free; a miss reads in-tile LDS
        // bytes and discards them): only the rank atomic and the slot store are predicated.  Gathers (LATE:
        // remaps, dictionaries) stay predicated so a miss never indexes a table with a stale id.
        if (LATE && !hit[q]) continue;
        uint32_t key = 0;
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          uint32_t id = cursor_value(gcur[g], u + q);
          if (LATE && gremap[g]) id = (uint32_t)gld(gremap[g] + id);
          key += id * (uint32_t)p.group_stride[g];
        }
        if (p.dbg_flags & 16) key = ((uint32_t)lane * 16411u + (uint32_t)(u + q) * 977u) % (uint32_t)p.num_groups;  // timing only: no key decode
        uint32_t vo = 0;
        if (p.num_vals && !(p.dbg_flags & 16)) {
          int64_t iv;
          double dv;
          if (LATE) read_value(vkind[0], vbase[0], vtab[0], cursor_value(vcur[0], u + q), iv, dv);
          else iv = vbase[0] + (int64_t)cursor_value(vcur[0], u + q);  // VK_PACKED: no gather
          vo = (uint32_t)(iv - p.part_vbase);
        }
        bk[q] = key >> p.part_klo;
        rec[q] = REC64 ? (Rec)(((unsigned long long)(key & kmask) << 32) | vo) : (Rec)(((key & kmask) << p.part_vbits) | vo);
        if (hit[q]) rk[q] = (p.dbg_flags & 8) ? 0u : atomicAdd(&lcnt[bk[q]], 1u);  // flag 8 (timing only): no rank atomic
      }
#pragma unroll
      for (int q = 0; q < UB; ++q) {
        if (!hit[q]) continue;
        if (rk[q] < C) slots[(bk[q] << cl) + rk[q]] = rec[q];
        else part_store<REC64>(p, bk[q], bcnt[bk[q]] + rk[q], rec[q]);  // slots full: straight to HBM
      }
    }
    return;
  }
  int u = 0;
  for (; u + UB <= nvalid; u += UB) {
    bool hit[UB];
    unsigned long long bal[UB];
#pragma unroll
    for (int q = 0; q < UB; ++q) hit[q] = filter_word(u + q);
#pragma unroll
    for (int q = 0; q < UB; ++q) {
      bal[q] = __ballot(hit[q]);
      acc.matched += __popcll(bal[q]);
    }
    if constexpr (MODE != MODE_COUNT) {
#pragma unroll
      for (int q = 0; q < UB; ++q)
        if (bal[q]) aggregate_word(u + q, hit[q], bal[q]);
    }
  }
  for (; u < nvalid; ++u) {
    const bool hit = filter_word(u);
    const unsigned long long bal = __ballot(hit);
    acc.matched += __popcll(bal);
    if constexpr (MODE != MODE_COUNT) {
      if (bal) aggregate_word(u, hit, bal);
    }
  }
}

// Persistent grid over the chunk list.  A chunk (<= 256 words of one segment) is processed in rounds: in
// round r wave w takes tile r * kWaves + w.  Rounds are workgroup-uniform (MODE_PARTITION flushes at round
// boundaries with workgroup barriers); the other modes never synchronise inside the loop.
template <int MODE, int NG, int REC64, int LATE>
__global__ void __launch_bounds__(kBlock) k_scan(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NL = NumLoads<MODE>::value;
  constexpr int VC = ValCap<MODE, REC64>::value;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform
  const int m = 1 << p.log2m;
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;

  uint32_t* lds_cnt = reinterpret_cast<uint32_t*>(smem + p.lds_cnt_off);
  uint32_t* lds_hll = reinterpret_cast<uint32_t*>(smem + p.lds_hll_off);
  uint8_t* wst = smem + p.stage_off + (size_t)wave * p.stage_stride;
  uint32_t* pl_n = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off);
  if (MODE == MODE_GROUP_LDS) {
    for (int64_t g = threadIdx.x; g < p.num_groups; g += kBlock) lds_cnt[g] = 0;
#pragma unroll
    for (int j = 0; j < VC; ++j) {
      if (j >= p.num_vals) continue;
      const int ops = p.val_ops[j];
      for (int64_t g = threadIdx.x; g < p.num_groups; g += kBlock) {
        if (ops & OPS_SUM) reinterpret_cast<int64_t*>(smem + p.lds_sum_off[j])[g] = 0;  // 0 == +0.0
        if (ops & OPS_MIN) reinterpret_cast<int64_t*>(smem + p.lds_min_off[j])[g] = INT64_MAX;
        if (ops & OPS_MAX) reinterpret_cast<int64_t*>(smem + p.lds_max_off[j])[g] = INT64_MIN;
      }
    }
    const int64_t nh = p.num_groups * p.num_hll * m;
    for (int64_t i = threadIdx.x; i < nh; i += kBlock) lds_hll[i] = 0;
  } else if (MODE == MODE_AGG) {
    for (int i = threadIdx.x; i < p.num_hll * m; i += kBlock) lds_hll[i] = 0;
  } else if (MODE == MODE_PARTITION) {
    if (threadIdx.x == 0) *pl_n = 0;
    uint32_t* lcnt = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
    uint32_t* bcnt = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
    for (int i = threadIdx.x; i < p.num_parts; i += kBlock) lcnt[i] = bcnt[i] = 0;
  }
  __syncthreads();

  ScanAcc acc;
  acc.matched = 0;
#pragma unroll
  for (int j = 0; j < VC; ++j) {
    acc.isum[j] = 0;
    acc.dsum[j] = 0.0;
    acc.vmin[j] = INT64_MAX;
    acc.vmax[j] = INT64_MIN;
  }

  // ---- round iterator: (chunk c, round r); the tile of this wave starts at word w0 and has nvalid words
  const int32_t tw = p.tile_words;
  const int32_t round_words = kWaves * tw;
  // each workgroup takes a contiguous run of chunks (mostly one segment: its descriptor stays in the
  // scalar cache, and neighbouring tiles are neighbours in HBM)
  const int64_t nch = p.chunk_end - p.chunk_begin;
  int32_t c = p.chunk_begin + (int32_t)(nch * blockIdx.x / gridDim.x), r = 0;
  const int32_t c_end = p.chunk_begin + (int32_t)(nch * (blockIdx.x + 1) / gridDim.x);
  int32_t cseg = 0, cbeg = 0, cend = 0;
  SegPtr S = nullptr;
  int32_t w0 = 0, nvalid = 0;
  auto locate = [&]() {
    if (c < c_end) {
      cseg = chunks[c].seg;
      cbeg = chunks[c].word_begin;
      cend = chunks[c].word_end;
      S = segs + cseg;
      w0 = cbeg + r * round_words + wave * tw;
      nvalid = min(tw, cend - w0);
    }
  };
  auto advance = [&]() {
    if (cbeg + (r + 1) * round_words < cend) {
      ++r;
    } else {
      ++c;
      r = 0;
    }
  };
  Prefetch<NL> pf;
  locate();
  if (c < c_end) tile_load<NL>(S, w0, nvalid, lane, pf);

  unsigned long long t_stage = 0, t_proc = 0, t_sync = 0, t0 = 0, t1 = 0;
  const bool stamps = p.dbg != nullptr;
  while (c < c_end) {
    if (stamps) t0 = __builtin_readcyclecounter();
    // stage the prefetched tile, then prefetch the next one of this wave
    tile_store<NL>(S, nvalid, wst, lane, pf);
    if (MODE == MODE_PARTITION) {
      // flush the slots filled in the previous round here, before this round's prefetch: the stores then
      // complete under the decode instead of stalling the next tile_store (stores count in vmcnt too)
      const uint32_t n = *pl_n;
      lds_barrier();  // every wave has read n before anyone appends again
      if (n >= (uint32_t)p.part_flush_at && !(p.dbg_flags & 2)) part_flush<REC64>(p, smem);
    }
    SegPtr cs = S;
    const int32_t cw0 = w0, cnvalid = nvalid;
    advance();
    locate();
    // early prefetch overlaps the next tile's loads with this tile's decode; a tile whose decode gathers
    // from HBM (bitsets, remaps, dictionaries) would wait behind them (vmcnt is in-order): prefetch late
    if (!LATE && c < c_end) tile_load<NL>(S, w0, nvalid, lane, pf);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (stamps) {
      t1 = __builtin_readcyclecounter();
      t_stage += t1 - t0;
      t0 = t1;
    }

    if (cnvalid > 0) {
      switch (cs->fkind) {
        case FK_ALL: process_tile<MODE, NG, REC64, FK_ALL, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_RANGE: process_tile<MODE, NG, REC64, FK_RANGE, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_SET: process_tile<MODE, NG, REC64, FK_SET, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_BITMAP: process_tile<MODE, NG, REC64, FK_BITMAP, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_DOCRANGE:
          process_tile<MODE, NG, REC64, FK_DOCRANGE, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc);
          break;
        default: process_tile<MODE, NG, REC64, FK_GENERIC, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
      }
    }
    if (LATE && c < c_end) tile_load<NL>(S, w0, nvalid, lane, pf);
    if (stamps) {
      t1 = __builtin_readcyclecounter();
      t_proc += t1 - t0;
      t0 = t1;
    }
    if (MODE == MODE_PARTITION) {
      lds_barrier();  // this round's appends are complete before the next round's flush check
      if (stamps) t_sync += __builtin_readcyclecounter() - t0;
    }
  }
  if (stamps && threadIdx.x == 0) {
    p.dbg[4 * blockIdx.x + 0] = t_stage;
    p.dbg[4 * blockIdx.x + 1] = t_proc;
    p.dbg[4 * blockIdx.x + 2] = t_sync;
    p.dbg[4 * blockIdx.x + 3] = 1;
  }

  // ---- workgroup epilogue
  if (MODE == MODE_PARTITION) {
    lds_barrier();
    if (*pl_n) part_flush<REC64>(p, smem);
    const uint32_t* bcnt = reinterpret_cast<const uint32_t*>(smem + p.pl_bcnt_off);
    for (int i = threadIdx.x; i < p.num_parts; i += kBlock) p.part_count[(size_t)i * gridDim.x + blockIdx.x] = bcnt[i];
    return;
  }
  const unsigned long long matched = acc.matched;
  __shared__ unsigned long long s_matched;
  if (threadIdx.x == 0) s_matched = 0;
  __syncthreads();
  if (lane == 0 && matched) atomicAdd(&s_matched, matched);
  if (MODE == MODE_AGG) {
    __shared__ int64_t s_isum[kWaves][kMaxVals], s_min[kWaves][kMaxVals], s_max[kWaves][kMaxVals];
    __shared__ double s_dsum[kWaves][kMaxVals];
#pragma unroll
    for (int j = 0; j < VC; ++j) {
      if (j >= p.num_vals) continue;
      const int64_t si = wave_sum_i64(acc.isum[j]);
      const double sd = wave_sum_f64(acc.dsum[j]);
      const int64_t mn = wave_min_i64(acc.vmin[j]);
      const int64_t mx = wave_max_i64(acc.vmax[j]);
      if (lane == 0) {
        s_isum[wave][j] = si;
        s_dsum[wave][j] = sd;
        s_min[wave][j] = mn;
        s_max[wave][j] = mx;
      }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)p.num_vals) {
      const int j = threadIdx.x;
      int64_t si = s_isum[0][j], mn = s_min[0][j], mx = s_max[0][j];
      double sd = s_dsum[0][j];
      for (int wv = 1; wv < kWaves; ++wv) {
        si += s_isum[wv][j];
        sd += s_dsum[wv][j];
        mn = s_min[wv][j] < mn ? s_min[wv][j] : mn;
        mx = s_max[wv][j] > mx ? s_max[wv][j] : mx;
      }
      const int ops = p.val_ops[j];
      if (ops & OPS_SUM) {
        if (p.val_is_int[j]) atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum[j]), (unsigned long long)si);
        else atomicAdd(reinterpret_cast<double*>(p.out_sum[j]), sd);
      }
      if (ops & OPS_MIN) atomicMin(reinterpret_cast<long long*>(p.out_min[j]), (long long)mn);
      if (ops & OPS_MAX) atomicMax(reinterpret_cast<long long*>(p.out_max[j]), (long long)mx);
    }
    for (int i = threadIdx.x; i < p.num_hll * m; i += kBlock)
      if (lds_hll[i]) atomicMax(&p.out_hll[i], lds_hll[i]);
  }
  if (MODE == MODE_GROUP_LDS) {
    __syncthreads();
    for (int64_t g = threadIdx.x; g < p.num_groups; g += kBlock) {
      const uint32_t cnt = lds_cnt[g];
      if (!cnt) continue;
      atomicAdd(&p.out_count[g], (unsigned long long)cnt);
#pragma unroll
      for (int j = 0; j < VC; ++j) {
        if (j >= p.num_vals) continue;
        const int ops = p.val_ops[j];
        if (ops & OPS_SUM) {
          if (p.val_is_int[j])
            atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum[j]) + g,
                      reinterpret_cast<const unsigned long long*>(smem + p.lds_sum_off[j])[g]);
          else
            atomicAdd(reinterpret_cast<double*>(p.out_sum[j]) + g,
                      reinterpret_cast<const double*>(smem + p.lds_sum_off[j])[g]);
        }
        if (ops & OPS_MIN)
          atomicMin(reinterpret_cast<long long*>(p.out_min[j]) + g,
                    reinterpret_cast<const long long*>(smem + p.lds_min_off[j])[g]);
        if (ops & OPS_MAX)
          atomicMax(reinterpret_cast<long long*>(p.out_max[j]) + g,
                    reinterpret_cast<const long long*>(smem + p.lds_max_off[j])[g]);
      }
    }
    const int64_t nh = p.num_groups * p.num_hll * m;
    for (int64_t i = threadIdx.x; i < nh; i += kBlock)
      if (lds_hll[i]) atomicMax(&p.out_hll[i], lds_hll[i]);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_matched && (MODE == MODE_COUNT || MODE == MODE_AGG))
    atomicAdd(&p.out_count[0], s_matched);
}

template <class K>
static void allow_lds(K kernel, size_t lds) {
  // kernels that use more than the default 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU)
  if (lds > 64 * 1024)
    PH_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
}

template <int MODE, int NG, int REC64>
static void launch_late(const KParams& p, int grid, size_t lds, hipStream_t s) {
  if (p.late_prefetch) {
    allow_lds(k_scan<MODE, NG, REC64, 1>, lds);
    hipLaunchKernelGGL((k_scan<MODE, NG, REC64, 1>), dim3(grid), dim3(kBlock), lds, s, p);
  } else {
    allow_lds(k_scan<MODE, NG, REC64, 0>, lds);
    hipLaunchKernelGGL((k_scan<MODE, NG, REC64, 0>), dim3(grid), dim3(kBlock), lds, s, p);
  }
}

template <int MODE, int NG>
static void launch_ng(const KParams& p, int rec64, int grid, size_t lds, hipStream_t s) {
  if (rec64) launch_late<MODE, NG, 1>(p, grid, lds, s);
  else launch_late<MODE, NG, 0>(p, grid, lds, s);
}

template <int MODE>
static void launch_mode(const KParams& p, int ng, int rec64, int grid, size_t lds, hipStream_t s) {
  switch (ng) {
    case 1: launch_ng<MODE, 1>(p, rec64, grid, lds, s); break;
    case 2: launch_ng<MODE, 2>(p, rec64, grid, lds, s); break;
    case 3: launch_ng<MODE, 3>(p, rec64, grid, lds, s); break;
    default: launch_ng<MODE, 4>(p, rec64, grid, lds, s); break;
  }
}

void launch_scan(const KParams& p, int mode, int ng, int rec64, int grid, size_t lds, hipStream_t s) {
  switch (mode) {
    case MODE_COUNT: launch_late<MODE_COUNT, 0, 0>(p, grid, lds, s); break;
    case MODE_AGG:
      if (p.num_vals <= 1) launch_late<MODE_AGG, 0, 1>(p, grid, lds, s);  // ValCap 1
      else launch_late<MODE_AGG, 0, 0>(p, grid, lds, s);
      break;
    case MODE_GROUP_LDS: launch_mode<MODE_GROUP_LDS>(p, ng, p.num_vals <= 1 ? 1 : 0, grid, lds, s); break;
    case MODE_GROUP_GLOBAL: launch_mode<MODE_GROUP_GLOBAL>(p, ng, p.num_vals <= 1 ? 1 : 0, grid, lds, s); break;
    default: launch_mode<MODE_PARTITION>(p, ng, rec64, grid, lds, s); break;
  }
  PH_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ kernel B: partition aggregation
// One workgroup per partition: every record of the partition (every region kernel A wrote) goes through an
// LDS table of the partition's keys, then the workgroup merges its key range into the dense result table
// (each key range has exactly one owner, so the merge needs no atomics).  Region fill levels are read
// once into LDS; each wave then keeps 4 regions' 16-byte-per-lane record loads in flight.  With pack_cs,
// COUNT and the value-offset SUM share one 64-bit LDS add (count << 40 | sum): 3 LDS atomics per record.
template <int REC64>
__device__ __forceinline__ void part_agg_record(const PartAggParams& p, unsigned long long r, uint32_t vmask,
                                                uint32_t* cnt, unsigned long long* cs, unsigned long long* sum,
                                                uint32_t* mn, uint32_t* mx) {
  uint32_t k, v;
  if (REC64) {
    k = (uint32_t)(r >> 32);
    v = (uint32_t)r;
  } else {
    k = (uint32_t)r >> p.part_vbits;
    v = (uint32_t)r & vmask;
  }
  if (p.pack_cs) {
    atomicAdd(&cs[k], (1ull << 40) | (unsigned long long)v);
  } else {
    atomicAdd(&cnt[k], 1u);
    if (p.has_sum) atomicAdd(&sum[k], (unsigned long long)v);
  }
  if (p.has_min) atomicMin(&mn[k], v);
  if (p.has_max) atomicMax(&mx[k], v);
}

template <int REC64>
__global__ void __launch_bounds__(1024) k_part_agg(const PartAggParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int part = blockIdx.x;
  const uint32_t KP = 1u << p.part_klo;
  const int R = p.regions;
  // LDS layout: [count u32 | count<<40|sum u64] [sum u64] [min u32] [max u32] [region fill u32 x R]
  size_t off = 0;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);
  unsigned long long* cs = reinterpret_cast<unsigned long long*>(smem);
  off += p.pack_cs ? 8 * (size_t)KP : 4 * (size_t)KP;
  unsigned long long* sum = reinterpret_cast<unsigned long long*>(smem + off);
  off += (p.has_sum && !p.pack_cs) ? 8 * (size_t)KP : 0;
  uint32_t* mn = reinterpret_cast<uint32_t*>(smem + off);
  off += p.has_min ? 4 * (size_t)KP : 0;
  uint32_t* mx = reinterpret_cast<uint32_t*>(smem + off);
  off += p.has_max ? 4 * (size_t)KP : 0;
  uint32_t* fill = reinterpret_cast<uint32_t*>(smem + off);
  for (uint32_t k = threadIdx.x; k < KP; k += blockDim.x) {
    if (p.pack_cs) cs[k] = 0; else cnt[k] = 0;
    if (p.has_sum && !p.pack_cs) sum[k] = 0;
    if (p.has_min) mn[k] = 0xffffffffu;
    if (p.has_max) mx[k] = 0u;
  }
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    const uint32_t c = p.part_count[(size_t)part * R + i];
    fill[i] = c < (uint32_t)p.part_cap ? c : (uint32_t)p.part_cap;
  }
  __syncthreads();
  const uint32_t vmask = p.part_vbits ? ((p.part_vbits >= 32) ? 0xffffffffu : ((1u << p.part_vbits) - 1u)) : 0u;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwaves = blockDim.x >> 6;
  constexpr int RPW = 4;                          // regions per wave per step
  constexpr int PER = REC64 ? 2 : 4;              // records per 16-byte lane load
  constexpr uint32_t SPAN = 64 * PER;             // records per wave-load
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  const Rec* buf = reinterpret_cast<const Rec*>(p.part_buf);
  for (int b0 = wave * RPW; b0 < R; b0 += nwaves * RPW) {
    uint32_t nn[RPW];
    uint32_t maxn = 0;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      nn[q] = (b0 + q < R) ? fill[b0 + q] : 0u;
      maxn = nn[q] > maxn ? nn[q] : maxn;
    }
    for (uint32_t base = 0; base < maxn; base += SPAN) {
      u32x4 v[RPW];
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const uint32_t i0 = base + lane * PER;
        if (i0 < nn[q]) {
          const Rec* src = buf + ((size_t)part * R + b0 + q) * (size_t)p.part_cap + i0;
          v[q] = *reinterpret_cast<const u32x4*>(src);
        }
      }
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        const uint32_t i0 = base + lane * PER;
#pragma unroll
        for (int e = 0; e < PER; ++e) {
          if (i0 + e >= nn[q]) continue;
          const unsigned long long r = REC64 ? ((unsigned long long)v[q][2 * e + 1] << 32) | v[q][2 * e]
                                             : (unsigned long long)v[q][e];
          part_agg_record<REC64>(p, r, vmask, cnt, cs, sum, mn, mx);
        }
      }
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < KP; k += blockDim.x) {
    uint32_t c;
    int64_t s = 0;
    if (p.pack_cs) {
      const unsigned long long x = cs[k];
      c = (uint32_t)(x >> 40);
      s = (int64_t)(x & ((1ull << 40) - 1ull));
    } else {
      c = cnt[k];
      if (p.has_sum) s = (int64_t)sum[k];
    }
    if (!c) continue;
    const int64_t g = ((int64_t)part << p.part_klo) | k;
    if (g >= p.num_groups) continue;
    p.out_count[g] += c;  // this block owns keys [part << klo, (part + 1) << klo)
    if (p.has_sum) p.out_sum[g] += s + (int64_t)c * p.part_vbase;
    if (p.has_min) {
      const int64_t v = p.part_vbase + (int64_t)mn[k];
      if (v < p.out_min[g]) p.out_min[g] = v;
    }
    if (p.has_max) {
      const int64_t v = p.part_vbase + (int64_t)mx[k];
      if (v > p.out_max[g]) p.out_max[g] = v;
    }
  }
}

void launch_part_agg(const PartAggParams& p, size_t lds, hipStream_t s) {
  if (p.rec64) {
    allow_lds(k_part_agg<1>, lds);
    hipLaunchKernelGGL(k_part_agg<1>, dim3(p.num_parts), dim3(1024), lds, s, p);
  } else {
    allow_lds(k_part_agg<0>, lds);
    hipLaunchKernelGGL(k_part_agg<0>, dim3(p.num_parts), dim3(1024), lds, s, p);
  }
  PH_HIP_CHECK(hipGetLastError());
}

__global__ void k_merge_overflow(const MergeParams p) {
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < p.n; g += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long c = p.ovf_count[g];
    if (!c) continue;
    p.out_count[g] += c;
    if (p.out_sum) p.out_sum[g] += p.ovf_sum[g];
    if (p.out_min && p.ovf_min[g] < p.out_min[g]) p.out_min[g] = p.ovf_min[g];
    if (p.out_max && p.ovf_max[g] > p.out_max[g]) p.out_max[g] = p.ovf_max[g];
  }
}

void launch_merge_overflow(const MergeParams& p, hipStream_t s) {
  const int grid = (int)std::min<int64_t>((p.n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_merge_overflow, dim3(grid), dim3(256), 0, s, p);
  PH_HIP_CHECK(hipGetLastError());
}

// Frame-of-reference re-encoding of an integer metric column (built once per pinned column, on first use
// by an aggregation): out holds (dictionary[dictId(doc)] - base) in vbits, in the same MSB-first big-endian
// layout the forward index uses, so the scan kernels read it with the same unpack.  Each thread assembles
// one output 32-bit word from the values overlapping it.
__global__ void k_encode_values(const uint32_t* __restrict__ fwd, int32_t bits, const int64_t* __restrict__ table,
                                int64_t base, int32_t vbits, int64_t n, uint32_t* __restrict__ out, int64_t nwords) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bit0 = w * 32;
    const int64_t first = bit0 / vbits;
    int64_t last = (bit0 + 31) / vbits;
    if (last >= n) last = n - 1;
    uint32_t x = 0;
    for (int64_t i = first; i <= last; ++i) {
      const uint32_t v = (uint32_t)(table[unpack_bits(fwd, bits, (uint32_t)i)] - base);
      const int64_t sft = i * vbits - bit0;  // in (-vbits, 32)
      x |= (uint32_t)((((uint64_t)v) << (64 - vbits)) >> (32 + sft));
    }
    out[w] = __builtin_bswap32(x);
  }
}

void launch_encode_values(const uint32_t* fwd, int32_t bits, const int64_t* table, int64_t base, int32_t vbits,
                          int64_t n, uint32_t* out, hipStream_t s) {
  const int64_t nwords = (n * vbits + 31) / 32;
  if (nwords <= 0) return;
  const int grid = (int)std::min<int64_t>((nwords + 255) / 256, 8192);
  hipLaunchKernelGGL(k_encode_values, dim3(grid), dim3(256), 0, s, fwd, bits, table, base, vbits, n, out, nwords);
  PH_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ result compaction
// Non-empty groups of the dense table, in key order: pass 1 counts per block, pass 2 scans the block
// counts, pass 3 writes keys (decoded from table-level dictionary values), counts and converted values.
__global__ void __launch_bounds__(256) k_compact_count(const CompactParams p) {
  const int64_t g0 = blockIdx.x * p.chunk, g1 = min(p.num_groups, g0 + p.chunk);
  uint32_t c = 0;
  unsigned long long d = 0;
  for (int64_t g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
    const unsigned long long n = p.count[g];
    c += n != 0;
    d += n;
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o, 64);
    d += __shfl_xor(d, o, 64);
  }
  __shared__ uint32_t ws[4];
  __shared__ unsigned long long wd[4];
  if ((threadIdx.x & 63) == 0) {
    ws[threadIdx.x >> 6] = c;
    wd[threadIdx.x >> 6] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    p.blk[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
    const unsigned long long bd = wd[0] + wd[1] + wd[2] + wd[3];
    if (bd) atomicAdd(&p.blk[kCompactBlocks + 1], bd);  // numDocsScanned without a host pass over the counts
  }
}

__global__ void __launch_bounds__(1024) k_compact_scan(const CompactParams p, int nblk) {
  __shared__ unsigned long long ws[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // exclusive scan of up to kCompactBlocks counts, 2 per thread
  unsigned long long a = (2 * t < nblk) ? p.blk[2 * t] : 0, b = (2 * t + 1 < nblk) ? p.blk[2 * t + 1] : 0;
  unsigned long long v = a + b, inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long x = __shfl_up(inc, o, 64);
    if (lane >= o) inc += x;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  if (t == 0) {
    unsigned long long acc = 0;
    for (int i = 0; i < 16; ++i) {
      const unsigned long long x = ws[i];
      ws[i] = acc;
      acc += x;
    }
    p.blk[kCompactBlocks] = acc;
  }
  __syncthreads();
  const unsigned long long ex = ws[w] + inc - v;
  if (2 * t < nblk) p.blk[2 * t] = ex;
  if (2 * t + 1 < nblk) p.blk[2 * t + 1] = ex + a;
}

__global__ void __launch_bounds__(256) k_compact_write(const CompactParams p) {
  const int64_t g0 = blockIdx.x * p.chunk, g1 = min(p.num_groups, g0 + p.chunk);
  __shared__ uint32_t ws[4];
  unsigned long long base = p.blk[blockIdx.x];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t t0 = g0; t0 < g1; t0 += blockDim.x) {
    const int64_t g = t0 + threadIdx.x;
    const unsigned long long c = g < g1 ? p.count[g] : 0ull;
    const unsigned long long bal = __ballot(c != 0);
    if (lane == 0) ws[w] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (int i = 0; i < 4; ++i) {
      before += i < w ? ws[i] : 0u;
      tot += ws[i];
    }
    if (c) {
      const unsigned long long r = base + before + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
      p.count_out[r] = (int64_t)c;
      for (int k = 0; k < kMaxAggs; ++k) {
        if (k >= p.num_aggs) continue;
        const int kind = p.agg_kind[k];
        if (kind == CK_COUNT) continue;
        const int64_t raw = p.agg_src[k][g];
        double v;
        if (kind == CK_INT) {
          v = (double)raw;
        } else if (kind == CK_REAL_SUM) {
          v = __longlong_as_double(raw);
        } else {
          v = double_from_order_key(raw);
        }
        p.agg_out[k][r] = v;
      }
      for (int j = 0; j < kMaxGroupCols; ++j) {
        if (j >= p.num_keys) continue;
        const int64_t id = ((g + p.key_base) / p.key_stride[j]) % p.key_size[j];
        switch (p.key_type[j]) {
          case PH_INT:
            reinterpret_cast<int32_t*>(p.key_out[j])[r] = (int32_t)reinterpret_cast<const int64_t*>(p.key_table[j])[id];
            break;
          case PH_LONG:
            reinterpret_cast<int64_t*>(p.key_out[j])[r] = reinterpret_cast<const int64_t*>(p.key_table[j])[id];
            break;
          case PH_FLOAT:
            reinterpret_cast<float*>(p.key_out[j])[r] = (float)reinterpret_cast<const double*>(p.key_table[j])[id];
            break;
          case PH_DOUBLE:
            reinterpret_cast<double*>(p.key_out[j])[r] = reinterpret_cast<const double*>(p.key_table[j])[id];
            break;
          default:
            reinterpret_cast<int32_t*>(p.key_out[j])[r] = (int32_t)id;
        }
      }
    }
    base += tot;
    __syncthreads();
  }
}

void launch_compact(const CompactParams& p, hipStream_t s) {
  const int nblk = (int)((p.num_groups + p.chunk - 1) / p.chunk);
  hipLaunchKernelGGL(k_compact_count, dim3(nblk), dim3(256), 0, s, p);
  hipLaunchKernelGGL(k_compact_scan, dim3(1), dim3(1024), 0, s, p, nblk);
  hipLaunchKernelGGL(k_compact_write, dim3(nblk), dim3(256), 0, s, p);
  PH_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ helpers
__global__ void k_selftest_unpack(const uint32_t* __restrict__ fwd, int64_t n, int bits, int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (int32_t)unpack_bits(fwd, bits, (uint32_t)i);
}

void launch_selftest_unpack(const uint32_t* fwd, int64_t n, int bits, int32_t* out, hipStream_t s) {
  if (n <= 0) return;
  int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_selftest_unpack, dim3(grid), dim3(256), 0, s, fwd, n, bits, out);
  PH_HIP_CHECK(hipGetLastError());
}

__global__ void k_fill_i64(int64_t* __restrict__ p, int64_t v, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

void launch_fill_i64(int64_t* p, int64_t v, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_fill_i64, dim3(grid), dim3(256), 0, s, p, v, n);
  PH_HIP_CHECK(hipGetLastError());
}

// clearspring MurmurHash.hashLong (stream 2.7.0), 32-bit wrapping arithmetic
__host__ __device__ inline int32_t murmur_long(int64_t data) {
  const uint32_t m = 0x5bd1e995u;
  uint32_t h = 0;
  uint32_t k = (uint32_t)(int32_t)data * m;
  k ^= k >> 24;
  h ^= k * m;
  k = (uint32_t)(int32_t)(data >> 32) * m;
  k ^= k >> 24;
  h *= m;
  h ^= k * m;
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}

// HyperLogLog.offerHashed: register j = h >>> (32 - log2m), rank r = nlz((h << log2m) | (1 << (log2m-1)) + 1) + 1
__host__ __device__ inline uint32_t hll_entry_of(int32_t hashed, int log2m) {
  const uint32_t h = (uint32_t)hashed;
  const uint32_t j = h >> (32 - log2m);
  const uint32_t x = (h << log2m) | ((1u << (log2m - 1)) + 1u);
  const uint32_t r = (uint32_t)__builtin_clz(x) + 1u;
  return (j << 8) | r;
}

__global__ void k_hll_table(const void* __restrict__ values, int32_t is_int, int64_t n, int log2m,
                            uint32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = is_int ? reinterpret_cast<const int64_t*>(values)[i]
                       : __double_as_longlong(reinterpret_cast<const double*>(values)[i]);  // doubleToRawLongBits
    out[i] = hll_entry_of(murmur_long(v), log2m);
  }
}

void launch_hll_table(const void* values, int32_t is_int, int64_t n, int log2m, uint32_t* out, hipStream_t s) {
  if (n <= 0) return;
  int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_hll_table, dim3(grid), dim3(256), 0, s, values, is_int, n, log2m, out);
  PH_HIP_CHECK(hipGetLastError());
}

int32_t murmur_hash_long(int64_t v) { return murmur_long(v); }
uint32_t hll_entry(int32_t hash, int log2m) { return hll_entry_of(hash, log2m); }

// Portable-roaring containers -> doc bitmap (one workgroup per container; bytes read individually because
// container payloads need not be 2-byte aligned inside the inverted-index buffer).
__device__ __forceinline__ uint32_t ld_u16(const uint8_t* b) { return (uint32_t)b[0] | ((uint32_t)b[1] << 8); }

__global__ void k_roaring_or(const RoaringContainer* __restrict__ cs, const uint8_t* __restrict__ base,
                             uint32_t* __restrict__ bitmap, int32_t num_docs) {
  const RoaringContainer c = cs[blockIdx.x];
  const uint8_t* pay = base + c.offset;
  const uint32_t hi = (uint32_t)c.key << 16;
  const uint32_t nwords = ((uint32_t)num_docs + 31u) >> 5;
  if (c.type == 0) {  // array container: card x uint16 LE
    for (int i = threadIdx.x; i < c.card; i += blockDim.x) {
      const uint32_t doc = hi | ld_u16(pay + 2 * i);
      if (doc < (uint32_t)num_docs) atomicOr(&bitmap[doc >> 5], 1u << (doc & 31u));
    }
  } else if (c.type == 1) {  // bitmap container: 1024 x uint64 LE = 2048 x uint32 LE
    for (int i = threadIdx.x; i < 2048; i += blockDim.x) {
      const uint8_t* q = pay + 4 * i;
      const uint32_t v = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
      const uint32_t wi = (hi >> 5) + i;
      if (v && wi < nwords) atomicOr(&bitmap[wi], v);
    }
  } else {  // run container: uint16 numRuns, then (start, length-1) pairs
    for (int r = threadIdx.x; r < c.card; r += blockDim.x) {
      const uint32_t start = hi | ld_u16(pay + 2 + 4 * r);
      const uint32_t end = start + ld_u16(pay + 4 + 4 * r);  // inclusive
      for (uint32_t d = start; d <= end && d < (uint32_t)num_docs;) {
        const uint32_t bit = d & 31u;
        const uint32_t take = min(32u - bit, end - d + 1u);
        const uint32_t mask = take == 32u ? 0xffffffffu : (((1u << take) - 1u) << bit);
        atomicOr(&bitmap[d >> 5], mask);
        d += take;
      }
    }
  }
}

void launch_roaring_or(const RoaringContainer* c, int n, const uint8_t* base, uint32_t* bitmap, int32_t num_docs,
                       hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_roaring_or, dim3(n), dim3(256), 0, s, c, base, bitmap, num_docs);
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph
