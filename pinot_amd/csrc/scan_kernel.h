// scan_kernel.h -- the persistent scan kernel template (k_scan) of libpinot_hip.so and its device helpers,
// included by one translation unit per plan mode (scan_*.hip) so the instantiations build in parallel.
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
#pragma once
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
// `fent` gains this doc's applyAnd filter entries: at an AND flagged with (lo = index-based children, len = scan
// children after them), the doc is fed to the first scan if every index-based child matched, and to scan i + 1 if
// it also passed scans 1..i (ScanBasedDocIdIterator.applyAnd, AndDocIdSet.java:168-170)
__device__ __forceinline__ bool eval_filter(const PH_CONST FilterInsn* prog, int32_t n, SegPtr S,
                                            uint32_t doc, uint32_t& fent) {
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
        if (in.len) {  // applyAnd statistic (kid i sits at bit col - 1 - i)
          const uint32_t ns = in.len, kids = st & m;
          const uint32_t imask = ((1u << in.lo) - 1u) << ns;  // index-based children: the top lo bits
          if ((kids & imask) == imask) {
            const uint32_t miss = ~kids & ((1u << ns) - 1u);  // failed scans; scan j at bit ns - 1 - j
            const uint32_t lead = miss ? (uint32_t)__builtin_clz(miss) - (32u - ns) : ns;  // leading passes
            fent += 1u + min(lead, ns - 1u);
          }
        }
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

// Two-deep form of the tile pipeline (k_part_scan2): the loads of a tile are issued two tiles ahead, into one of
// two register sets, so a wave keeps two tiles of HBM reads in flight.  Every tile issues exactly NL buffer loads
// with every lane active; a piece the tile does not need (beyond the segment's pieces, or past the tile's bytes)
// gets an offset outside its descriptor's range, which the hardware answers with zeros and no memory access.
// So the waitcnt pass can keep the younger set in flight: the wait before a set is consumed is vmcnt(NL), not
// vmcnt(0) (plain loads with a shared fallback address were merged by the compiler into register copies of one
// load, which forced a vmcnt(0) per tile).
template <int NL>
__device__ __forceinline__ void tile_load_fixed(bool live, SegPtr S, int32_t w0, int32_t nvalid, int lane,
                                                Prefetch<NL>& pf) {
  const int np = live ? S->npieces : 0;  // no tile: NL loads that all answer zeros (the count stays fixed)
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const bool have = k < np;
    const int32_t stride = have ? S->pieces[k].stride : 0, off = have ? S->pieces[k].off : 0;
    const uint8_t* base = have ? S->pieces[k].fwd : nullptr;
    const bool need = have && off < nvalid * stride + 8;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0,
                                                                        need ? 0x7fffffff : 0, 0x00020000);
    const uint32_t vo = need ? (uint32_t)(w0 * stride + lane * 16) : 0x80000000u;
    pf.r[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
  }
}

template <int NL>
__device__ __forceinline__ void tile_store_nowait(SegPtr S, int32_t nvalid, uint8_t* wst, int lane,
                                                  const Prefetch<NL>& pf) {
  // the waitcnt pass waits for this set's loads only (vmcnt(2 NL - 1) .. vmcnt(NL)): the other set stays in flight
  const int np = S->npieces;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int32_t stride = S->pieces[k].stride, off = S->pieces[k].off, lds = S->pieces[k].lds;
    if (k < np && off + lane * 16 < nvalid * stride + 8) {
      u32x4 v = pf.r[k];
      v.x = __builtin_bswap32(v.x);
      v.y = __builtin_bswap32(v.y);
      v.z = __builtin_bswap32(v.z);
      v.w = __builtin_bswap32(v.w);
      *reinterpret_cast<u32x4*>(wst + lds + lane * 16) = v;
    }
  }
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

// ---- lean decode cursors (the lean kernels): the same decode as BitCursor on absolute LDS addresses, one per
// stream and lane, advanced by the stream's 8*b bytes per word
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;

// LDS address (not offset from the dynamic-LDS base: that add would be paid per value)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)(p);
}

// value of the staged stream whose bits for this lane sit in the dword pair at LDS address `a` (the last bit in
// the second dword): one ds_read2 with non-negative offsets, one funnel shift, one AND
__device__ __forceinline__ uint32_t lds_value(uint32_t a, uint32_t rsh, uint32_t mask) {
  lds_cu32* w = reinterpret_cast<lds_cu32*>((uintptr_t)a);
  return __builtin_amdgcn_alignbit(w[0], w[1], rsh) & mask;
}

struct LaneStream {
  uint32_t off;   // LDS address of the dword before this lane's last-bit dword, in word 0 of the tile
  uint32_t rsh;
  uint32_t mask;
  uint32_t step;  // bytes per 64-doc word = 8 * bits
};

__device__ __forceinline__ LaneStream lane_stream(uint32_t stage_base, int32_t bits, int lane) {
  LaneStream c;
  const uint32_t e1 = (uint32_t)lane * (uint32_t)bits + (uint32_t)bits - 1u;
  c.off = stage_base + 12u + ((e1 >> 5) << 2);
  c.rsh = 31u - (e1 & 31u);
  c.mask = bits >= 32 ? 0xffffffffu : ((1u << bits) - 1u);
  c.step = 8u * (uint32_t)bits;
  return c;
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

// ------------------------------------------------------------------ partition rings (MODE_PARTITION)
// Each workgroup owns one region of every partition's buffer (region (partition, blockIdx) is written by
// exactly one workgroup: no global atomics, no cross-workgroup reservations).  A matched record's region
// position is its RANK: one returning 32-bit LDS add on the partition's word (flushed/CH << 16 | pending)
// hands out rank = flushed + pending.  Ranks [flushed, flushed + C) live in the partition's LDS ring of C
// slots (slot = rank mod C).  Every round the workgroup flushes, per partition, the whole 64-byte chunks of
// pending ranks (16 u32 / 8 u64 records, chunk-aligned in the region) with 16-byte stores and keeps the
// partial chunk in the ring, so HBM sees full, aligned 64-byte segments instead of short unaligned runs (r1:
// 32-byte runs at random alignment wrote 2.4x the record bytes).  `flushed` therefore stays a multiple of
// CH.  A record that finds its ring full (pending >= C: a skewed round) or whose rank is beyond the region
// capacity is aggregated straight into the overflow table with global atomics; a ring that overflowed is
// closed at F + C at the next flush, so region positions stay dense.

// Region (partition b, workgroup blk) of the record buffer.  A workgroup's regions are contiguous (blk-major):
// kernel A writes all P of them at once, and P regions a partition apart would each sit in its own page (r2:
// the partition-major layout missed the CU's L1 TLB on 14 % of kernel A's accesses); kernel B reads a
// partition's regions one after another.
__device__ __forceinline__ size_t part_region(const KParams& p, uint32_t b, uint32_t blk) {
  return (size_t)blk * (size_t)p.num_parts + b;
}

template <int REC64>
__device__ __forceinline__ void part_overflow(const KParams& p, uint32_t b,
                                              typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type r) {
  const uint32_t klo = REC64 ? (uint32_t)((unsigned long long)r >> 32) : (uint32_t)r >> p.part_vbits;
  const uint32_t vo = REC64 ? (uint32_t)r : ((uint32_t)r & (p.part_vbits ? ((1u << p.part_vbits) - 1u) : 0u));
  const int64_t g = ((int64_t)b << p.part_klo) | klo;
  const int64_t v = p.part_vbase + (int64_t)vo;
  atomicAdd(&p.ovf_count[g], 1ull);
  if (p.ovf_sum) atomicAdd(reinterpret_cast<unsigned long long*>(p.ovf_sum) + g, (unsigned long long)v);
  if (p.ovf_min) atomicMin(reinterpret_cast<long long*>(p.ovf_min) + g, (long long)v);
  if (p.ovf_max) atomicMax(reinterpret_cast<long long*>(p.ovf_max) + g, (long long)v);
}

template <int REC64>
__device__ __forceinline__ void part_store(const KParams& p, uint32_t b, uint32_t dst,
                                           typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type r) {
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  if (dst < (uint32_t)p.part_cap)
    reinterpret_cast<Rec*>(p.part_buf)[part_region(p, b, blockIdx.x) * (size_t)p.part_cap + dst] = r;
  else
    part_overflow<REC64>(p, b, r);  // region full (skewed keys)
}

// Flush of every partition's whole pending 64-byte chunks (final: every pending rank).  Four lanes per 64-byte
// chunk (one 16-byte LDS read and one 16-byte store each), so a store instruction writes 16 whole segments;
// the lanes of one partition are in one wave, which reads the partition's word before its first lane
// rewrites it.
template <int REC64, int BLOCK>
__device__ void part_flush(const KParams& p, uint8_t* smem, bool final) {
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  constexpr uint32_t CH = 64 / sizeof(Rec);  // records per 64-byte chunk
  constexpr uint32_t PQ = 16 / sizeof(Rec);  // records per 16-byte quarter
  const Rec* slots = reinterpret_cast<const Rec*>(smem + p.pl_slot_off);
  uint32_t* words = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  const int P = p.num_parts;
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  const uint32_t cpr = C / CH;                 // chunk slots per ring (power of two)
  const uint32_t tpp = 4 * cpr;                // threads per partition
  const int total = P * (int)tpp;
  const uint32_t cap = (uint32_t)p.part_cap;
  for (int t = threadIdx.x; t < total; t += BLOCK) {
    const uint32_t b = (uint32_t)t / tpp, ch = ((uint32_t)t % tpp) >> 2, qt = (uint32_t)t & 3u;
    const uint32_t w = words[b];
    const uint32_t F = (w >> 16) * CH, n = w & 0xffffu;
    const uint32_t inring = min(n, C);  // pending ranks >= F + C were aggregated into the overflow table
    const uint32_t out = final ? inring : (n >= C ? C : (n & ~(CH - 1u)));
    const uint32_t r = F + ch * CH + qt * PQ;  // this lane's first rank
    const uint32_t end = F + out;
    if (r < end) {
      const Rec* ring = slots + ((size_t)b << cl);
      Rec* region = reinterpret_cast<Rec*>(p.part_buf) + part_region(p, b, blockIdx.x) * (size_t)p.part_cap;
      if (r + PQ <= min(end, cap)) {
        *reinterpret_cast<u32x4*>(region + r) = *reinterpret_cast<const u32x4*>(ring + (r & (C - 1u)));
      } else {
        for (uint32_t i = r; i < min(r + PQ, end); ++i) part_store<REC64>(p, b, i, ring[i & (C - 1u)]);
      }
    }
    if (((uint32_t)t % tpp) == 0) {
      if (final) p.part_count[(size_t)b * gridDim.x + blockIdx.x] = end;  // records of region (b, blockIdx)
      else if (out) words[b] = ((end / CH) << 16) | (n >= C ? 0u : n - out);
    }
  }
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
// 2-operand expression terms run on the kMaxVals variant, or on REC64 = 2: the one-column variant with the
// expression's second cursor (~15 VGPRs more than REC64 = 1; SSB Q1.x / Q4.x: one SUM(a*b) / SUM(a-b) column).
template <int MODE, int REC64>
struct ValCap {
  // MODE_PARTITION is only planned for <= 1 value column (query.cpp part_ok)
  static constexpr int value = (MODE == MODE_PARTITION || REC64) ? 1 : kMaxVals;
};

// Per-wave accumulation state of the scan (registers).
struct ScanAcc {
  unsigned long long matched;  // wave-uniform
  uint32_t fent;               // per lane: applyAnd filter entries (eval_filter)
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
  // conjunctive scan leaves (FK_CONJ)
  BitCursor ccur[FK == FK_CONJ ? kMaxConj : 1];
  uint32_t clo[FK == FK_CONJ ? kMaxConj : 1], clen[FK == FK_CONJ ? kMaxConj : 1];
  const uint32_t* cset[FK == FK_CONJ ? kMaxConj : 1];
  const int nconj = FK == FK_CONJ ? S->nconj : 0;
  const int cnidx = FK == FK_CONJ ? S->conj_nidx : 0;
  if constexpr (FK == FK_CONJ) {
#pragma unroll
    for (int k = 0; k < kMaxConj; ++k) {
      if (k >= nconj) continue;
      const int cs = S->cstream[k];
      ccur[k] = bit_cursor(wst + p.stage_soff[cs], S->streams[cs].bits, lane);
      clo[k] = S->clo[k];
      clen[k] = S->clen[k];
      cset[k] = S->cset[k];
    }
  }
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
  // second operand of a 2-operand expression term (MODE_PARTITION never plans one)
  int vkind2[kMaxVals];
  int64_t vbase2[kMaxVals];
  const void* vtab2[kMaxVals];
  BitCursor vcur2[kMaxVals];
#pragma unroll
  for (int j = 0; j < VC; ++j) {
    if (MODE == MODE_COUNT || j >= p.num_vals || (MODE == MODE_PARTITION && j > 0)) continue;
    vcur[j] = bit_cursor(wst + p.stage_soff[p.v_stream[j]], S->streams[p.v_stream[j]].bits, lane);
    vkind[j] = S->vals[j].kind;
    vbase[j] = S->vals[j].base;
    vtab[j] = S->vals[j].table;
    if (MODE != MODE_PARTITION && (VC > 1 || REC64 == 2) && p.val_op[j]) {  // expressions: kMaxVals or REC64 2
      vcur2[j] = bit_cursor(wst + p.stage_soff[p.v2_stream[j]], S->streams[p.v2_stream[j]].bits, lane);
      vkind2[j] = S->vals2[j].kind;
      vbase2[j] = S->vals2[j].base;
      vtab2[j] = S->vals2[j].table;
    }
  }
  uint32_t* lds_cnt = reinterpret_cast<uint32_t*>(smem + p.lds_cnt_off);
  uint32_t* lds_hll = reinterpret_cast<uint32_t*>(smem + p.lds_hll_off);

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
      if (hit) hit = eval_filter((const PH_CONST FilterInsn*)p.prog + S->prog_off, S->prog_len, S, doc, acc.fent);
    } else if constexpr (FK == FK_CONJ) {
      uint32_t pb = 0;  // leaf k passed -> bit k
#pragma unroll
      for (int k = 0; k < kMaxConj; ++k) {
        if (k >= nconj) continue;
        const uint32_t v = cursor_value(ccur[k], u);
        bool pk;
        if (LATE && cset[k]) pk = (bool)((gld(cset[k] + (v >> 5)) >> (v & 31u)) & 1u);
        else pk = (v - clo[k]) < clen[k];
        hit &= pk;
        pb |= (uint32_t)pk << k;
      }
      if (cnidx && doc < ndocs) {  // applyAnd statistic (see eval_filter): leading range-index leaves, then scans
        const uint32_t im = (1u << cnidx) - 1u, ns = (uint32_t)(nconj - cnidx);
        if ((pb & im) == im) {
          const uint32_t lead = (uint32_t)__builtin_ctz(~(pb >> cnidx));
          acc.fent += 1u + min(lead, ns - 1u);
        }
      }
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
          const int eop = (MODE != MODE_PARTITION && (VC > 1 || REC64 == 2)) ? p.val_op[j] : 0;
          if (eop) {
            // `a <op> b` per row: exact int64 for integer terms, else double like the reference's
            // transformToDoubleValuesSV (MultiplicationTransformFunction.java:89-104)
            int64_t ib;
            double db = 0.0;
            if (LATE) read_value(vkind2[j], vbase2[j], vtab2[j], cursor_value(vcur2[j], u), ib, db);
            else ib = vbase2[j] + (int64_t)cursor_value(vcur2[j], u);
            if (p.val_is_int[j]) {
              vi[j] = eop == PH_EXPR_MULT ? vi[j] * ib : (eop == PH_EXPR_SUB ? vi[j] - ib : vi[j] + ib);
            } else {
              const double x = (LATE && vkind[j] == VK_DICT_F64) ? vd[j] : (double)vi[j];
              const double y = (LATE && vkind2[j] == VK_DICT_F64) ? db : (double)ib;
              vd[j] = eop == PH_EXPR_MULT ? (1.0 * x) * y : (eop == PH_EXPR_SUB ? x - y : x + y);
              vi[j] = double_order_key(vd[j]);
            }
          }
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
      int64_t g = key;
      if constexpr (MODE == MODE_GROUP_HASH) {
        // LongMapBasedHolder / ArrayMapBasedHolder regime (DictionaryBasedGroupKeyGenerator.java:598,778):
        // linear probing on the raw mixed-radix key; the table has >= 2x the slots of the keys it can receive,
        // so the probe always ends (bounded anyway)
        unsigned long long h = (unsigned long long)key;
        h ^= h >> 33;
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
        h *= 0xc4ceb9fe1a85ec53ull;
        h ^= h >> 33;
        int64_t slot = (int64_t)(h & (unsigned long long)p.hmask);
        for (int64_t probe = 0; probe <= p.hmask; ++probe) {
          // plain read first: a key already placed costs no atomic (the common case once the table warms up)
          unsigned long long old = __hip_atomic_load(&p.hkeys[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (old == (unsigned long long)key) break;
          if (old == kHashEmpty) {
            old = atomicCAS(&p.hkeys[slot], kHashEmpty, (unsigned long long)key);
            if (old == kHashEmpty || old == (unsigned long long)key) break;
          }
          slot = (slot + 1) & p.hmask;
        }
        g = slot;
      }
      if (MODE == MODE_GROUP_GLOBAL && LATE && p.first_doc) {  // numGroupsLimit pass: first doc of every key
        atomicMin(&S->first_doc[g], doc);
        return;
      }
      if (MODE == MODE_GROUP_HASH && LATE && p.first_doc) {  // the same over one segment's first-seen hash table
        atomicMin(&p.first_doc[g], doc);
        return;
      }
      if (MODE != MODE_GROUP_HASH && LATE && S->keep && !((gld(S->keep + (g >> 5)) >> (g & 31)) & 1u))
        return;  // beyond numGroupsLimit
      if (MODE == MODE_GROUP_HASH && LATE && S->keep) {
        // beyond numGroupsLimit?  the key's slot in the segment's first-seen table (the pass placed every key this
        // scan meets) indexes the keep bitset
        unsigned long long h = (unsigned long long)key;
        h ^= h >> 33;
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
        h *= 0xc4ceb9fe1a85ec53ull;
        h ^= h >> 33;
        int64_t ls = (int64_t)(h & (unsigned long long)p.lmask);
        for (int64_t probe = 0; probe <= p.lmask; ++probe) {
          const unsigned long long k = gld(p.lkeys + ls);
          if (k == (unsigned long long)key || k == kHashEmpty) break;
          ls = (ls + 1) & p.lmask;
        }
        if (!((gld(S->keep + (ls >> 5)) >> (ls & 31)) & 1u)) return;
      }
      // MODE_GROUP_GLOBAL: the workgroup's LDS group cache first (slot found -> aggregate in LDS like MODE_GROUP_LDS)
      bool local = MODE == MODE_GROUP_LDS;
      if (MODE == MODE_GROUP_GLOBAL && p.gc_slots) {
        uint32_t* gkeys = reinterpret_cast<uint32_t*>(smem + p.gc_key_off);
        const uint32_t k32 = (uint32_t)g;
        const uint32_t smask = (uint32_t)p.gc_slots - 1u;
        uint32_t h = (k32 * 2654435761u) & smask;
#pragma unroll 1
        for (int probe = 0; probe < 8; ++probe) {
          uint32_t k = gkeys[h];
          if (k == 0xffffffffu) k = atomicCAS(&gkeys[h], 0xffffffffu, k32);
          if (k == 0xffffffffu || k == k32) {
            local = true;
            g = h;
            break;
          }
          h = (h + 1u) & smask;
        }
      }
      if (local) atomicAdd(&lds_cnt[g], 1u);
      else if (MODE == MODE_GROUP_GLOBAL || MODE == MODE_GROUP_HASH) atomicAdd(&p.out_count[g], 1ull);
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
          void* sb = local ? (void*)(smem + p.lds_sum_off[j]) : p.out_sum[j];
          long long* mnb = local ? reinterpret_cast<long long*>(smem + p.lds_min_off[j])
                                 : reinterpret_cast<long long*>(p.out_min[j]);
          long long* mxb = local ? reinterpret_cast<long long*>(smem + p.lds_max_off[j])
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
        if (MODE == MODE_GROUP_GLOBAL || MODE == MODE_GROUP_HASH) atomicMax(&p.out_hll[ri], e & 0xffu);  // g: slot
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
    uint32_t* words = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
    constexpr uint32_t CH = 64 / sizeof(Rec);
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
      if (tot == 0) continue;
      uint32_t bk[UB], rk[UB], rf[UB];
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
        uint32_t vo = 0;
        if (p.num_vals) {
          int64_t iv;
          double dv;
          if (LATE) read_value(vkind[0], vbase[0], vtab[0], cursor_value(vcur[0], u + q), iv, dv);
          else iv = vbase[0] + (int64_t)cursor_value(vcur[0], u + q);  // VK_PACKED: no gather
          vo = (uint32_t)(iv - p.part_vbase);
        }
        bk[q] = key >> p.part_klo;
        rec[q] = REC64 ? (Rec)(((unsigned long long)(key & kmask) << 32) | vo) : (Rec)(((key & kmask) << p.part_vbits) | vo);
        if (hit[q]) {
          const uint32_t w = atomicAdd(&words[bk[q]], 1u);
          rf[q] = (w >> 16) * CH;  // flushed ranks
          rk[q] = w & 0xffffu;     // pending before this record
        }
      }
#pragma unroll
      for (int q = 0; q < UB; ++q) {
        if (!hit[q]) continue;
        if (rk[q] < C) slots[(bk[q] << cl) + ((rf[q] + rk[q]) & (C - 1u))] = rec[q];
        else part_overflow<REC64>(p, bk[q], rec[q]);  // ring full (skewed round): overflow table
      }
    }
    return;
  }
  // ph_filter_execute: the ballots ARE the segment's doc bitmap words (FilterPlanNode's BitmapDocIdSet); lane q of the
  // wave stores word u + q of a step, one 8-byte store per word
  unsigned long long* const dset = MODE == MODE_COUNT ? reinterpret_cast<unsigned long long*>(S->docset) : nullptr;
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
    if constexpr (MODE == MODE_COUNT) {
      if (dset) {
        unsigned long long mine = bal[0];
#pragma unroll
        for (int q = 1; q < UB; ++q) mine = lane == q ? bal[q] : mine;
        if (lane < UB) dset[w0 + u + lane] = mine;
      }
    } else {
#pragma unroll
      for (int q = 0; q < UB; ++q)
        if (bal[q]) aggregate_word(u + q, hit[q], bal[q]);
    }
  }
  for (; u < nvalid; ++u) {
    const bool hit = filter_word(u);
    const unsigned long long bal = __ballot(hit);
    acc.matched += __popcll(bal);
    if constexpr (MODE == MODE_COUNT) {
      if (dset && lane == 0) dset[w0 + u] = bal;
    } else {
      if (bal) aggregate_word(u, hit, bal);
    }
  }
}

// Persistent grid over the chunk list.  A chunk (<= 256 words of one segment) is processed in rounds: in
// round r wave w takes tile r * kWaves + w.  Rounds are workgroup-uniform (MODE_PARTITION flushes at round
// boundaries with workgroup barriers); the other modes never synchronise inside the loop.
template <int MODE, int NG, int REC64, int LATE>
__global__ void __launch_bounds__(MODE == MODE_PARTITION ? kPartBlock : kBlock) k_scan(const KParams p) {
  constexpr int BLOCK = MODE == MODE_PARTITION ? kPartBlock : kBlock;
  constexpr int WAVES = BLOCK / 64;
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
  } else if (MODE == MODE_GROUP_GLOBAL) {
    if (p.gc_slots) {  // LDS group cache: empty keys, zero counts / sums, min / max identities
      uint32_t* gkeys = reinterpret_cast<uint32_t*>(smem + p.gc_key_off);
      for (int i = threadIdx.x; i < p.gc_slots; i += kBlock) {
        gkeys[i] = 0xffffffffu;
        lds_cnt[i] = 0;
#pragma unroll
        for (int j = 0; j < VC; ++j) {
          if (j >= p.num_vals) continue;
          const int ops = p.val_ops[j];
          if (ops & OPS_SUM) reinterpret_cast<int64_t*>(smem + p.lds_sum_off[j])[i] = 0;
          if (ops & OPS_MIN) reinterpret_cast<int64_t*>(smem + p.lds_min_off[j])[i] = INT64_MAX;
          if (ops & OPS_MAX) reinterpret_cast<int64_t*>(smem + p.lds_max_off[j])[i] = INT64_MIN;
        }
      }
    }
  } else if (MODE == MODE_PARTITION) {
    uint32_t* words = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
    for (int i = threadIdx.x; i < p.num_parts; i += BLOCK) words[i] = 0;
  }
  __syncthreads();

  ScanAcc acc;
  acc.matched = 0;
  acc.fent = 0;
#pragma unroll
  for (int j = 0; j < VC; ++j) {
    acc.isum[j] = 0;
    acc.dsum[j] = 0.0;
    acc.vmin[j] = INT64_MAX;
    acc.vmax[j] = INT64_MIN;
  }

  // ---- round iterator: (chunk c, round r); the tile of this wave starts at word w0 and has nvalid words
  const int32_t tw = p.tile_words;
  const int32_t round_words = WAVES * tw;
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

  while (c < c_end) {
    // stage the prefetched tile, then prefetch the next one of this wave
    tile_store<NL>(S, nvalid, wst, lane, pf);
    if (MODE == MODE_PARTITION) {
      // flush the chunks completed in the previous round here, before this round's prefetch: the stores
      // then complete under the decode instead of stalling the next tile_store (stores count in vmcnt too)
      part_flush<REC64, BLOCK>(p, smem, false);
      lds_barrier();  // ring words are final before anyone appends again
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

    if (cnvalid > 0) {
      switch (cs->fkind) {
        case FK_ALL: process_tile<MODE, NG, REC64, FK_ALL, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_RANGE: process_tile<MODE, NG, REC64, FK_RANGE, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_SET: process_tile<MODE, NG, REC64, FK_SET, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_BITMAP: process_tile<MODE, NG, REC64, FK_BITMAP, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        case FK_DOCRANGE:
          process_tile<MODE, NG, REC64, FK_DOCRANGE, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc);
          break;
        case FK_CONJ: process_tile<MODE, NG, REC64, FK_CONJ, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
        default: process_tile<MODE, NG, REC64, FK_GENERIC, LATE>(p, cs, smem, wst, lane, cw0, cnvalid, acc); break;
      }
    }
    if (LATE && c < c_end) tile_load<NL>(S, w0, nvalid, lane, pf);
    if (MODE == MODE_PARTITION) lds_barrier();  // this round's appends are complete before the next round's flush check
  }

  // ---- workgroup epilogue
  if (MODE == MODE_PARTITION) {
    if (lane == 0 && acc.matched && p.matched_total) atomicAdd(p.matched_total, acc.matched);
    lds_barrier();
    part_flush<REC64, BLOCK>(p, smem, true);  // also writes the region record counts
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
  if (MODE == MODE_GROUP_GLOBAL && p.gc_slots) {  // the workgroup's cached groups -> the HBM table, once each
    __syncthreads();
    const uint32_t* gkeys = reinterpret_cast<const uint32_t*>(smem + p.gc_key_off);
    for (int i = threadIdx.x; i < p.gc_slots; i += kBlock) {
      const uint32_t key = gkeys[i];
      const uint32_t cnt = lds_cnt[i];
      if (key == 0xffffffffu || !cnt) continue;
      atomicAdd(&p.out_count[key], (unsigned long long)cnt);
#pragma unroll
      for (int j = 0; j < VC; ++j) {
        if (j >= p.num_vals) continue;
        const int ops = p.val_ops[j];
        if (ops & OPS_SUM) {
          if (p.val_is_int[j])
            atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum[j]) + key,
                      reinterpret_cast<const unsigned long long*>(smem + p.lds_sum_off[j])[i]);
          else
            atomicAdd(reinterpret_cast<double*>(p.out_sum[j]) + key, reinterpret_cast<const double*>(smem + p.lds_sum_off[j])[i]);
        }
        if (ops & OPS_MIN)
          atomicMin(reinterpret_cast<long long*>(p.out_min[j]) + key, reinterpret_cast<const long long*>(smem + p.lds_min_off[j])[i]);
        if (ops & OPS_MAX)
          atomicMax(reinterpret_cast<long long*>(p.out_max[j]) + key, reinterpret_cast<const long long*>(smem + p.lds_max_off[j])[i]);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_matched && (MODE == MODE_COUNT || MODE == MODE_AGG))
    atomicAdd(&p.out_count[0], s_matched);
  if (threadIdx.x == 0 && s_matched && p.matched_total) atomicAdd(p.matched_total, s_matched);
  if (p.filter_entries) {  // the wave's applyAnd filter entries
    const int64_t fe = wave_sum_i64((int64_t)acc.fent);
    if ((threadIdx.x & 63) == 0 && fe) atomicAdd(p.filter_entries, (unsigned long long)fe);
  }
}

// kernels that use more than the default 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU); the attribute is set once
// per (kernel, device) and raised when a launch needs more (the call costs host time on every launch otherwise)
void allow_lds_raw(const void* kernel, size_t lds);
template <class K>
inline void allow_lds(K kernel, size_t lds) {
  if (lds > 64 * 1024) allow_lds_raw(reinterpret_cast<const void*>(kernel), lds);
}

template <int MODE, int NG, int REC64>
inline void launch_late(const KParams& p, int grid, size_t lds, hipStream_t s) {
  if (p.late_prefetch) {
    allow_lds(k_scan<MODE, NG, REC64, 1>, lds);
    hipLaunchKernelGGL((k_scan<MODE, NG, REC64, 1>), dim3(grid), dim3(MODE == MODE_PARTITION ? kPartBlock : kBlock), lds, s, p);
  } else {
    allow_lds(k_scan<MODE, NG, REC64, 0>, lds);
    hipLaunchKernelGGL((k_scan<MODE, NG, REC64, 0>), dim3(grid), dim3(MODE == MODE_PARTITION ? kPartBlock : kBlock), lds, s, p);
  }
}

template <int MODE, int NG>
inline void launch_ng(const KParams& p, int rec64, int grid, size_t lds, hipStream_t s) {
  if constexpr (MODE != MODE_PARTITION) {
    if (rec64 == 2) {
      launch_late<MODE, NG, 2>(p, grid, lds, s);
      return;
    }
  }
  if (rec64) launch_late<MODE, NG, 1>(p, grid, lds, s);
  else launch_late<MODE, NG, 0>(p, grid, lds, s);
}

// the value-column variant of a non-partition launch: 1 = one plain column, 2 = one 2-operand expression, 0 = any
inline int value_variant(const KParams& p) { return p.num_vals <= 1 ? (p.val_op[0] ? 2 : 1) : 0; }

template <int MODE>
inline void launch_mode(const KParams& p, int ng, int rec64, int grid, size_t lds, hipStream_t s) {
  switch (ng) {
    case 1: launch_ng<MODE, 1>(p, rec64, grid, lds, s); break;
    case 2: launch_ng<MODE, 2>(p, rec64, grid, lds, s); break;
    case 3: launch_ng<MODE, 3>(p, rec64, grid, lds, s); break;
    default: launch_ng<MODE, 4>(p, rec64, grid, lds, s); break;
  }
}

}  // namespace ph
