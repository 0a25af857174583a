// range_slices.hip -- k_range_slices: the doc bitmap of an exact bit-sliced range-index leaf, evaluated from the
// index's bit slices as BitSlicedRangeIndexReader.getMatchingDocIds does (BitSlicedRangeIndexReader.java:123-211:
// RangeBitmap.lte / gte / between / eq of the dictId range).  The index is RoaringBitmap's RangeBitmap (0.9.38, a
// dependency the reference does not vendor; its layout is restated in segment.cpp parse_range_bitmap): per 65536-doc
// key, slice i holds the docs whose value has bit i CLEAR, so `v <= c` composes low bit to high as
//   state = c_i ? (state | Z_i) : (state & Z_i),   state_0 = all docs
// (O'Neil & Quass's range evaluation over a bit-sliced index).  lo <= v <= hi is lte(hi) AND NOT lte(lo - 1).
//
// One workgroup per (eighth of a key, leaf): thread t owns the part's 32-bit word t and keeps both running states in
// registers.  The key's (container offset, kind, size) per slice are staged in LDS first (one dependent load chain
// per workgroup, not one per slice); a bitmap container's word is read with two aligned dword loads and a funnel
// shift (containers start at any byte), the words of the next kBatch bitmap slices all in flight before the batch
// composes; an array / run container's u16 payload is staged in LDS and each thread binary-searches its 32 docs.  Bytes: the leaf's containers
// once, the doc bitmap written once -- HBM-bound.  r5 on a 10M-doc, 20-slice segment (23.2 MB of containers):
// one workgroup per key 530 us; 4 parts, one slice of look-ahead 215 us; 8 parts, batched loads 128 us (its runs
// expanded serially per thread with LDS atomics); this form 24 us (~1.0 TB/s; profiles/r5_range_slices_kernel_stats.csv).
#include "ph_internal.h"

namespace ph {

namespace {
constexpr int kRbBitmap = 0, kRbRun = 1, kRbArray = 2;  // RangeBitmap container kinds
constexpr int kKeyWords = 2048;                          // 32-bit words of a 65536-doc key
constexpr int kParts = 8;                                // workgroups per key
constexpr int kPartWords = kKeyWords / kParts;           // 256: one per thread
constexpr int kBatch = 8;                                // bitmap slices whose words are loaded together
constexpr int kMaxSlices = 64;
constexpr int kStageU16 = 4096;                          // an array / run container's u16 payload (checked at pin)

__device__ inline uint32_t ld_u16(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }

// the 32-bit little-endian word at byte address p (any alignment) from two aligned dword loads; the payload buffer
// carries 16 bytes of padding, so the second load never leaves the allocation
__device__ inline uint32_t ld_u32_any(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  const uint32_t lo = w[0], hi = w[1];
  return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
}
}  // namespace

__global__ void __launch_bounds__(256) k_range_slices(const RangeSliceLeaf* __restrict__ leaves) {
  __shared__ uint16_t u16s[kStageU16];
  __shared__ int32_t s_off[kMaxSlices];
  __shared__ int32_t s_kind[kMaxSlices];
  __shared__ int32_t s_size[kMaxSlices];
  const RangeSliceLeaf L = leaves[blockIdx.y];
  const int key = blockIdx.x / kParts, part = blockIdx.x % kParts, t = threadIdx.x;
  const int64_t w0 = (int64_t)key * kKeyWords + part * kPartWords;  // this workgroup's first bitmap word
  if (w0 >= L.padded_words) return;  // uniform over the workgroup
  const uint32_t d_lo = (uint32_t)part * kPartWords * 32;  // the part's first doc in the key
  uint32_t le_hi = ~0u, le_lo = ~0u;
  const int S = key < L.nkeys ? L.nslices : 0;
  if (t < S) {
    const int32_t off = L.dir[(int64_t)key * L.nslices + t];
    s_off[t] = off;
    s_kind[t] = off >= 0 ? (int32_t)L.payload[off] : -1;
    s_size[t] = off >= 0 ? (int32_t)ld_u16(L.payload + off + 1) : 0;
  }
  __syncthreads();
  for (int i0 = 0; i0 < S; i0 += kBatch) {
    // the batch's bitmap-container words, all loads issued before any is used; kinds and offsets are wave-uniform
    // (readfirstlane), so a slice without a bitmap container is a scalar branch around its load -- it reads nothing
    // (an index of array / run containers only can be smaller than the 4 * 256 bytes a thread offset spans)
    uint32_t bw[kBatch];
    bool isbm[kBatch];
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int i = min(i0 + b, S - 1);
      isbm[b] = i0 + b < S && __builtin_amdgcn_readfirstlane(s_kind[i]) == kRbBitmap;
      bw[b] = 0;
      if (isbm[b])
        bw[b] = ld_u32_any(L.payload + __builtin_amdgcn_readfirstlane(s_off[i]) + 3 + 4 * part * kPartWords + 4 * t);
    }
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int i = i0 + b;
      if (i >= S) break;
      const int kind = __builtin_amdgcn_readfirstlane(s_kind[i]);
      uint32_t zw = bw[b];  // a bitmap container's word; none: no doc of the key has bit i clear
      if (kind == kRbArray || kind == kRbRun) {
        // the container's u16 payload (<= 4096 values / < 2048 run pairs: <= 8 KB) staged in LDS, then each thread
        // builds its own word by a binary search -- no serial per-run expansion, no atomics
        const uint8_t* p = L.payload + __builtin_amdgcn_readfirstlane(s_off[i]) + 3;
        const uint32_t size = (uint32_t)__builtin_amdgcn_readfirstlane(s_size[i]);
        const uint32_t nv = min(kind == kRbArray ? size : 2 * size, (uint32_t)kStageU16);
        __syncthreads();  // the previous such slice's searches are done with the stage
        for (uint32_t k = t; k < nv; k += 256) u16s[k] = (uint16_t)ld_u16(p + 2 * k);
        __syncthreads();
        const uint32_t a = d_lo + 32 * t;  // this thread's 32 docs [a, a + 32)
        uint32_t w = 0;
        if (kind == kRbArray) {
          uint32_t lo = 0, hi = nv;  // first value >= a
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (u16s[mid] < a) lo = mid + 1; else hi = mid;
          }
          for (uint32_t k = lo; k < nv && u16s[k] < a + 32; ++k) w |= 1u << (u16s[k] - a);
        } else {
          const uint32_t nr = nv / 2;
          uint32_t lo = 0, hi = nr;  // first run whose end (start + length) > a
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint32_t)u16s[2 * mid] + u16s[2 * mid + 1] + 1 <= a) lo = mid + 1; else hi = mid;
          }
          for (uint32_t k = lo; k < nr && u16s[2 * k] < a + 32; ++k) {
            const uint32_t rs = max((uint32_t)u16s[2 * k], a);
            const uint32_t re = min((uint32_t)u16s[2 * k] + u16s[2 * k + 1] + 1, a + 32);
            if (re > rs) w |= (re - rs == 32 ? ~0u : ((1u << (re - rs)) - 1)) << (rs - a);
          }
        }
        zw = w;
      }
      le_hi = ((L.hi >> i) & 1) ? (le_hi | zw) : (le_hi & zw);
      le_lo = ((L.lo_m1 >> i) & 1) ? (le_lo | zw) : (le_lo & zw);
    }
  }
  const int64_t gw = w0 + t;
  if (gw < L.padded_words) {
    const int64_t rem = (int64_t)L.num_docs - 32 * gw;
    const uint32_t live = rem >= 32 ? ~0u : (rem <= 0 ? 0u : ((1u << rem) - 1));
    L.bitmap[gw] = le_hi & (L.use_lo ? ~le_lo : ~0u) & live;
  }
}

void launch_range_slices(const RangeSliceLeaf* leaves, int nleaves, int max_chunks, hipStream_t s) {
  if (nleaves <= 0 || max_chunks <= 0) return;
  hipLaunchKernelGGL(k_range_slices, dim3((unsigned)(max_chunks * kParts), (unsigned)nleaves), dim3(256), 0, s,
                     leaves);
}

}  // namespace ph
