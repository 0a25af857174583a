// range_slices.hip -- k_range_slices: the doc bitmap of an exact bit-sliced range-index leaf, evaluated from the
// index's bit slices as BitSlicedRangeIndexReader.getMatchingDocIds does (BitSlicedRangeIndexReader.java:123-211:
// RangeBitmap.lte / gte / between / eq of the dictId range).  The index is RoaringBitmap's RangeBitmap (0.9.38, a
// dependency the reference does not vendor; its layout is restated in segment.cpp parse_range_bitmap): per 65536-doc
// key, slice i holds the docs whose value has bit i CLEAR, so `v <= c` composes low bit to high as
//   state = c_i ? (state | Z_i) : (state & Z_i),   state_0 = all docs
// (O'Neil & Quass's range evaluation over a bit-sliced index).  lo <= v <= hi is lte(hi) AND NOT lte(lo - 1).
//
// One workgroup per (key, leaf): thread t owns the key's 32-bit words t + 256 j (j < 8) and keeps both running states
// in registers; each slice's container is expanded to its eight words -- a bitmap container read straight from HBM,
// an array / run container scattered into an 8 KB LDS bitmap first.  Bytes: the leaf's containers once, the bitmap
// written once (HBM-bound; tiny against the queries that read it).
#include "ph_internal.h"

namespace ph {

namespace {
constexpr int kRbBitmap = 0, kRbRun = 1, kRbArray = 2;  // RangeBitmap container kinds
constexpr int kKeyWords = 2048;                          // 32-bit words of a 65536-doc key
constexpr int kPerThread = kKeyWords / 256;

__device__ inline uint32_t ld_u16(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }
__device__ inline uint32_t ld_u32(const uint8_t* p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}
}  // namespace

__global__ void __launch_bounds__(256) k_range_slices(const RangeSliceLeaf* __restrict__ leaves) {
  __shared__ uint32_t z[kKeyWords];
  const RangeSliceLeaf L = leaves[blockIdx.y];
  const int key = blockIdx.x, t = threadIdx.x;
  const int64_t w0 = (int64_t)key * kKeyWords;
  if (w0 >= L.padded_words) return;  // uniform over the workgroup
  uint32_t le_hi[kPerThread], le_lo[kPerThread];
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) le_hi[j] = le_lo[j] = ~0u;
  if (key < L.nkeys) {
    for (int i = 0; i < L.nslices; ++i) {
      const int32_t off = L.dir[(int64_t)key * L.nslices + i];
      uint32_t zw[kPerThread];
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) zw[j] = 0;  // no container: no doc of the key has bit i clear
      if (off >= 0) {
        const uint8_t* c = L.payload + off;
        const int type = c[0];
        const uint32_t size = ld_u16(c + 1);
        const uint8_t* p = c + 3;
        if (type == kRbBitmap) {
#pragma unroll
          for (int j = 0; j < kPerThread; ++j) zw[j] = ld_u32(p + 4 * (t + 256 * j));
        } else {
#pragma unroll
          for (int j = 0; j < kPerThread; ++j) z[t + 256 * j] = 0;
          __syncthreads();
          if (type == kRbArray) {
            for (uint32_t k = t; k < size; k += 256) {
              const uint32_t r = ld_u16(p + 2 * k);
              atomicOr(&z[r >> 5], 1u << (r & 31));
            }
          } else if (type == kRbRun) {
            for (uint32_t k = t; k < size; k += 256) {
              const uint32_t s = ld_u16(p + 4 * k);
              const uint32_t e = min(65536u, s + ld_u16(p + 4 * k + 2) + 1);  // [s, e)
              uint32_t d = s;
              while (d < e) {
                const uint32_t w = d >> 5, b = d & 31, n = min(32u - b, e - d);
                atomicOr(&z[w], (n == 32 ? ~0u : ((1u << n) - 1)) << b);
                d += n;
              }
            }
          }
          __syncthreads();
#pragma unroll
          for (int j = 0; j < kPerThread; ++j) zw[j] = z[t + 256 * j];
          // the next slice's zeroing touches only this thread's own words, read just above; the other threads'
          // scatters into them wait behind that slice's first barrier
        }
      }
      const bool hb = (L.hi >> i) & 1, lb = (L.lo_m1 >> i) & 1;
#pragma unroll
      for (int j = 0; j < kPerThread; ++j) {
        le_hi[j] = hb ? (le_hi[j] | zw[j]) : (le_hi[j] & zw[j]);
        le_lo[j] = lb ? (le_lo[j] | zw[j]) : (le_lo[j] & zw[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    const int64_t gw = w0 + t + 256 * j;
    if (gw >= L.padded_words) continue;
    const int64_t rem = (int64_t)L.num_docs - 32 * gw;
    const uint32_t live = rem >= 32 ? ~0u : (rem <= 0 ? 0u : ((1u << rem) - 1));
    L.bitmap[gw] = le_hi[j] & (L.use_lo ? ~le_lo[j] : ~0u) & live;
  }
}

void launch_range_slices(const RangeSliceLeaf* leaves, int nleaves, int max_chunks, hipStream_t s) {
  if (nleaves <= 0 || max_chunks <= 0) return;
  hipLaunchKernelGGL(k_range_slices, dim3((unsigned)max_chunks, (unsigned)nleaves), dim3(256), 0, s, leaves);
}

}  // namespace ph
