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
#include "ph_internal.h"

namespace ph {

__device__ __forceinline__ uint32_t unpack_bits(const uint32_t* __restrict__ fwd, int32_t bits, uint32_t doc) {
  const uint64_t bit = (uint64_t)doc * (uint32_t)bits;
  const uint32_t w = (uint32_t)(bit >> 5);
  const uint32_t sh = (uint32_t)bit & 31u;
  const uint32_t hi = __builtin_bswap32(fwd[w]);
  const uint32_t lo = __builtin_bswap32(fwd[w + 1]);
  const uint64_t x = ((uint64_t)hi << 32) | lo;
  return (uint32_t)((x << sh) >> (64 - bits));
}

__device__ __forceinline__ uint32_t unpack_col(const DevColumn& c, uint32_t doc) {
  return unpack_bits(c.fwd, c.bits, doc);
}

// Postfix filter program over a bit stack (bit 0 = top).  Control flow is wave-uniform: every lane of a
// wave runs the same instruction sequence on its own doc.
__device__ __forceinline__ bool eval_filter(const FilterInsn* __restrict__ prog, int32_t n, const DevSegment* S,
                                            uint32_t doc) {
  uint32_t st = 0;
  for (int32_t i = 0; i < n; ++i) {
    const FilterInsn in = prog[i];
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
        b = (in.ptr[v >> 5] >> (v & 31u)) & 1u;
        st = (st << 1) | b;
        break;
      }
      case OP_DOCRANGES: {
        const int32_t* r = reinterpret_cast<const int32_t*>(in.ptr);
        for (uint32_t k = 0; k < in.lo; ++k) b |= ((int32_t)doc >= r[2 * k]) & ((int32_t)doc <= r[2 * k + 1]);
        st = (st << 1) | b;
        break;
      }
      case OP_BITMAP:
        b = (in.ptr[doc >> 5] >> (doc & 31u)) & 1u;
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

__device__ __forceinline__ bool doc_matches(const KParams& p, const DevSegment* S, uint32_t doc) {
  if (S->fast_range == 1) {
    const uint32_t v = unpack_col(S->cols[S->fast_col], doc);
    return (v - S->fast_lo) < S->fast_len;
  }
  if (S->fast_range == 2) return true;  // filter simplified to match-all for this segment
  return eval_filter(p.prog + S->prog_off, S->prog_len, S, doc);
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

// value of aggregation k for the doc: int64 (integer SUM, MIN/MAX order key) or double (real SUM)
__device__ __forceinline__ void agg_value(const KParams& p, int k, const DevSegment* S, uint32_t doc, int64_t& iv,
                                          double& dv) {
  const DevColumn& c = S->cols[p.agg_slot[k]];
  const uint32_t id = unpack_col(c, doc);
  if (p.agg_is_int[k]) {
    iv = reinterpret_cast<const int64_t*>(c.values)[id];
    dv = 0.0;
  } else {
    dv = reinterpret_cast<const double*>(c.values)[id];
    iv = double_order_key(dv);
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) k_scan(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int m = 1 << p.log2m;

  // ---- LDS initialisation
  uint32_t* lds_cnt = reinterpret_cast<uint32_t*>(smem);
  uint32_t* lds_hll = reinterpret_cast<uint32_t*>(smem + p.lds_hll_off);
  if (MODE == MODE_GROUP_LDS) {
    for (int64_t g = threadIdx.x; g < p.num_groups; g += blockDim.x) lds_cnt[g] = 0;
#pragma unroll
    for (int k = 0; k < kMaxAggs; ++k) {
      if (k < p.num_aggs && p.agg_type[k] != AGG_COUNT && p.agg_type[k] != AGG_HLL) {
        int64_t init = p.agg_type[k] == AGG_MIN ? INT64_MAX : (p.agg_type[k] == AGG_MAX ? INT64_MIN : 0);
        int64_t* t = reinterpret_cast<int64_t*>(smem + p.lds_off[k]);
        for (int64_t g = threadIdx.x; g < p.num_groups; g += blockDim.x) t[g] = init;
      }
    }
    const int64_t nh = p.num_groups * p.num_hll * m;
    for (int64_t i = threadIdx.x; i < nh; i += blockDim.x) lds_hll[i] = 0;
  } else if (MODE == MODE_AGG) {
    for (int i = threadIdx.x; i < p.num_hll * m; i += blockDim.x) lds_hll[i] = 0;
  }
  __syncthreads();

  unsigned long long matched = 0;  // wave-uniform
  int64_t ai[kMaxAggs];
  double ad[kMaxAggs];
#pragma unroll
  for (int k = 0; k < kMaxAggs; ++k) {
    ai[k] = (k < p.num_aggs && p.agg_type[k] == AGG_MIN) ? INT64_MAX
            : (k < p.num_aggs && p.agg_type[k] == AGG_MAX) ? INT64_MIN
                                                            : 0;
    ad[k] = 0.0;
  }

  for (int32_t c = blockIdx.x; c < p.num_chunks; c += gridDim.x) {
    const Chunk ch = p.chunks[c];
    const DevSegment* S = p.segs + ch.seg;
    const uint32_t ndocs = (uint32_t)S->num_docs;
    for (int32_t w = ch.word_begin + wave; w < ch.word_end; w += nwaves) {
      const uint32_t doc = (uint32_t)w * 64u + (uint32_t)lane;
      bool hit = doc < ndocs;
      if (hit) hit = doc_matches(p, S, doc);
      const unsigned long long bal = __ballot(hit);
      matched += __popcll(bal);
      if (MODE == MODE_COUNT || bal == 0ull) continue;
      if (!hit) continue;
      if (MODE == MODE_AGG) {
#pragma unroll
        for (int k = 0; k < kMaxAggs; ++k) {
          if (k >= p.num_aggs) break;
          const int t = p.agg_type[k];
          if (t == AGG_COUNT) continue;
          if (t == AGG_HLL) {
            const DevColumn& col = S->cols[p.agg_slot[k]];
            const uint32_t e = col.hll[unpack_col(col, doc)];
            atomicMax(&lds_hll[p.agg_hll[k] * m + (e >> 8)], e & 0xffu);
            continue;
          }
          int64_t iv;
          double dv;
          agg_value(p, k, S, doc, iv, dv);
          if (t == AGG_SUM) {
            if (p.agg_is_int[k]) ai[k] += iv; else ad[k] += dv;
          } else if (t == AGG_MIN) {
            ai[k] = iv < ai[k] ? iv : ai[k];
          } else {
            ai[k] = iv > ai[k] ? iv : ai[k];
          }
        }
      } else {
        // group key: mixed radix over table-level global ids, column 0 least significant
        // (DictionaryBasedGroupKeyGenerator.java:283-313 over per-segment dictIds)
        int64_t key = 0;
#pragma unroll
        for (int g = 0; g < kMaxGroupCols; ++g) {
          if (g >= p.num_group_cols) break;
          const DevColumn& col = S->cols[p.group_slot[g]];
          uint32_t v = unpack_col(col, doc);
          if (col.remap) v = (uint32_t)col.remap[v];
          key += (int64_t)v * p.group_stride[g];
        }
        if (MODE == MODE_GROUP_LDS) atomicAdd(&lds_cnt[key], 1u);
        else atomicAdd(&p.out_count[key], 1ull);
#pragma unroll
        for (int k = 0; k < kMaxAggs; ++k) {
          if (k >= p.num_aggs) break;
          const int t = p.agg_type[k];
          if (t == AGG_COUNT) continue;
          if (t == AGG_HLL) {
            const DevColumn& col = S->cols[p.agg_slot[k]];
            const uint32_t e = col.hll[unpack_col(col, doc)];
            const int64_t r = (key * p.num_hll + p.agg_hll[k]) * m + (e >> 8);
            if (MODE == MODE_GROUP_LDS) atomicMax(&lds_hll[r], e & 0xffu);
            else atomicMax(&p.out_hll[r], e & 0xffu);
            continue;
          }
          int64_t iv;
          double dv;
          agg_value(p, k, S, doc, iv, dv);
          void* base = MODE == MODE_GROUP_LDS ? (void*)(smem + p.lds_off[k]) : p.out_agg[k];
          if (t == AGG_SUM) {
            if (p.agg_is_int[k])
              atomicAdd(reinterpret_cast<unsigned long long*>(base) + key, (unsigned long long)iv);
            else
              atomicAdd(reinterpret_cast<double*>(base) + key, dv);
          } else if (t == AGG_MIN) {
            atomicMin(reinterpret_cast<long long*>(base) + key, (long long)iv);
          } else {
            atomicMax(reinterpret_cast<long long*>(base) + key, (long long)iv);
          }
        }
      }
    }
  }

  // ---- block epilogue
  __shared__ unsigned long long s_matched;
  if (threadIdx.x == 0) s_matched = 0;
  __syncthreads();
  if (lane == 0 && matched) atomicAdd(&s_matched, matched);
  if (MODE == MODE_AGG) {
    __shared__ int64_t s_ai[4][kMaxAggs];
    __shared__ double s_ad[4][kMaxAggs];
#pragma unroll
    for (int k = 0; k < kMaxAggs; ++k) {
      if (k >= p.num_aggs) break;
      const int t = p.agg_type[k];
      int64_t v = ai[k];
      if (t == AGG_MIN) v = wave_min_i64(v);
      else if (t == AGG_MAX) v = wave_max_i64(v);
      else v = wave_sum_i64(v);
      const double d = wave_sum_f64(ad[k]);
      if (lane == 0 && wave < 4) {
        s_ai[wave][k] = v;
        s_ad[wave][k] = d;
      }
    }
    __syncthreads();
    if (threadIdx.x < (unsigned)p.num_aggs) {
      const int k = threadIdx.x;
      const int t = p.agg_type[k];
      if (t == AGG_SUM || t == AGG_MIN || t == AGG_MAX) {
        int64_t v = s_ai[0][k];
        double d = s_ad[0][k];
        for (int wv = 1; wv < nwaves && wv < 4; ++wv) {
          const int64_t x = s_ai[wv][k];
          if (t == AGG_MIN) v = x < v ? x : v;
          else if (t == AGG_MAX) v = x > v ? x : v;
          else v += x;
          d += s_ad[wv][k];
        }
        if (t == AGG_SUM) {
          if (p.agg_is_int[k]) atomicAdd(reinterpret_cast<unsigned long long*>(p.out_agg[k]), (unsigned long long)v);
          else atomicAdd(reinterpret_cast<double*>(p.out_agg[k]), d);
        } else if (t == AGG_MIN) {
          atomicMin(reinterpret_cast<long long*>(p.out_agg[k]), (long long)v);
        } else {
          atomicMax(reinterpret_cast<long long*>(p.out_agg[k]), (long long)v);
        }
      }
    }
    for (int i = threadIdx.x; i < p.num_hll * m; i += blockDim.x)
      if (lds_hll[i]) atomicMax(&p.out_hll[i], lds_hll[i]);
  }
  if (MODE == MODE_GROUP_LDS) {
    __syncthreads();
    for (int64_t g = threadIdx.x; g < p.num_groups; g += blockDim.x) {
      const uint32_t cnt = lds_cnt[g];
      if (!cnt) continue;
      atomicAdd(&p.out_count[g], (unsigned long long)cnt);
#pragma unroll
      for (int k = 0; k < kMaxAggs; ++k) {
        if (k >= p.num_aggs) break;
        const int t = p.agg_type[k];
        if (t == AGG_COUNT || t == AGG_HLL) continue;
        const int64_t v = reinterpret_cast<const int64_t*>(smem + p.lds_off[k])[g];
        if (t == AGG_SUM) {
          if (p.agg_is_int[k])
            atomicAdd(reinterpret_cast<unsigned long long*>(p.out_agg[k]) + g, (unsigned long long)v);
          else
            atomicAdd(reinterpret_cast<double*>(p.out_agg[k]) + g, reinterpret_cast<const double*>(smem + p.lds_off[k])[g]);
        } else if (t == AGG_MIN) {
          atomicMin(reinterpret_cast<long long*>(p.out_agg[k]) + g, (long long)v);
        } else {
          atomicMax(reinterpret_cast<long long*>(p.out_agg[k]) + g, (long long)v);
        }
      }
    }
    const int64_t nh = p.num_groups * p.num_hll * m;
    for (int64_t i = threadIdx.x; i < nh; i += blockDim.x)
      if (lds_hll[i]) atomicMax(&p.out_hll[i], lds_hll[i]);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_matched && (MODE == MODE_COUNT || MODE == MODE_AGG))
    atomicAdd(&p.out_count[0], s_matched);
}

void launch_scan(const KParams& p, int mode, int grid, int block, size_t lds, hipStream_t s) {
  switch (mode) {
    case MODE_COUNT: hipLaunchKernelGGL(k_scan<MODE_COUNT>, dim3(grid), dim3(block), lds, s, p); break;
    case MODE_AGG: hipLaunchKernelGGL(k_scan<MODE_AGG>, dim3(grid), dim3(block), lds, s, p); break;
    case MODE_GROUP_LDS: hipLaunchKernelGGL(k_scan<MODE_GROUP_LDS>, dim3(grid), dim3(block), lds, s, p); break;
    default: hipLaunchKernelGGL(k_scan<MODE_GROUP_GLOBAL>, dim3(grid), dim3(block), lds, s, p); break;
  }
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
