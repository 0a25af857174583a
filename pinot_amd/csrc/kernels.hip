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

__device__ __forceinline__ uint32_t unpack_bits(const uint32_t* __restrict__ fwd, int32_t bits, uint32_t doc) {
  const uint64_t bit = (uint64_t)doc * (uint32_t)bits;
  const uint32_t w = (uint32_t)(bit >> 5);
  const uint32_t sh = (uint32_t)bit & 31u;
  const uint32_t hi = __builtin_bswap32(gld(fwd + w));
  const uint32_t lo = __builtin_bswap32(gld(fwd + w + 1));
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
    const PH_GLOBAL FilterInsn* gi = (const PH_GLOBAL FilterInsn*)(prog + i);
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
        for (uint32_t k = 0; k < in.lo; ++k) b |= ((int32_t)doc >= gld(r + 2 * k)) & ((int32_t)doc <= gld(r + 2 * k + 1));
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

constexpr int U = 4;  // 64-doc words per wave per iteration (memory-level parallelism)

// compile-time loop: the body sees `u` as a constant expression, so per-word register arrays never spill
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Stage the first p.nstage streams of this wave's U words into its private LDS area: one coalesced
// 16-byte-per-lane load per stream (a 64-doc word of a b-bit stream is exactly 8*b bytes, so the span
// of U words starts 8-byte aligned), all loads issued before any LDS write.
__device__ __forceinline__ void stage_streams(const KParams& p, const DevSegment* S, int32_t w0, int32_t nvalid,
                                              uint32_t* wst, int lane) {
  u32x4 raw[kMaxStage];
  int nb[kMaxStage];
#pragma unroll
  for (int s = 0; s < kMaxStage; ++s) {
    nb[s] = 0;
    if (s >= p.nstage) continue;
    const int bits = S->streams[s].bits;
    if (bits == 0) continue;  // nothing to stage for this segment
    nb[s] = nvalid * 8 * bits + 8;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(S->streams[s].fwd) + (size_t)w0 * 8 * bits;
    if (lane * 16 < nb[s]) raw[s] = gld(reinterpret_cast<const u32x4a8*>(src + lane * 16));
  }
#pragma unroll
  for (int s = 0; s < kMaxStage; ++s)
    if (lane * 16 < nb[s]) *reinterpret_cast<u32x4*>(wst + s * (kStageBytes / 4) + lane * 4) = raw[s];
}

__device__ __forceinline__ uint32_t staged_bits(const uint32_t* stg, int32_t bits, uint32_t local) {
  const uint32_t bit = local * (uint32_t)bits;
  const uint32_t d = bit >> 5, sh = bit & 31u;
  const uint64_t x = ((uint64_t)__builtin_bswap32(stg[d]) << 32) | __builtin_bswap32(stg[d + 1]);
  return (uint32_t)((x << sh) >> (64 - bits));
}

// value of stream s for word u of this wave (LDS-staged or straight from HBM)
__device__ __forceinline__ uint32_t stream_bits(const KParams& p, const DevSegment* S, const uint32_t* wst, int s,
                                                int u, int lane, uint32_t doc) {
  const int32_t bits = S->streams[s].bits;
  if (s < p.nstage) return staged_bits(wst + s * (kStageBytes / 4), bits, (uint32_t)(u * 64 + lane));
  return unpack_bits(S->streams[s].fwd, bits, doc);
}

// Applies the segment's filter to U words of one wave (control flow uniform per segment).
__device__ __forceinline__ void filter_words(const KParams& p, const DevSegment* S, const uint32_t* wst, int lane,
                                             const uint32_t (&doc)[U], bool (&hit)[U]) {
  switch (S->fkind) {
    case FK_ALL:
      break;
    case FK_RANGE: {
      const uint32_t lo = S->flo, len = S->flen;
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = hit[u] ? stream_bits(p, S, wst, p.f_stream, u, lane, doc[u]) : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) hit[u] = hit[u] && (v[u] - lo) < len;
      break;
    }
    case FK_SET: {
      const uint32_t* bs = S->fptr;
      uint32_t v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = hit[u] ? stream_bits(p, S, wst, p.f_stream, u, lane, doc[u]) : 0u;
#pragma unroll
      for (int u = 0; u < U; ++u) hit[u] = hit[u] && ((gld(bs + (v[u] >> 5)) >> (v[u] & 31u)) & 1u);
      break;
    }
    case FK_BITMAP: {
      const uint32_t* bm = S->fptr;
#pragma unroll
      for (int u = 0; u < U; ++u) hit[u] = hit[u] && ((gld(bm + (doc[u] >> 5)) >> (doc[u] & 31u)) & 1u);
      break;
    }
    case FK_DOCRANGE: {
#pragma unroll
      for (int u = 0; u < U; ++u) hit[u] = hit[u] && (doc[u] - S->flo) < S->flen;
      break;
    }
    default: {
#pragma unroll
      for (int u = 0; u < U; ++u) hit[u] = hit[u] && eval_filter(p.prog + S->prog_off, S->prog_len, S, doc[u]);
    }
  }
}

// value of value-column j for a doc: int64 (integer columns) or float64 (real columns)
__device__ __forceinline__ void read_value(const DevValCol& c, uint32_t x, int64_t& iv, double& dv) {
  if (c.kind == VK_PACKED) {
    iv = c.base + (int64_t)x;
    dv = 0.0;
  } else if (c.kind == VK_DICT_I64) {
    iv = gld(reinterpret_cast<const int64_t*>(c.table) + x);
    dv = 0.0;
  } else {
    dv = gld(reinterpret_cast<const double*>(c.table) + x);
    iv = double_order_key(dv);
  }
}

template <class T>
__device__ __forceinline__ T pick(const T (&a)[kMaxVals], int j) {
  T x = a[0];
#pragma unroll
  for (int i = 1; i < kMaxVals; ++i)
    if (j == i) x = a[i];
  return x;
}

template <int NG>
__device__ __forceinline__ int64_t group_key(const KParams& p, const DevSegment* S, const uint32_t* wst, int u,
                                             int lane, uint32_t doc) {
  int64_t key = 0;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    const int32_t* remap = S->cols[p.group_slot[g]].remap;
    uint32_t v = stream_bits(p, S, wst, p.g_stream[g], u, lane, doc);
    if (remap) v = (uint32_t)gld(remap + v);
    key += (int64_t)v * p.group_stride[g];
  }
  return key;
}

// ------------------------------------------------------------------ partition staging (MODE_PARTITION)
constexpr int kMaxParts = 1024;

template <int REC64>
struct PartLds {  // with the 8-wave staging area: <= 160 KiB, one 512-thread block per CU
  static constexpr int kStage = REC64 ? 5120 : 8192;  // staged records per flush
  uint32_t st_key[kStage];
  uint32_t st_val[kStage];
  typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type sorted[kStage];
  uint16_t sbucket[kStage];
  uint32_t cnt[kMaxParts];
  uint32_t off[kMaxParts];
  uint32_t gpos[kMaxParts];
  uint32_t wsum[32];
  uint32_t stage_n;
};
constexpr size_t part_stage_off(int rec64) {
  return ((rec64 ? sizeof(PartLds<1>) : sizeof(PartLds<0>)) + 15) / 16 * 16;
}
static_assert(part_stage_off(0) + (kPartBlock / 64) * kMaxStage * kStageBytes <= 160 * 1024, "partition LDS");
static_assert(part_stage_off(1) + (kPartBlock / 64) * kMaxStage * kStageBytes <= 160 * 1024, "partition LDS");

template <int REC64>
__device__ void part_flush(const KParams& p, PartLds<REC64>& L, int shard) {
  __syncthreads();
  const int tid = threadIdx.x;
  const uint32_t n = L.stage_n;
  const int P = p.num_parts;
  for (int i = tid; i < P; i += blockDim.x) L.cnt[i] = 0;
  __syncthreads();
  constexpr int K = PartLds<REC64>::kStage / kPartBlock;
  uint32_t rk[K], pb[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t i = tid + k * kPartBlock;
    if (i < n) {
      pb[k] = L.st_key[i] >> p.part_klo;
      rk[k] = atomicAdd(&L.cnt[pb[k]], 1u);
    }
  }
  __syncthreads();
  // exclusive scan of the bucket counts (P <= blockDim.x) + one reservation per non-empty bucket
  {
    const int lane = tid & 63, w = tid >> 6;
    const uint32_t v = tid < P ? L.cnt[tid] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) L.wsum[w] = inc;
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
        const uint32_t t = L.wsum[i];
        L.wsum[i] = acc;
        acc += t;
      }
    }
    __syncthreads();
    if (tid < P) {
      L.off[tid] = L.wsum[w] + inc - v;
      L.gpos[tid] = v ? atomicAdd(&p.part_cursor[shard * P + tid], v) : 0u;
    }
  }
  __syncthreads();
  const uint32_t kmask = (1u << p.part_klo) - 1u;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t i = tid + k * kPartBlock;
    if (i < n) {
      const uint32_t pos = L.off[pb[k]] + rk[k];
      const uint32_t klo = L.st_key[i] & kmask;
      if (REC64) L.sorted[pos] = (((unsigned long long)klo << 32) | L.st_val[i]);
      else L.sorted[pos] = (klo << p.part_vbits) | L.st_val[i];
      L.sbucket[pos] = (uint16_t)pb[k];
    }
  }
  __syncthreads();
  for (uint32_t j = tid; j < n; j += blockDim.x) {
    const uint32_t b = L.sbucket[j];
    const uint32_t dst = L.gpos[b] + (j - L.off[b]);
    const unsigned long long rec = (unsigned long long)L.sorted[j];
    const size_t slot = ((size_t)shard * P + b) * (size_t)p.part_cap + dst;
    if (dst < (uint32_t)p.part_cap) {
      if (REC64) reinterpret_cast<unsigned long long*>(p.part_buf)[slot] = rec;
      else reinterpret_cast<uint32_t*>(p.part_buf)[slot] = (uint32_t)rec;
    } else {
      // partition overflow (skewed keys): aggregate directly into the overflow table
      const uint32_t klo = REC64 ? (uint32_t)(rec >> 32) : (uint32_t)rec >> p.part_vbits;
      const uint32_t vo = REC64 ? (uint32_t)rec : ((uint32_t)rec & ((p.part_vbits ? (1u << p.part_vbits) : 1u) - 1u));
      const int64_t g = ((int64_t)b << p.part_klo) | klo;
      const int64_t v = p.part_vbase + (int64_t)vo;
      atomicAdd(&p.ovf_count[g], 1ull);
      if (p.ovf_sum) atomicAdd(reinterpret_cast<unsigned long long*>(p.ovf_sum) + g, (unsigned long long)v);
      if (p.ovf_min) atomicMin(reinterpret_cast<long long*>(p.ovf_min) + g, (long long)v);
      if (p.ovf_max) atomicMax(reinterpret_cast<long long*>(p.ovf_max) + g, (long long)v);
    }
  }
  __syncthreads();
  if (tid == 0) L.stage_n = 0;
  __syncthreads();
}


// ------------------------------------------------------------------ the scan kernel
enum : int32_t { OPS_SUM = 1, OPS_MIN = 2, OPS_MAX = 4 };

template <int MODE, int NG, int REC64>
__global__ void __launch_bounds__(MODE == MODE_PARTITION ? kPartBlock : 256) k_scan(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int nwaves = blockDim.x >> 6;
  const int m = 1 << p.log2m;

  uint32_t* lds_cnt = reinterpret_cast<uint32_t*>(smem + p.lds_cnt_off);
  uint32_t* lds_hll = reinterpret_cast<uint32_t*>(smem + p.lds_hll_off);
  PartLds<REC64>& PL = *reinterpret_cast<PartLds<REC64>*>(smem);
  uint32_t* wst = reinterpret_cast<uint32_t*>(smem + p.stage_off + (size_t)wave * kMaxStage * kStageBytes);
  if (MODE == MODE_GROUP_LDS) {
    for (int64_t g = threadIdx.x; g < p.num_groups; g += blockDim.x) lds_cnt[g] = 0;
#pragma unroll
    for (int j = 0; j < kMaxVals; ++j) {
      if (j >= p.num_vals) continue;
      const int ops = p.val_ops[j];
      for (int64_t g = threadIdx.x; g < p.num_groups; g += blockDim.x) {
        if (ops & OPS_SUM) reinterpret_cast<int64_t*>(smem + p.lds_sum_off[j])[g] = 0;  // 0 == +0.0
        if (ops & OPS_MIN) reinterpret_cast<int64_t*>(smem + p.lds_min_off[j])[g] = INT64_MAX;
        if (ops & OPS_MAX) reinterpret_cast<int64_t*>(smem + p.lds_max_off[j])[g] = INT64_MIN;
      }
    }
    const int64_t nh = p.num_groups * p.num_hll * m;
    for (int64_t i = threadIdx.x; i < nh; i += blockDim.x) lds_hll[i] = 0;
  } else if (MODE == MODE_AGG) {
    for (int i = threadIdx.x; i < p.num_hll * m; i += blockDim.x) lds_hll[i] = 0;
  } else if (MODE == MODE_PARTITION) {
    if (threadIdx.x == 0) PL.stage_n = 0;
  }
  __syncthreads();
  const int shard = blockIdx.x & (kPartShards - 1);

  unsigned long long matched = 0;  // wave-uniform
  // MODE_AGG per-lane accumulators, one set per value column
  int64_t a_isum[kMaxVals], a_min[kMaxVals], a_max[kMaxVals];
  double a_dsum[kMaxVals];
#pragma unroll
  for (int j = 0; j < kMaxVals; ++j) {
    a_isum[j] = 0;
    a_dsum[j] = 0.0;
    a_min[j] = INT64_MAX;
    a_max[j] = INT64_MIN;
  }

  for (int32_t c = p.chunk_begin + blockIdx.x; c < p.chunk_end; c += gridDim.x) {
    const Chunk ch = p.chunks[c];
    const DevSegment* S = p.segs + ch.seg;
    const uint32_t ndocs = (uint32_t)S->num_docs;
    const int32_t iters = (ch.word_end - ch.word_begin + nwaves * U - 1) / (nwaves * U);
    for (int32_t it = 0; it < iters; ++it) {
      const int32_t w0 = ch.word_begin + (it * nwaves + wave) * U;
      uint32_t doc[U];
      bool hit[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        doc[u] = (uint32_t)(w0 + u) * 64u + (uint32_t)lane;
        hit[u] = (w0 + u) < ch.word_end && doc[u] < ndocs;
      }
      const int32_t nvalid = min(U, ch.word_end - w0);
      if (nvalid > 0) stage_streams(p, S, w0, nvalid, wst, lane);
      filter_words(p, S, wst, lane, doc, hit);
      unsigned long long bal[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        bal[u] = __ballot(hit[u]);
        matched += __popcll(bal[u]);
      }
      if (MODE == MODE_COUNT) continue;

      // decode-once: group key and every value column of the U docs (independent loads in flight)
      int64_t vi[U][kMaxVals];
      double vd[U][kMaxVals];
      int64_t key[U];
      static_for<0, U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        key[u] = 0;
#pragma unroll
        for (int j = 0; j < kMaxVals; ++j) {
          vi[u][j] = 0;
          vd[u][j] = 0.0;
        }
        if (!hit[u]) return;
#pragma unroll
        for (int j = 0; j < kMaxVals; ++j)
          if (j < p.num_vals)
            read_value(S->vals[j], stream_bits(p, S, wst, p.v_stream[j], u, lane, doc[u]), vi[u][j], vd[u][j]);
        if (NG > 0) key[u] = group_key<NG>(p, S, wst, u, lane, doc[u]);
      });

      if (MODE == MODE_PARTITION) {
        // append matched records to the block's LDS stage (one LDS atomic per wave)
        uint32_t tot = 0, pre[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          pre[u] = tot;
          tot += (uint32_t)__popcll(bal[u]);
        }
        uint32_t base = 0;
        if (tot) {
          if (lane == 0) base = atomicAdd(&PL.stage_n, tot);
          base = __shfl(base, 0, 64);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (hit[u]) {
            const uint32_t idx = base + pre[u] + lanes_below(bal[u], lane);
            PL.st_key[idx] = (uint32_t)key[u];
            PL.st_val[idx] = p.num_vals ? (uint32_t)(vi[u][0] - p.part_vbase) : 0u;
          }
        }
        __syncthreads();
        if (PL.stage_n > (uint32_t)(PartLds<REC64>::kStage - kPartBlock * U)) part_flush<REC64>(p, PL, shard);
        continue;
      }

      static_for<0, U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if (!hit[u]) return;
        const int64_t g = key[u];
        if (MODE == MODE_GROUP_LDS) atomicAdd(&lds_cnt[g], 1u);
        else if (MODE == MODE_GROUP_GLOBAL) atomicAdd(&p.out_count[g], 1ull);
#pragma unroll
        for (int j = 0; j < kMaxVals; ++j) {
          if (j >= p.num_vals) continue;
          const int ops = p.val_ops[j];
          const int64_t iv = vi[u][j];
          if (MODE == MODE_AGG) {
            if (ops & OPS_SUM) {
              if (p.val_is_int[j]) a_isum[j] += iv; else a_dsum[j] += vd[u][j];
            }
            if (ops & OPS_MIN) a_min[j] = iv < a_min[j] ? iv : a_min[j];
            if (ops & OPS_MAX) a_max[j] = iv > a_max[j] ? iv : a_max[j];
          } else {
            void* sb = MODE == MODE_GROUP_LDS ? (void*)(smem + p.lds_sum_off[j]) : p.out_sum[j];
            long long* mnb = MODE == MODE_GROUP_LDS ? reinterpret_cast<long long*>(smem + p.lds_min_off[j])
                                                    : reinterpret_cast<long long*>(p.out_min[j]);
            long long* mxb = MODE == MODE_GROUP_LDS ? reinterpret_cast<long long*>(smem + p.lds_max_off[j])
                                                    : reinterpret_cast<long long*>(p.out_max[j]);
            if (ops & OPS_SUM) {
              if (p.val_is_int[j]) atomicAdd(reinterpret_cast<unsigned long long*>(sb) + g, (unsigned long long)iv);
              else atomicAdd(reinterpret_cast<double*>(sb) + g, vd[u][j]);
            }
            if (ops & OPS_MIN) atomicMin(mnb + g, (long long)iv);
            if (ops & OPS_MAX) atomicMax(mxb + g, (long long)iv);
          }
        }
#pragma unroll
        for (int h = 0; h < kMaxHll; ++h) {
          if (h >= p.num_hll) continue;
          const DevColumn& col = S->cols[p.hll_slot[h]];
          const uint32_t e = gld(col.hll + unpack_col(col, doc[u]));
          const int64_t r = (g * p.num_hll + h) * m + (e >> 8);
          if (MODE == MODE_GROUP_GLOBAL) atomicMax(&p.out_hll[r], e & 0xffu);
          else atomicMax(&lds_hll[r], e & 0xffu);
        }
      });
    }
  }

  // ---- block epilogue
  if (MODE == MODE_PARTITION) {
    __syncthreads();
    if (PL.stage_n) part_flush<REC64>(p, PL, shard);
    return;
  }
  __shared__ unsigned long long s_matched;
  if (threadIdx.x == 0) s_matched = 0;
  __syncthreads();
  if (lane == 0 && matched) atomicAdd(&s_matched, matched);
  if (MODE == MODE_AGG) {
    __shared__ int64_t s_isum[4][kMaxVals], s_min[4][kMaxVals], s_max[4][kMaxVals];
    __shared__ double s_dsum[4][kMaxVals];
#pragma unroll
    for (int j = 0; j < kMaxVals; ++j) {
      if (j >= p.num_vals) continue;
      const int64_t si = wave_sum_i64(a_isum[j]);
      const double sd = wave_sum_f64(a_dsum[j]);
      const int64_t mn = wave_min_i64(a_min[j]);
      const int64_t mx = wave_max_i64(a_max[j]);
      if (lane == 0 && wave < 4) {
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
      for (int wv = 1; wv < nwaves && wv < 4; ++wv) {
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
      for (int j = 0; j < kMaxVals; ++j) {
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
    for (int64_t i = threadIdx.x; i < nh; i += blockDim.x)
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

template <int MODE, int NG>
static void launch_ng(const KParams& p, int rec64, int grid, int block, size_t lds, hipStream_t s) {
  if (rec64) {
    allow_lds(k_scan<MODE, NG, 1>, lds);
    hipLaunchKernelGGL((k_scan<MODE, NG, 1>), dim3(grid), dim3(block), lds, s, p);
  } else {
    allow_lds(k_scan<MODE, NG, 0>, lds);
    hipLaunchKernelGGL((k_scan<MODE, NG, 0>), dim3(grid), dim3(block), lds, s, p);
  }
}

template <int MODE>
static void launch_mode(const KParams& p, int ng, int rec64, int grid, int block, size_t lds, hipStream_t s) {
  switch (ng) {
    case 0: launch_ng<MODE, 0>(p, rec64, grid, block, lds, s); break;
    case 1: launch_ng<MODE, 1>(p, rec64, grid, block, lds, s); break;
    case 2: launch_ng<MODE, 2>(p, rec64, grid, block, lds, s); break;
    case 3: launch_ng<MODE, 3>(p, rec64, grid, block, lds, s); break;
    default: launch_ng<MODE, 4>(p, rec64, grid, block, lds, s); break;
  }
}

size_t partition_stage_offset(int rec64) { return part_stage_off(rec64); }

void launch_scan(const KParams& p, int mode, int ng, int rec64, int grid, int block, size_t lds, hipStream_t s) {
  switch (mode) {
    case MODE_COUNT: hipLaunchKernelGGL((k_scan<MODE_COUNT, 0, 0>), dim3(grid), dim3(block), lds, s, p); break;
    case MODE_AGG: hipLaunchKernelGGL((k_scan<MODE_AGG, 0, 0>), dim3(grid), dim3(block), lds, s, p); break;
    case MODE_GROUP_LDS: launch_mode<MODE_GROUP_LDS>(p, ng, 0, grid, block, lds, s); break;
    case MODE_GROUP_GLOBAL: launch_mode<MODE_GROUP_GLOBAL>(p, ng, 0, grid, block, lds, s); break;
    default:
      launch_mode<MODE_PARTITION>(p, ng, rec64, grid, kPartBlock,
                                  part_stage_off(rec64) + (kPartBlock / 64) * kMaxStage * kStageBytes, s);
      break;
  }
  PH_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ kernel B: partition aggregation
__global__ void __launch_bounds__(1024) k_part_agg(const PartAggParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int P = p.num_parts;
  const int part = blockIdx.x;
  const uint32_t KP = 1u << p.part_klo;
  // compact LDS layout: count | sum (8 B) | min | max, only the tables the query needs
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);
  size_t off = 4 * (size_t)KP;
  unsigned long long* sum = reinterpret_cast<unsigned long long*>(smem + off);
  off += p.has_sum ? 8 * (size_t)KP : 0;
  uint32_t* mn = reinterpret_cast<uint32_t*>(smem + off);
  off += p.has_min ? 4 * (size_t)KP : 0;
  uint32_t* mx = reinterpret_cast<uint32_t*>(smem + off);
  for (uint32_t k = threadIdx.x; k < KP; k += blockDim.x) {
    cnt[k] = 0;
    if (p.has_sum) sum[k] = 0;
    if (p.has_min) mn[k] = 0xffffffffu;
    if (p.has_max) mx[k] = 0u;
  }
  __shared__ uint32_t s_n[kPartShards];
  if (threadIdx.x < kPartShards) {
    const uint32_t c = p.part_cursor[threadIdx.x * P + part];
    s_n[threadIdx.x] = c < (uint32_t)p.part_cap ? c : (uint32_t)p.part_cap;
  }
  __syncthreads();
  const uint32_t vmask = p.part_vbits ? ((p.part_vbits >= 32) ? 0xffffffffu : ((1u << p.part_vbits) - 1u)) : 0u;
  for (int sh = 0; sh < kPartShards; ++sh) {
    const uint32_t n = s_n[sh];
    const size_t base = ((size_t)sh * P + part) * (size_t)p.part_cap;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
      uint32_t k, v;
      if (p.rec64) {
        const unsigned long long r = reinterpret_cast<const unsigned long long*>(p.part_buf)[base + i];
        k = (uint32_t)(r >> 32);
        v = (uint32_t)r;
      } else {
        const uint32_t r = reinterpret_cast<const uint32_t*>(p.part_buf)[base + i];
        k = r >> p.part_vbits;
        v = r & vmask;
      }
      atomicAdd(&cnt[k], 1u);
      if (p.has_sum) atomicAdd(&sum[k], (unsigned long long)v);
      if (p.has_min) atomicMin(&mn[k], v);
      if (p.has_max) atomicMax(&mx[k], v);
    }
  }
  __syncthreads();
  if (threadIdx.x < kPartShards) p.part_cursor[threadIdx.x * P + part] = 0;  // ready for the next batch
  for (uint32_t k = threadIdx.x; k < KP; k += blockDim.x) {
    const uint32_t c = cnt[k];
    if (!c) continue;
    const int64_t g = ((int64_t)part << p.part_klo) | k;
    if (g >= p.num_groups) continue;
    p.out_count[g] += c;  // this block owns keys [part << klo, (part + 1) << klo)
    if (p.has_sum) p.out_sum[g] += (int64_t)sum[k] + (int64_t)c * p.part_vbase;
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
  allow_lds(k_part_agg, lds);
  hipLaunchKernelGGL(k_part_agg, dim3(p.num_parts), dim3(1024), lds, s, p);
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
  for (int64_t g = g0 + threadIdx.x; g < g1; g += blockDim.x) c += p.count[g] != 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ uint32_t ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) p.blk[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
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
        const int64_t id = (g / p.key_stride[j]) % p.key_size[j];
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
