// kernels.hip -- gfx950 kernels of libpinot_hip.so outside the scan template: the launch dispatcher, value
// re-encoding, result compaction, self-tests, HLL tables and the roaring OR (the scan kernel itself is
// scan_kernel.h, instantiated per plan mode by scan_*.hip).
#include <map>
#include <mutex>
#include <utility>

#include "scan_kernel.h"

namespace ph {

void launch_scan_agg(const KParams& p, int mode, int grid, size_t lds, hipStream_t s);
void launch_scan_group_lds(const KParams& p, int ng, int grid, size_t lds, hipStream_t s);
void launch_scan_group_global(const KParams& p, int ng, int grid, size_t lds, hipStream_t s);
void launch_scan_partition(const KParams& p, int ng, int rec64, int grid, size_t lds, hipStream_t s);
void launch_scan_group_hash(const KParams& p, int ng, int grid, size_t lds, hipStream_t s);

void launch_scan(const KParams& p, int mode, int ng, int rec64, int grid, size_t lds, hipStream_t s) {
  if (mode == MODE_COUNT && p.count_reg) {  // register-direct COUNT over RANGE / ALL / DOCRANGE leaves
    launch_count_reg(p, grid, s);
    return;
  }
  if ((mode == MODE_GROUP_LDS || mode == MODE_GROUP_GLOBAL) && p.group_sparse && !p.first_doc) {
    launch_group_sparse(p, mode, grid, lds, s);  // selective bitmap ANDs: gathers of the matched docs
    return;
  }
  if (mode == MODE_GROUP_LDS && p.group_reg) {  // register-direct form of k_group_lds_lean
    launch_group_reg(p, ng, grid, lds, s);
    return;
  }
  PH_HIP_CHECK(hipGetLastError());  // a failure left by an earlier unchecked call is reported as such, not as ours
  switch (mode) {
    case MODE_COUNT:
    case MODE_AGG: launch_scan_agg(p, mode, grid, lds, s); break;
    case MODE_GROUP_LDS: launch_scan_group_lds(p, ng, grid, lds, s); break;
    case MODE_GROUP_GLOBAL: launch_scan_group_global(p, ng, grid, lds, s); break;
    case MODE_GROUP_HASH: launch_scan_group_hash(p, ng, grid, lds, s); break;
    default: launch_scan_partition(p, ng, rec64, grid, lds, s); break;
  }
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
  PH_HIP_CHECK(hipGetLastError());  // a failure left by an earlier unchecked call is reported as such, not as ours
  hipLaunchKernelGGL(k_encode_values, dim3(grid), dim3(256), 0, s, fwd, bits, table, base, vbits, n, out, nwords);
  PH_HIP_CHECK(hipGetLastError());
}

void allow_lds_raw(const void* kernel, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> set;  // the largest dynamic LDS set per (kernel, device)
  int dev = 0;
  PH_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  size_t& cur = set[{kernel, dev}];
  if (cur >= lds) return;
  PH_HIP_CHECK(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  cur = lds;
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
        const int64_t kid = p.hkeys ? (int64_t)p.hkeys[g] : g + p.key_base;
        const int64_t id = (kid / p.key_stride[j]) % p.key_size[j];
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

// ------------------------------------------------------------------ numGroupsLimit (first-seen keys)
// DictionaryBasedGroupKeyGenerator hands out group ids in first-seen doc order and drops the docs of every key
// that arrives after numGroupsLimit ids were taken (IntGroupIdMap.getGroupId, :992-1017; INVALID_ID rows are
// ignored by the result holders).  Given first[g] = the first matching doc of key g in one segment (UINT32_MAX:
// absent), the kept keys are exactly the `limit` keys with the smallest first docs: distinct keys have distinct
// first docs, so the keys kept are those whose first doc is below the doc of the limit-th set bit of the
// first-doc bitmap.
// (blockIdx.y = limit segment: its first-doc table, doc bitmap, scalars and keep bitset)
__global__ void __launch_bounds__(256) k_limit_mark(const uint32_t* __restrict__ first, int64_t G,
                                                    uint32_t* __restrict__ docbits, int64_t dbw,
                                                    unsigned long long* distinct) {
  first += (int64_t)blockIdx.y * G;
  docbits += (int64_t)blockIdx.y * dbw;
  distinct += 3 * (int64_t)blockIdx.y;
  unsigned long long d = 0;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < G; g += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t f = first[g];
    if (f != 0xffffffffu) {
      ++d;
      atomicOr(&docbits[f >> 5], 1u << (f & 31u));
    }
  }
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
  if ((threadIdx.x & 63) == 0 && d) atomicAdd(distinct, d);
}

// one workgroup: threshold = (doc of the limit-th set bit) + 1, or UINT32_MAX when distinct <= limit
__global__ void __launch_bounds__(1024) k_limit_threshold(const uint32_t* __restrict__ docbits, int64_t nwords,
                                                          int64_t limit, unsigned long long* scal) {
  docbits += (int64_t)blockIdx.x * nwords;
  const unsigned long long* distinct = scal + 3 * (int64_t)blockIdx.x;
  uint32_t* threshold = reinterpret_cast<uint32_t*>(scal + 3 * (int64_t)blockIdx.x + 1);
  unsigned long long* reached = scal + 3 * (int64_t)blockIdx.x + 2;
  __shared__ unsigned long long wsum[1024];
  __shared__ uint32_t found;
  const int t = threadIdx.x;
  const unsigned long long D = *distinct;
  if (t == 0) {
    found = 0xffffffffu;
    if ((int64_t)D >= limit) *reached = 1;  // GroupByOperator: numGroups >= numGroupsLimit
  }
  if ((int64_t)D <= limit) {
    if (t == 0) *threshold = 0xffffffffu;
    return;
  }
  const int64_t per = (nwords + 1023) / 1024, w0 = t * per, w1 = min(nwords, w0 + per);
  unsigned long long c = 0;
  for (int64_t w = w0; w < w1; ++w) c += __popc(docbits[w]);
  wsum[t] = c;
  __syncthreads();
  if (t == 0) {  // exclusive prefix (1024 entries, once per segment)
    unsigned long long acc = 0;
    for (int i = 0; i < 1024; ++i) {
      const unsigned long long x = wsum[i];
      wsum[i] = acc;
      acc += x;
    }
  }
  __syncthreads();
  // the thread whose range holds the limit-th bit (1-based rank `limit`) walks its words
  const unsigned long long before = wsum[t];
  if (before < (unsigned long long)limit && before + c >= (unsigned long long)limit) {
    unsigned long long need = (unsigned long long)limit - before;  // >= 1
    for (int64_t w = w0; w < w1; ++w) {
      uint32_t bits = docbits[w];
      const uint32_t pc = __popc(bits);
      if (need > pc) {
        need -= pc;
        continue;
      }
      for (;;) {
        const uint32_t b = __ffs(bits) - 1;
        if (--need == 0) {
          found = (uint32_t)(w * 32 + b) + 1u;
          break;
        }
        bits &= bits - 1;
      }
      break;
    }
  }
  __syncthreads();
  if (t == 0) *threshold = found;
}

// keep bit g  <=>  key g is present and its first doc is below the threshold
__global__ void __launch_bounds__(256) k_limit_keep(const uint32_t* __restrict__ first, int64_t G,
                                                    const unsigned long long* scal, uint32_t* __restrict__ keep) {
  const int64_t nw = (G + 31) / 32;
  first += (int64_t)blockIdx.y * G;
  keep += (int64_t)blockIdx.y * nw;
  const uint32_t T = *reinterpret_cast<const uint32_t*>(scal + 3 * (int64_t)blockIdx.y + 1);
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    uint32_t bits = 0;
    for (int i = 0; i < 32; ++i) {
      const int64_t g = w * 32 + i;
      if (g < G && first[g] < T) bits |= 1u << i;
    }
    keep[w] = bits;
  }
}

void launch_limit_select(const uint32_t* first, int64_t G, int64_t limit, int nseg, int64_t dbw, uint32_t* docbits,
                         uint32_t* keep, unsigned long long* scal, hipStream_t s) {
  if (nseg <= 0) return;
  const int grid = (int)std::min<int64_t>((G + 255) / 256, 4096);
  hipLaunchKernelGGL(k_limit_mark, dim3(grid, nseg), dim3(256), 0, s, first, G, docbits, dbw, scal);
  hipLaunchKernelGGL(k_limit_threshold, dim3(nseg), dim3(1024), 0, s, docbits, dbw, limit, scal);
  const int grid2 = (int)std::min<int64_t>(((G + 31) / 32 + 255) / 256, 4096);
  hipLaunchKernelGGL(k_limit_keep, dim3(grid2, nseg), dim3(256), 0, s, first, G, scal, keep);
  PH_HIP_CHECK(hipGetLastError());
}

// Non-empty groups of a dense / hash count table (the optimistic numGroupsLimit check: when the merged table has
// fewer than `limit` groups, no segment can have reached the limit, so its first-seen pass is not needed)
__global__ void __launch_bounds__(256) k_count_nonzero(const unsigned long long* __restrict__ cnt, int64_t n,
                                                       unsigned long long* out) {
  unsigned long long d = 0;
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x)
    d += cnt[g] != 0;
  for (int o = 32; o > 0; o >>= 1) d += __shfl_xor(d, o, 64);
  if ((threadIdx.x & 63) == 0 && d) atomicAdd(out, d);
}

void launch_count_nonzero(const unsigned long long* cnt, int64_t n, unsigned long long* out, hipStream_t s) {
  PH_HIP_CHECK(hipMemsetAsync(out, 0, 8, s));
  if (n <= 0) return;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_count_nonzero, dim3(grid), dim3(256), 0, s, cnt, n, out);
  PH_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------ helpers
// Self-test of the scan kernels' staged decode: the same tile_load / tile_store / BitCursor code k_scan runs
// (one stream, stage offset 0), writing every decoded dictId out.
__global__ void __launch_bounds__(kBlock) k_selftest_staged(const DevSegment* segs, int32_t tile_words,
                                                            int32_t stage_stride, int32_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  SegPtr S = (SegPtr)segs;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* wst = smem + (size_t)wave * stage_stride;
  const int32_t ndocs = S->num_docs;
  const int32_t nwords = (ndocs + 63) / 64;
  const int bits = S->streams[0].bits;
  for (int32_t w0 = (blockIdx.x * kWaves + wave) * tile_words; w0 < nwords; w0 += gridDim.x * kWaves * tile_words) {
    const int32_t nvalid = min(tile_words, nwords - w0);
    Prefetch<kPrefetchOther> pf;
    tile_load<kPrefetchOther>(S, w0, nvalid, lane, pf);
    tile_store<kPrefetchOther>(S, nvalid, wst, lane, pf);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const BitCursor c = bit_cursor(wst, bits, lane);
    for (int u = 0; u < nvalid; ++u) {
      const int32_t doc = (w0 + u) * 64 + lane;
      if (doc < ndocs) out[doc] = (int32_t)cursor_value(c, u);
    }
    __builtin_amdgcn_wave_barrier();  // the staging area is rewritten by the next tile
  }
}

void launch_selftest_staged(const DevSegment* seg, int32_t tile_words, int32_t stage_stride, int64_t n, int32_t* out,
                            hipStream_t s) {
  if (n <= 0) return;
  const int64_t tiles = ((n + 63) / 64 + tile_words - 1) / tile_words;
  const int grid = (int)std::min<int64_t>((tiles + kWaves - 1) / kWaves, 1024);
  hipLaunchKernelGGL(k_selftest_staged, dim3(grid), dim3(kBlock), (size_t)kWaves * stage_stride, s, seg, tile_words,
                     stage_stride, out);
  PH_HIP_CHECK(hipGetLastError());
}

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

// ------------------------------------------------------------------ filter-entry statistic (AndDocIdIterator)
// Doc bitmaps of up to kMaxFbProgs leaves of one segment's filter tree (the leaves k_leaf_bitmaps does not take:
// sorted ranges, inverted-index bitmaps, large dictId sets), one wave per 64-doc word, each leaf into its output row:
// the filter-statistic pass walks or simulates the reference's iterators over them (query.cpp).
__global__ void __launch_bounds__(256) k_filter_bitmaps(const FilterInsn* __restrict__ prog, const DevSegment* segs,
                                                        const FbJob job) {
  SegPtr S = (SegPtr)(segs + job.seg);
  const int lane = threadIdx.x & 63;
  const uint32_t ndocs = (uint32_t)S->num_docs;
  for (int64_t w = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; w < job.nwords;
       w += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const uint32_t doc = (uint32_t)w * 64u + (uint32_t)lane;
    for (int k = 0; k < job.nprog; ++k) {
      uint32_t fent = 0;
      const bool b = doc < ndocs && eval_filter((const PH_CONST FilterInsn*)prog + job.off[k], job.len[k], S, doc, fent);
      const unsigned long long bal = __ballot(b);
      if (lane == 0) job.out[(int64_t)job.row[k] * job.nwords + w] = bal;
    }
  }
}

void launch_filter_bitmaps(const FilterInsn* prog, const DevSegment* segs, const FbJob& job, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((job.nwords + 3) / 4, 4096);
  if (blocks <= 0) return;
  PH_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_filter_bitmaps, dim3((unsigned)blocks), dim3(256), 0, s, prog, segs, job);
  PH_HIP_CHECK(hipGetLastError());
}

// The multi-device combine's local transport (logical shards sharing one device, multi.cpp): dst = dst (op) src over n
// elements of one dense partial table (ph_reduce_op; identities never change a live value)
__global__ void k_reduce_table(void* dst, const void* src, int64_t n, int32_t op) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    switch (op) {
      case PH_REDUCE_SUM_I64: static_cast<int64_t*>(dst)[i] += static_cast<const int64_t*>(src)[i]; break;
      case PH_REDUCE_SUM_F64: static_cast<double*>(dst)[i] += static_cast<const double*>(src)[i]; break;
      case PH_REDUCE_MIN_I64: {
        int64_t* d = static_cast<int64_t*>(dst) + i;
        *d = min(*d, static_cast<const int64_t*>(src)[i]);
        break;
      }
      case PH_REDUCE_MAX_I64: {
        int64_t* d = static_cast<int64_t*>(dst) + i;
        *d = max(*d, static_cast<const int64_t*>(src)[i]);
        break;
      }
      default: {
        uint32_t* d = static_cast<uint32_t*>(dst) + i;
        *d = max(*d, static_cast<const uint32_t*>(src)[i]);
      }
    }
  }
}

void launch_reduce_table(void* dst, const void* src, int64_t n, int32_t op, hipStream_t s) {
  if (n <= 0) return;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_reduce_table, dim3(grid), dim3(256), 0, s, dst, src, n, op);
  PH_HIP_CHECK(hipGetLastError());
}

// identity of a reduce op over [0, n) elements (padding rows, and the tables of a device without segments)
__global__ void k_fill_identity(void* dst, int64_t n, int32_t op) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (op == PH_REDUCE_MAX_U32) static_cast<uint32_t*>(dst)[i] = 0u;
    else if (op == PH_REDUCE_SUM_F64) static_cast<double*>(dst)[i] = 0.0;
    else static_cast<int64_t*>(dst)[i] = op == PH_REDUCE_MIN_I64 ? INT64_MAX : (op == PH_REDUCE_MAX_I64 ? INT64_MIN : 0);
  }
}

void launch_fill_identity(void* dst, int64_t n, int32_t op, hipStream_t s) {
  if (n <= 0) return;
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_fill_identity, dim3(grid), dim3(256), 0, s, dst, n, op);
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

// clearspring MurmurHash.hash(Object) of a dictionary value: Integer / Long -> hashLong(value), Double ->
// hashLong(doubleToRawLongBits), Float -> hashLong(floatToRawIntBits) (the int bits widened to long); the device table
// holds every value widened to int64 / float64 (a FLOAT's float64 is exact, so it narrows back to its own bits)
__global__ void k_hll_table(const void* __restrict__ values, int32_t kind, int64_t n, int log2m,
                            uint32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t v;
    if (kind == PH_HLL_HASH_INT) {
      v = reinterpret_cast<const int64_t*>(values)[i];
    } else if (kind == PH_HLL_HASH_FLOAT) {
      v = (int64_t)__float_as_int((float)reinterpret_cast<const double*>(values)[i]);  // floatToRawIntBits
    } else {
      v = __double_as_longlong(reinterpret_cast<const double*>(values)[i]);  // doubleToRawLongBits
    }
    out[i] = hll_entry_of(murmur_long(v), log2m);
  }
}

void launch_hll_table(const void* values, int32_t kind, int64_t n, int log2m, uint32_t* out, hipStream_t s) {
  if (n <= 0) return;
  int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_hll_table, dim3(grid), dim3(256), 0, s, values, kind, n, log2m, out);
  PH_HIP_CHECK(hipGetLastError());
}

int32_t murmur_hash_long(int64_t v) { return murmur_long(v); }
uint32_t hll_entry(int32_t hash, int log2m) { return hll_entry_of(hash, log2m); }

// Portable-roaring containers -> doc bitmap (bytes read individually because container payloads need not be
// 2-byte aligned inside the inverted-index buffer).
__device__ __forceinline__ uint32_t ld_u16(const uint8_t* b) { return (uint32_t)b[0] | ((uint32_t)b[1] << 8); }

// ORs one container's docs (hi | low 16 bits) below `limit` into `bitmap` (word = doc / 32); `bitmap` is the
// device doc bitmap (hi = key << 16, limit = num_docs) or a workgroup's LDS chunk (hi = 0, limit = docs in chunk)
__device__ __forceinline__ void roaring_or_container(const RoaringContainer& c, const uint8_t* __restrict__ base,
                                                     uint32_t* bitmap, uint32_t hi, uint32_t limit, int lane,
                                                     int nlanes = 64) {
  const uint8_t* pay = base + c.offset;
  if (c.type == 0) {  // array container: card x uint16 LE
    for (int i = lane; i < c.card; i += nlanes) {
      const uint32_t doc = hi | ld_u16(pay + 2 * i);
      if (doc < limit) atomicOr(&bitmap[doc >> 5], 1u << (doc & 31u));
    }
  } else if (c.type == 1) {  // bitmap container: 1024 x uint64 LE = 2048 x uint32 LE
    // aligned dword loads, funnel-shifted when the payload is not 4-byte aligned (one load per word instead of four
    // byte loads; the device buffer carries 16 bytes past its end, so the dword after the last one is readable)
    const uintptr_t pa = reinterpret_cast<uintptr_t>(pay);
    const uint32_t* A = reinterpret_cast<const uint32_t*>(pa & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(pa & 3u) * 8u;  // (wave-uniform)
    // the words below `limit` (no early exit inside the loop, so the loads of several iterations overlap)
    const int nw = limit > hi ? (int)min(2048u, (limit - hi + 31u) >> 5) : 0;
#pragma unroll 4
    for (int i = lane; i < nw; i += nlanes) {
      const uint32_t d0 = hi + 32u * (uint32_t)i;
      uint32_t v = A[i];
      if (sh) v = __builtin_amdgcn_alignbit(A[i + 1], v, sh);
      if (limit - d0 < 32u) v &= (1u << (limit - d0)) - 1u;
      if (v) atomicOr(&bitmap[d0 >> 5], v);
    }
  } else {  // run container: uint16 numRuns, then (start, length-1) pairs
    for (int r = lane; r < c.card; r += nlanes) {
      const uint32_t start = hi | ld_u16(pay + 2 + 4 * r);
      const uint32_t end = start + ld_u16(pay + 4 + 4 * r);  // inclusive
      for (uint32_t d = start; d <= end && d < limit;) {
        const uint32_t w = d >> 5, b0 = d & 31u;
        const uint32_t last = min(end, min(limit - 1u, (w << 5) + 31u));
        const uint32_t nb = last - d + 1u;
        const uint32_t m = (nb >= 32u ? 0xffffffffu : ((1u << nb) - 1u)) << b0;
        atomicOr(&bitmap[w], m);
        d = last + 1u;
      }
    }
  }
}

// one workgroup per work item (a leaf's dictId, up to kRoaringWorkContainers of its containers): the 4 waves take
// the containers round-robin, each OR-ed by one wave straight into the zeroed device bitmap (device atomics)
__global__ void __launch_bounds__(256) k_roaring_or(const RoaringWork* __restrict__ work,
                                                    const RoaringTarget* __restrict__ targets) {
  const RoaringWork w = work[blockIdx.x];
  const RoaringTarget t = targets[w.target];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = wave; k < w.count; k += 4) {
    const RoaringContainer c = w.dir[w.first + k];
    roaring_or_container(c, t.base, t.bitmap, (uint32_t)c.key << 16, (uint32_t)t.num_docs, lane);
  }
}

void launch_roaring_or(const RoaringWork* w, int n, const RoaringTarget* targets, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_roaring_or, dim3(n), dim3(256), 0, s, w, targets);
  PH_HIP_CHECK(hipGetLastError());
}

// One workgroup per (65536-doc chunk, leaf): each wave finds, for its share of the leaf's dictIds, the container
// whose key is the chunk (64 keys per ballot, 4 ballots in flight), ORs it into the chunk's 8 KiB LDS bitmap, and
// the workgroup then stores the chunk's words (padding words included) with plain coalesced stores -- no memset,
// and LDS atomics instead of one device atomic per matched doc.
__global__ void __launch_bounds__(256) k_roaring_chunk(const RoaringLeaf* __restrict__ leaves,
                                                       const RoaringRange* __restrict__ ranges) {
  __shared__ uint32_t bm[2048];
  const RoaringLeaf L = leaves[blockIdx.y];
  const uint32_t chunk = blockIdx.x, w0 = chunk * 2048u;
  if (w0 >= (uint32_t)L.padded_words) return;  // whole workgroup
  for (int i = threadIdx.x; i < 2048; i += 256) bm[i] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nd = (uint32_t)L.num_docs, d0 = chunk << 16;
  const uint32_t limit = nd > d0 ? min(nd - d0, 65536u) : 0u;
  // the four waves share the leaf's dictIds: `per` waves OR each container together (a one-dictId leaf -- EQ, most SSB
  // dimension leaves -- takes the whole workgroup; r5 gave every dictId one wave and left the others idle)
  const int per = L.ids_count >= 4 ? 1 : 4 / max(1, L.ids_count);
  const int sub = wave % per;
  for (int r = wave / per; r < L.ids_count; r += 4 / per) {
    const RoaringRange rg = ranges[L.ids_first + r];
    int found = -1;
    // a dictId with a container in every chunk has the chunk's at index `chunk` (keys ascend): one load, no search
    if ((int)chunk < rg.count && L.dir[rg.first + chunk].key == (int)chunk) found = (int)chunk;
    for (int b = 0; b < rg.count && found < 0; b += 256) {
      int key[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int i = b + 64 * q + lane;
        key[q] = i < rg.count ? L.dir[rg.first + i].key : -1;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned long long m = __ballot(key[q] == (int)chunk);
        if (m && found < 0) found = b + 64 * q + (int)__ffsll((long long)m) - 1;
      }
    }
    if (found >= 0) roaring_or_container(L.dir[rg.first + found], L.base, bm, 0u, limit, sub * 64 + lane, per * 64);
  }
  __syncthreads();
  const uint32_t nw = min(2048u, (uint32_t)L.padded_words - w0);
  for (uint32_t i = threadIdx.x; i < nw; i += 256) L.bitmap[w0 + i] = bm[i];
}

void launch_roaring_chunk(const RoaringLeaf* leaves, int nleaves, int max_chunks, const RoaringRange* ranges,
                          hipStream_t s) {
  if (nleaves <= 0 || max_chunks <= 0) return;
  hipLaunchKernelGGL(k_roaring_chunk, dim3(max_chunks, nleaves), dim3(256), 0, s, leaves, ranges);
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph
