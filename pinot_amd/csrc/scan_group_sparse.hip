// scan_group_sparse.hip -- k_group_sparse: group-by over a SELECTIVE AND of inverted-index leaves (SSB Q2.x - Q4.x:
// `c_region = 'ASIA' AND s_region = 'ASIA' AND d_year BETWEEN ...` with c_region / s_region inverted), SURVEY 8(a10)
// InvertedIndexFilterOperator + AndDocIdSet -> DefaultGroupByExecutor.
//
// The streaming kernels read every referenced column of every doc; at the 0.05-4 % selectivity of these filters
// that is 25-2000x the bytes of the matched docs.  Here a wave walks 4096 docs per step through the AND of the
// segment's doc bitmaps (k_roaring_chunk's, one 8-byte word per lane and bitmap), lists the surviving docs in LDS
// (k_agg_sparse's wave prefix sum), and then every lane takes one listed doc at a time: the remaining scan leaves
// (dictId range or bitset, in the applyAnd order -- ScanBasedDocIdIterator.applyAnd feeds scan i + 1 the docs that
// passed scans 1..i, AndDocIdSet.java:168-170, counted into numEntriesScannedInFilter), then the group key (remapped
// dictIds, mixed radix) and the value are gathered straight from the packed streams.  Aggregation is the generic
// plan's: MODE_GROUP_LDS into the workgroup's LDS table, MODE_GROUP_GLOBAL through the LDS group cache in front of
// the HBM table.  A segment filtered by scan leaves only (sp_reg) gets its step words from conj_reg.h instead of
// bitmaps: the leaves are decoded register-direct and only the matched docs' keys and values are gathered.
#include "scan_kernel.h"
#include "conj_reg.h"

namespace ph {

__device__ __forceinline__ uint32_t gs_u16(const uint8_t* b) { return (uint32_t)b[0] | ((uint32_t)b[1] << 8); }

// Container mode (C < 0): OR the docs [lo, lo + n) of container c into a chunk bitmap of 32-doc words in LDS (bit
// d - lo).  Chunks are whole 65536-doc container keys (kContWords words): lo = 0 today, n <= 65536.  A bitmap
// container's words are split over the workgroup's waves (part `part` of `parts`); array / run containers take
// one wave (part 0 of 1).
__device__ void gs_or_container(const RoaringContainer c, const uint8_t* __restrict__ base, uint32_t lo, uint32_t n,
                                uint32_t* bm, int lane, int part, int parts) {
  const uint8_t* pay = base + c.offset;
  if (c.type == 0) {  // array: sorted low halves; start near the chunk's first entry, stop past its last
    int i0 = 0;
    if (c.card > 256) {  // one probe per lane at card / 64 strides: the lanes below lo are a prefix
      const int idx = (int)((int64_t)lane * c.card / 64);
      const int nb = __popcll(__ballot(gs_u16(pay + 2 * idx) < lo));
      i0 = nb > 0 ? (int)((int64_t)(nb - 1) * c.card / 64) : 0;
    }
    for (int b0 = i0; b0 < c.card; b0 += 64) {
      const int i = b0 + lane;
      const uint32_t v = i < c.card ? gs_u16(pay + 2 * i) : 0xffffffffu;
      const uint32_t d = v - lo;
      if (d < n) atomicOr(&bm[d >> 5], 1u << (d & 31u));
      if (__ballot(v < lo + n) == 0ull) break;  // every later entry is past the chunk too
    }
  } else if (c.type == 1) {  // bitmap: 2048 little-endian 32-bit words, the chunk's n / 32 of them
    const bool al = ((uintptr_t)pay & 3u) == 0u;  // 4-byte aligned payload: one dword load per word
    for (uint32_t i = (uint32_t)(part * 64 + lane); i < (n + 31u) / 32u; i += 64u * (uint32_t)parts) {
      const uint8_t* q = pay + 4 * (lo / 32u + i);
      uint32_t v = al ? *reinterpret_cast<const uint32_t*>(q)
                      : (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
      if (n - 32u * i < 32u) v &= (1u << (n - 32u * i)) - 1u;
      if (v) atomicOr(&bm[i], v);
    }
  } else {  // run: (start, length - 1) pairs
    for (int r = lane; r < c.card; r += 64) {
      const uint32_t s0 = gs_u16(pay + 2 + 4 * r), e0 = s0 + gs_u16(pay + 4 + 4 * r);  // inclusive
      if (e0 < lo || s0 >= lo + n) continue;
      uint32_t d = s0 > lo ? s0 - lo : 0u;
      const uint32_t last = min(e0 - lo, n - 1u);
      while (d <= last) {
        const uint32_t w = d >> 5, b0 = d & 31u, hi = min(last, (w << 5) + 31u), nb = hi - d + 1u;
        atomicOr(&bm[w], (nb >= 32u ? 0xffffffffu : ((1u << nb) - 1u)) << b0);
        d = hi + 1u;
      }
    }
  }
}

template <int MODE, int EX, int C>
__global__ void __launch_bounds__(kBlock) k_group_sparse(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int WAVES = kWaves;
  constexpr int SW = kSparseStepWords;  // bitmap words per wave step
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  uint32_t* lds_cnt = reinterpret_cast<uint32_t*>(smem + p.lds_cnt_off);
  uint32_t* gkeys = reinterpret_cast<uint32_t*>(smem + p.gc_key_off);
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + p.pl_misc_off) + (size_t)wave * (SW * 64);
  uint32_t* csets = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off + (size_t)WAVES * SW * 64 * sizeof(uint16_t));
  const bool cached = MODE == MODE_GROUP_GLOBAL && p.gc_slots > 0;
  const int nslots = MODE == MODE_GROUP_LDS ? (int)p.num_groups : (cached ? p.gc_slots : 0);
  const int ops = p.num_vals ? p.val_ops[0] : 0;
  const bool is_int = p.num_vals ? p.val_is_int[0] != 0 : true;
  for (int i = threadIdx.x; i < nslots; i += kBlock) {
    lds_cnt[i] = 0;
    if (ops & OPS_SUM) {
      if (is_int) reinterpret_cast<long long*>(smem + p.lds_sum_off[0])[i] = 0;
      else reinterpret_cast<double*>(smem + p.lds_sum_off[0])[i] = 0.0;
    }
    if (ops & OPS_MIN) reinterpret_cast<long long*>(smem + p.lds_min_off[0])[i] = INT64_MAX;
    if (ops & OPS_MAX) reinterpret_cast<long long*>(smem + p.lds_max_off[0])[i] = INT64_MIN;
    if (cached) gkeys[i] = 0xffffffffu;
  }
  __syncthreads();
  unsigned long long matched = 0;
  uint32_t fent = 0;
  const int64_t nch = p.chunk_end - p.chunk_begin;
  const int32_t c0 = p.chunk_begin + (int32_t)(nch * blockIdx.x / gridDim.x);
  const int32_t c1 = p.chunk_begin + (int32_t)(nch * (blockIdx.x + 1) / gridDim.x);
  for (int32_t c = c0; c < c1; ++c) {
    SegPtr S = segs + chunks[c].seg;
    const uint32_t ndocs = (uint32_t)S->num_docs;
    const bool reg = S->sp_reg != 0;  // chunk-uniform: every wave of the workgroup walks the same chunks
    const int nbm = S->sp_nbm, nscan = reg ? 0 : S->sp_nscan;
    const int32_t wb = chunks[c].word_begin, we = chunks[c].word_end;
    if (C > 0 && reg) {
      __syncthreads();
      conj_stage_sets(S, csets, threadIdx.x, kBlock);
      __syncthreads();
    }
    uint32_t* cbm = reinterpret_cast<uint32_t*>(smem + p.cont_bm_off);  // C < 0: [nbm][kContWords * 2] words
    if constexpr (C < 0) {
      // the chunk's leaf bitmaps straight from the roaring containers (no doc bitmap in HBM): the 4 waves take the
      // leaves' dictIds round-robin (InvertedIndexFilterOperator -> BitmapInvertedIndexReader.java:45-62)
      __syncthreads();  // every wave is done with the previous chunk's words
      for (int i = threadIdx.x; i < nbm * kContWords * 2; i += kBlock) cbm[i] = 0u;
      __syncthreads();
      const uint32_t dlo = (uint32_t)wb * 64u;
      const uint32_t n = min((uint32_t)(we - wb) * 64u, ndocs - dlo);
      // the host's table names each range's container of this key (no directory search)
      const int32_t* ct = S->sp_ctab + (size_t)(dlo >> 16) * (size_t)S->sp_ntot;
      int t = 0;
      for (int k = 0; k < nbm; ++k)
        for (int r = 0; r < S->sp_nrng[k]; ++r, ++t) {
          const int32_t ci = ct[t];
          if (ci < 0) continue;
          const RoaringContainer c = S->sp_cdir[k][ci];
          if (c.type == 1)  // bitmap: every wave takes a quarter of the chunk's words
            gs_or_container(c, S->sp_cbase[k], dlo & 0xffffu, n, cbm + k * kContWords * 2, lane, wave, WAVES);
          else if ((t & (WAVES - 1)) == wave)
            gs_or_container(c, S->sp_cbase[k], dlo & 0xffffu, n, cbm + k * kContWords * 2, lane, 0, 1);
        }
      __syncthreads();
    }
    auto bm_word = [&](int32_t w) -> unsigned long long {  // the AND (of ORs) of the segment's doc bitmaps, 64 docs
      if (w >= we) return 0ull;
      unsigned long long x = ~0ull, grp = 0ull;
#pragma unroll
      for (int k = 0; k < kSparseBitmaps; ++k) {
        if (k >= nbm) continue;
        const unsigned long long v =
            C < 0 ? reinterpret_cast<const unsigned long long*>(cbm + k * kContWords * 2)[w - wb]
                  : reinterpret_cast<const unsigned long long*>(S->sp_bm[k])[w];
        if (k > 0 && S->sp_or[k]) {
          grp |= v;
        } else {
          if (k > 0) x &= grp;
          grp = v;
        }
      }
      return x & grp;
    };
    int32_t w = wb + wave * SW;
    unsigned long long nxt = reg ? 0ull : bm_word(w + lane);
    for (; w < we; w += WAVES * SW) {
      unsigned long long bits;
      if (reg) {
        if constexpr (C > 0) bits = conj_step_word<C>(S, w, we, lane, csets);
        else bits = 0ull;  // not reached: the host picks C > 0 when a segment has register-direct leaves
      } else {
        bits = nxt;
        nxt = bm_word(w + WAVES * SW + lane);  // the next step's bitmap words are in flight meanwhile
      }
      const uint32_t d0 = (uint32_t)(w + lane) * 64u;
      if (d0 + 64u > ndocs) bits &= d0 >= ndocs ? 0ull : ((1ull << (ndocs - d0)) - 1ull);
      const uint32_t cnt = (uint32_t)__popcll(bits);
      uint32_t incl = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      const uint32_t total = __shfl(incl, 63, 64);
      if (total == 0) continue;
      uint32_t pos = incl - cnt;
      while (bits) {
        list[pos++] = (uint16_t)(lane * 64 + __builtin_ctzll(bits));
        bits &= bits - 1ull;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (uint32_t base = 0; base < total; base += 64) {
        if (base + (uint32_t)lane >= total) continue;
        const uint32_t doc = (uint32_t)w * 64u + list[base + lane];
        // scan leaves in order; doc passed every bitmap (the applyAnd statistic's |D0| step)
        uint32_t lead = 0;
        bool hit = true;
#pragma unroll
        for (int k = 0; k < kMaxConj; ++k) {
          if (k >= nscan) continue;
          const uint32_t v = unpack_col(S->cols[S->sp_slot[k]], doc);
          const bool pk = S->sp_set[k] ? (bool)((gld(S->sp_set[k] + (v >> 5)) >> (v & 31u)) & 1u)
                                       : (v - S->sp_lo[k]) < S->sp_len[k];
          lead += (hit && pk) ? 1u : 0u;
          hit = hit && pk;
        }
        if (S->sp_stats && nscan) fent += 1u + min(lead, (uint32_t)nscan - 1u);
        if (!hit) continue;
        ++matched;  // numDocsScanned counts the docs of keys beyond numGroupsLimit too (GroupByOperator.java:106-107)
        int64_t key = 0;
        for (int g = 0; g < p.num_group_cols; ++g) {
          ColRef col = S->cols[p.group_slot[g]];
          uint32_t id = unpack_col(col, doc);
          if (col.remap) id = (uint32_t)gld(col.remap + id);
          key += (int64_t)id * p.group_stride[g];
        }
        if (S->keep && !((gld(S->keep + (key >> 5)) >> (key & 31)) & 1u)) continue;  // beyond numGroupsLimit
        int64_t iv = 0;
        double dv = 0.0;
        if (p.num_vals) {
          const PH_CONST DevValCol& vc = S->vals[0];
          read_value(vc.kind, vc.base, vc.table, unpack_bits(vc.fwd, vc.bits, doc), iv, dv);
          if constexpr (EX != 0) {  // `a <op> b`: exact int64 for integer terms, else double (k_scan's value term)
            const PH_CONST DevValCol& v2 = S->vals2[0];
            int64_t ib;
            double db;
            read_value(v2.kind, v2.base, v2.table, unpack_bits(v2.fwd, v2.bits, doc), ib, db);
            if (is_int) {
              iv = EX == PH_EXPR_MULT ? iv * ib : (EX == PH_EXPR_SUB ? iv - ib : iv + ib);
            } else {
              const double x = vc.kind == VK_DICT_F64 ? dv : (double)iv;
              const double y = v2.kind == VK_DICT_F64 ? db : (double)ib;
              dv = EX == PH_EXPR_MULT ? (1.0 * x) * y : (EX == PH_EXPR_SUB ? x - y : x + y);
              iv = double_order_key(dv);
            }
          }
        }
        // the workgroup's slot: the key itself (LDS table) or its group-cache slot (probe <= 8), else HBM
        int64_t g = key;
        bool local = MODE == MODE_GROUP_LDS;
        if (cached) {
          const uint32_t k32 = (uint32_t)key;
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
        else atomicAdd(&p.out_count[g], 1ull);
        if (!p.num_vals) continue;
        void* sb = local ? (void*)(smem + p.lds_sum_off[0]) : p.out_sum[0];
        long long* mnb = local ? reinterpret_cast<long long*>(smem + p.lds_min_off[0]) : reinterpret_cast<long long*>(p.out_min[0]);
        long long* mxb = local ? reinterpret_cast<long long*>(smem + p.lds_max_off[0]) : reinterpret_cast<long long*>(p.out_max[0]);
        if (ops & OPS_SUM) {
          if (is_int) atomicAdd(reinterpret_cast<unsigned long long*>(sb) + g, (unsigned long long)iv);
          else atomicAdd(reinterpret_cast<double*>(sb) + g, dv);
        }
        if (ops & OPS_MIN) atomicMin(mnb + g, (long long)iv);
        if (ops & OPS_MAX) atomicMax(mxb + g, (long long)iv);
      }
      // every lane has read its list entries before the next step rewrites the list
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  const int64_t mt = wave_sum_i64((int64_t)matched);
  if (lane == 0 && mt && p.matched_total) atomicAdd(p.matched_total, (unsigned long long)mt);
  if (p.filter_entries) {
    const int64_t fe = wave_sum_i64((int64_t)fent);
    if (lane == 0 && fe) atomicAdd(p.filter_entries, (unsigned long long)fe);
  }
  __syncthreads();
  // the workgroup's table (or cached groups) -> the HBM table, once per key
  for (int i = threadIdx.x; i < nslots; i += kBlock) {
    const uint32_t cnt = lds_cnt[i];
    if (!cnt) continue;
    const int64_t key = MODE == MODE_GROUP_LDS ? (int64_t)i : (int64_t)gkeys[i];
    atomicAdd(&p.out_count[key], (unsigned long long)cnt);
    if (!p.num_vals) continue;
    if (ops & OPS_SUM) {
      if (is_int)
        atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum[0]) + key,
                  reinterpret_cast<const unsigned long long*>(smem + p.lds_sum_off[0])[i]);
      else
        atomicAdd(reinterpret_cast<double*>(p.out_sum[0]) + key, reinterpret_cast<const double*>(smem + p.lds_sum_off[0])[i]);
    }
    if (ops & OPS_MIN)
      atomicMin(reinterpret_cast<long long*>(p.out_min[0]) + key, reinterpret_cast<const long long*>(smem + p.lds_min_off[0])[i]);
    if (ops & OPS_MAX)
      atomicMax(reinterpret_cast<long long*>(p.out_max[0]) + key, reinterpret_cast<const long long*>(smem + p.lds_max_off[0])[i]);
  }
}

template <int MODE, int C>
static void launch_sparse_mode(const KParams& p, int grid, size_t lds, hipStream_t s) {
  switch (p.num_vals ? p.val_op[0] : 0) {
#define PH_SPARSE_CASE(e)                                                              \
  case e:                                                                              \
    allow_lds(k_group_sparse<MODE, e, C>, lds);                                        \
    hipLaunchKernelGGL((k_group_sparse<MODE, e, C>), dim3(grid), dim3(kBlock), lds, s, p); \
    break;
    PH_SPARSE_CASE(PH_EXPR_MULT) PH_SPARSE_CASE(PH_EXPR_SUB) PH_SPARSE_CASE(PH_EXPR_ADD)
    default: PH_SPARSE_CASE(0)
#undef PH_SPARSE_CASE
  }
}

void launch_group_sparse(const KParams& p, int mode, int grid, size_t lds, hipStream_t s) {
  // register-direct scan leaves (conj_reg.h): 16-byte loads per lane and leaf, by the widest leaf column
  // (0: no segment has them -- the bitmap-only form)
  if (p.group_cont) {  // chunk bitmaps built in LDS from the containers
    if (mode == MODE_GROUP_LDS) launch_sparse_mode<MODE_GROUP_LDS, -1>(p, grid, lds, s);
    else launch_sparse_mode<MODE_GROUP_GLOBAL, -1>(p, grid, lds, s);
  } else if (mode == MODE_GROUP_LDS) {
    if (p.sparse_c > 4) launch_sparse_mode<MODE_GROUP_LDS, 8>(p, grid, lds, s);
    else if (p.sparse_c > 2) launch_sparse_mode<MODE_GROUP_LDS, 4>(p, grid, lds, s);
    else if (p.sparse_c > 0) launch_sparse_mode<MODE_GROUP_LDS, 2>(p, grid, lds, s);
    else launch_sparse_mode<MODE_GROUP_LDS, 0>(p, grid, lds, s);
  } else {
    if (p.sparse_c > 4) launch_sparse_mode<MODE_GROUP_GLOBAL, 8>(p, grid, lds, s);
    else if (p.sparse_c > 2) launch_sparse_mode<MODE_GROUP_GLOBAL, 4>(p, grid, lds, s);
    else if (p.sparse_c > 0) launch_sparse_mode<MODE_GROUP_GLOBAL, 2>(p, grid, lds, s);
    else launch_sparse_mode<MODE_GROUP_GLOBAL, 0>(p, grid, lds, s);
  }
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph
