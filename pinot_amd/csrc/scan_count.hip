// scan_count.hip -- k_scan instantiations of the aggregation-only plans (MODE_COUNT, MODE_AGG), and the lean
// aggregation kernel k_agg_lean.
#include "scan_kernel.h"
#include "conj_reg.h"

namespace ph {

// ------------------------------------------------------------------ lean MODE_AGG
// k_agg_lean is k_scan<MODE_AGG> for the common shape -- one integer value column read from its packed
// frame-of-reference stream, no HLL, filter leaf ALL / RANGE / DOCRANGE (AggregationOperator over SUM / MIN /
// MAX / COUNT, AggregationPlanNode.java) -- written for issue efficiency: per word and lane the value offset is
// folded into 32-bit tile accumulators (sum of offsets, min / max offset; offsets < 2^26 and <= 32 words per
// tile, so the 32-bit sum cannot wrap), and the 64-bit absolute values are formed once per tile: SUM =
// sum(offsets) + matches * base (the match count from the wave's ballots), MIN / MAX = base + min / max offset.
// No LDS traffic beyond the wave's own staging, no barriers: every wave streams independently.
//
// Also FK_CONJ filters of range leaves only (an AND of dictId ranges on <= kMaxConj scan streams, no applyAnd
// statistic) and integer 2-operand value terms `a <op> b` of two packed columns (EX = PH_EXPR_MULT / SUB / ADD: SSB
// Q1.x's SUM(lo_extendedprice * lo_discount)), which fold per doc in exact int64 like k_scan's value-term path.
template <int FK, int EX>
__device__ __forceinline__ void agg_tile(const KParams& p, SegPtr S, uint32_t wst_off, int lane, int32_t w0,
                                         int32_t nvalid, int64_t& asum, int64_t& amin, int64_t& amax,
                                         unsigned long long& matched) {
  const uint32_t ndocs = (uint32_t)S->num_docs;
  LaneStream fs = lane_stream(wst_off + (uint32_t)p.stage_soff[p.f_stream],
                              FK == FK_RANGE ? S->streams[p.f_stream].bits : 1, lane);
  LaneStream vs = lane_stream(wst_off + (uint32_t)p.stage_soff[p.v_stream[0]], S->streams[p.v_stream[0]].bits, lane);
  LaneStream vs2 = vs;
  if constexpr (EX != 0)
    vs2 = lane_stream(wst_off + (uint32_t)p.stage_soff[p.v2_stream[0]], S->streams[p.v2_stream[0]].bits, lane);
  const uint32_t flo = S->flo, flen = S->flen;
  constexpr int NC = FK == FK_CONJ ? kMaxConj : 1;
  LaneStream cs[NC];
  uint32_t clo[NC], clen[NC];
  const int nconj = FK == FK_CONJ ? S->nconj : 0;
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    if (k >= nconj) continue;
    cs[k] = lane_stream(wst_off + (uint32_t)p.stage_soff[S->cstream[k]], S->streams[S->cstream[k]].bits, lane);
    clo[k] = S->clo[k];
    clen[k] = S->clen[k];
  }
  const int64_t base = S->vals[0].base, base2 = EX != 0 ? S->vals2[0].base : 0;
  uint32_t doc = (uint32_t)w0 * 64u + (uint32_t)lane;
  uint32_t tsum = 0, tmin = 0xffffffffu, tmax = 0;
  uint32_t tcnt = 0;  // wave-uniform
  for (int u = 0; u < nvalid; u += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bool hh = (u + q < nvalid) & (doc < ndocs);
      if constexpr (FK == FK_RANGE) hh &= (lds_value(fs.off, fs.rsh, fs.mask) - flo) < flen;
      if constexpr (FK == FK_DOCRANGE) hh &= (doc - flo) < flen;
      if constexpr (FK == FK_CONJ) {
#pragma unroll
        for (int k = 0; k < NC; ++k) {
          if (k >= nconj) continue;
          hh &= (lds_value(cs[k].off, cs[k].rsh, cs[k].mask) - clo[k]) < clen[k];
          cs[k].off += cs[k].step;
        }
      }
      const uint32_t v = lds_value(vs.off, vs.rsh, vs.mask);
      if constexpr (EX == 0) {
        const uint32_t m0 = hh ? v : 0u;
        tsum += m0;
        tmax = max(tmax, m0);
        tmin = min(tmin, hh ? v : 0xffffffffu);
      } else {
        const int64_t x = base + (int64_t)v, y = base2 + (int64_t)lds_value(vs2.off, vs2.rsh, vs2.mask);
        const int64_t e = EX == PH_EXPR_MULT ? x * y : (EX == PH_EXPR_SUB ? x - y : x + y);
        asum += hh ? e : 0;
        amin = min(amin, hh ? e : INT64_MAX);
        amax = max(amax, hh ? e : INT64_MIN);
        vs2.off += vs2.step;
      }
      tcnt += (uint32_t)__popcll(__ballot(hh));
      vs.off += vs.step;
      if (FK == FK_RANGE) fs.off += fs.step;
      doc += 64u;
    }
  }
  matched += tcnt;
  if constexpr (EX == 0) {
    asum += (int64_t)tsum;
    if (lane == 0) asum += base * (int64_t)tcnt;  // the matches' common base, once per wave
    if (tmin != 0xffffffffu) {                     // this lane matched in the tile
      amin = min(amin, base + (int64_t)tmin);
      amax = max(amax, base + (int64_t)tmax);
    }
  }
}

template <int EX>
__device__ __forceinline__ void agg_tile_any(const KParams& p, SegPtr S, uint32_t wst_off, int lane, int32_t w0,
                                             int32_t nvalid, int64_t& asum, int64_t& amin, int64_t& amax,
                                             unsigned long long& matched) {
  switch (S->fkind) {
    case FK_RANGE: agg_tile<FK_RANGE, EX>(p, S, wst_off, lane, w0, nvalid, asum, amin, amax, matched); break;
    case FK_DOCRANGE: agg_tile<FK_DOCRANGE, EX>(p, S, wst_off, lane, w0, nvalid, asum, amin, amax, matched); break;
    case FK_CONJ: agg_tile<FK_CONJ, EX>(p, S, wst_off, lane, w0, nvalid, asum, amin, amax, matched); break;
    default: agg_tile<FK_ALL, EX>(p, S, wst_off, lane, w0, nvalid, asum, amin, amax, matched); break;
  }
}

template <int EX>
__global__ void __launch_bounds__(kBlock) k_agg_lean(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NL = kPrefetchOther;
  constexpr int WAVES = kWaves;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  uint8_t* wst = smem + p.stage_off + (size_t)wave * p.stage_stride;
  const uint32_t wst_off = lds_addr(wst);
  int64_t asum = 0, amin = INT64_MAX, amax = INT64_MIN;
  unsigned long long matched = 0;
  const int32_t tw = p.tile_words;
  const int32_t round_words = WAVES * tw;
  const int64_t nch = p.chunk_end - p.chunk_begin;
  int32_t c = p.chunk_begin + (int32_t)(nch * blockIdx.x / gridDim.x), r = 0;
  const int32_t c_end = p.chunk_begin + (int32_t)(nch * (blockIdx.x + 1) / gridDim.x);
  int32_t cbeg = 0, cend = 0;
  SegPtr S = nullptr;
  int32_t w0 = 0, nvalid = 0;
  auto locate = [&]() {
    if (c < c_end) {
      cbeg = chunks[c].word_begin;
      cend = chunks[c].word_end;
      S = segs + chunks[c].seg;
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
    tile_store<NL>(S, nvalid, wst, lane, pf);
    SegPtr cs = S;
    const int32_t cw0 = w0, cnvalid = nvalid;
    advance();
    locate();
    if (c < c_end) tile_load<NL>(S, w0, nvalid, lane, pf);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (cnvalid > 0) agg_tile_any<EX>(p, cs, wst_off, lane, cw0, cnvalid, asum, amin, amax, matched);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the staging area is rewritten by the next tile_store
  }
  // one set of device atomics per wave (a few thousand in all)
  const int64_t si = wave_sum_i64(asum);
  const int64_t mn = wave_min_i64(amin);
  const int64_t mx = wave_max_i64(amax);
  if (lane == 0) {
    if (matched) atomicAdd(&p.out_count[0], matched);
    const int ops = p.val_ops[0];
    if (ops & OPS_SUM) atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum[0]), (unsigned long long)si);
    if ((ops & OPS_MIN) && mn != INT64_MAX) atomicMin(reinterpret_cast<long long*>(p.out_min[0]), (long long)mn);
    if ((ops & OPS_MAX) && mx != INT64_MIN) atomicMax(reinterpret_cast<long long*>(p.out_max[0]), (long long)mx);
  }
}

// ------------------------------------------------------------------ sparse MODE_AGG (selective bitmap leaves)
// k_agg_sparse serves aggregation-only queries whose every segment is filtered by an inverted-index bitmap that
// matches few docs (InvertedIndexFilterOperator -> DocIdSetOperator -> AggregationOperator): instead of streaming
// the aggregated columns through the staging tiles, it gathers the value / HLL entry of each matched doc straight
// from its packed stream.  At 1 % selectivity a 24-bit column is touched on ~19 % of its 64-byte sectors
//  instead of all of them.
// A wave step covers 64 bitmap words = 4096 docs: one 8-byte load per lane (the next step's is issued before this
// one is processed), a wave prefix sum of the lanes' popcounts places every matched doc's offset in a per-wave LDS
// list, and the list is gathered 64 docs per round with every lane busy -- so a wave pays the dependent gather
// latency once per ~41 matched docs (1 %), not once per 64-doc word.  Values: read_value on the gathered code
// (packed offset or dictId); HLL: the segment's per-dictId (register, rank) table, registers in LDS.  A segment
// filtered by an AND of scan leaves only (sp_reg) takes its step words from conj_reg.h (the leaves decoded
// register-direct) instead of a bitmap; EX: the value term `a <op> b` of one value column (SSB Q1.x's
// SUM(lo_extendedprice * lo_discount)), exact int64 for integer terms as k_scan's.
// a little-endian uint16 of a roaring payload (payloads need not be 2-byte aligned in the inverted buffer)
__device__ __forceinline__ uint32_t cont_u16(const uint8_t* b) { return (uint32_t)b[0] | ((uint32_t)b[1] << 8); }

template <int EX, int C>
__global__ void __launch_bounds__(kBlock) k_agg_sparse(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int WAVES = kWaves;
  constexpr int SW = kSparseStepWords;  // bitmap words per wave step
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = 1 << p.log2m;
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  uint32_t* lds_hll = reinterpret_cast<uint32_t*>(smem + p.lds_hll_off);
  uint16_t* list = reinterpret_cast<uint16_t*>(smem + p.pl_misc_off) + (size_t)wave * (SW * 64);
  uint32_t* csets = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off + (size_t)WAVES * SW * 64 * sizeof(uint16_t));
  for (int i = threadIdx.x; i < p.num_hll * m; i += kBlock) lds_hll[i] = 0;
  __syncthreads();
  int64_t isum[kMaxVals], vmin[kMaxVals], vmax[kMaxVals];
  double dsum[kMaxVals];
#pragma unroll
  for (int j = 0; j < kMaxVals; ++j) {
    isum[j] = 0;
    dsum[j] = 0.0;
    vmin[j] = INT64_MAX;
    vmax[j] = INT64_MIN;
  }
  unsigned long long matched = 0;  // wave-uniform
  // one matched doc: its value terms / HLL entries
  auto agg_doc = [&](SegPtr S, uint32_t doc) {
    for (int j = 0; j < p.num_vals && j < kMaxVals; ++j) {
      const PH_CONST DevValCol& vc = S->vals[j];
      int64_t iv;
      double dv;
      read_value(vc.kind, vc.base, vc.table, unpack_bits(vc.fwd, vc.bits, doc), iv, dv);
      if constexpr (EX != 0) {  // one value column with a 2-operand term (the host picks EX only then)
        const PH_CONST DevValCol& v2 = S->vals2[0];
        int64_t ib;
        double db;
        read_value(v2.kind, v2.base, v2.table, unpack_bits(v2.fwd, v2.bits, doc), ib, db);
        if (p.val_is_int[0]) {
          iv = EX == PH_EXPR_MULT ? iv * ib : (EX == PH_EXPR_SUB ? iv - ib : iv + ib);
        } else {
          const double x = vc.kind == VK_DICT_F64 ? dv : (double)iv;
          const double y = v2.kind == VK_DICT_F64 ? db : (double)ib;
          dv = EX == PH_EXPR_MULT ? (1.0 * x) * y : (EX == PH_EXPR_SUB ? x - y : x + y);
          iv = double_order_key(dv);
        }
      }
      const int ops = p.val_ops[j];
      if (ops & OPS_SUM) {
        if (p.val_is_int[j]) isum[j] += iv; else dsum[j] += dv;
      }
      if (ops & OPS_MIN) vmin[j] = iv < vmin[j] ? iv : vmin[j];
      if (ops & OPS_MAX) vmax[j] = iv > vmax[j] ? iv : vmax[j];
    }
    for (int h = 0; h < p.num_hll && h < kMaxHll; ++h) {
      ColRef col = S->cols[p.hll_slot[h]];
      const uint32_t e = gld(col.hll + unpack_col(col, doc));
      atomicMax(&lds_hll[h * m + (e >> 8)], e & 0xffu);
    }
  };
  // one wave step: lane l holds the 64-doc word of docs sb + 64 l ..; a wave prefix sum of the popcounts places every
  // matched doc in the wave's LDS list, gathered 64 docs per round with every lane busy
  auto step = [&](SegPtr S, uint32_t sb, unsigned long long bits) {
    const uint32_t cnt = (uint32_t)__popcll(bits);
    uint32_t incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    if (total == 0) return;
    uint32_t pos = incl - cnt;
    while (bits) {
      list[pos++] = (uint16_t)(lane * 64 + __builtin_ctzll(bits));
      bits &= bits - 1ull;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    matched += total;
    for (uint32_t base = 0; base < total; base += 64)
      if (base + (uint32_t)lane < total) agg_doc(S, sb + list[base + lane]);
    // every lane has read its list entries before the next step rewrites the list
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  const int64_t nch = p.chunk_end - p.chunk_begin;
  const int32_t c0 = p.chunk_begin + (int32_t)(nch * blockIdx.x / gridDim.x);
  const int32_t c1 = p.chunk_begin + (int32_t)(nch * (blockIdx.x + 1) / gridDim.x);
  for (int32_t c = c0; c < c1; ++c) {
    SegPtr S = segs + chunks[c].seg;
    const uint32_t ndocs = (uint32_t)S->num_docs;
    if constexpr (C < 0) {
      // container mode (InvertedIndexFilterOperator over EQ / IN, BitmapInvertedIndexReader.java:45-62): the chunk
      // is a range of one dictId's roaring containers (a single-value column's ids have disjoint doc sets, so the
      // leaf is their disjoint union), a wave takes one at a time -- an array container IS the matched-doc list
      // (no doc bitmap is built, written or re-read)
      for (int32_t ci = chunks[c].word_begin + wave; ci < chunks[c].word_end; ci += WAVES) {
        const RoaringContainer ct = S->cdir[ci];
        const uint8_t* pay = S->cbase + ct.offset;
        const uint32_t hi = (uint32_t)ct.key << 16;
        const bool arr = ct.type == 0;
        // an array container is one pass over its sorted low halves; bitmap / run containers are 16 wave steps of
        // 4096 docs whose 64-doc words (read, or OR-ed from the runs) are listed in LDS first
        for (int st = 0; st < (arr ? 1 : 16); ++st) {
          uint32_t n = (uint32_t)ct.card, sb = hi;
          if (!arr) {
            const uint32_t wd = hi + 4096u * (uint32_t)st + 64u * (uint32_t)lane;  // this lane's 64-doc word
            unsigned long long bits = 0;
            if (ct.type == 1) {
              const uint8_t* q = pay + 8 * (st * 64 + lane);
#pragma unroll
              for (int y = 0; y < 8; ++y) bits |= (unsigned long long)q[y] << (8 * y);
            } else {
              for (int r = 0; r < ct.card; ++r) {  // (start, length - 1) pairs; runs are rare on this path
                const uint32_t rs = hi | cont_u16(pay + 2 + 4 * r), re = rs + cont_u16(pay + 4 + 4 * r);
                if (re < wd || rs >= wd + 64u) continue;
                const uint32_t lo = rs > wd ? rs - wd : 0u, up = re - wd < 63u ? re - wd : 63u;
                bits |= (up - lo == 63u ? ~0ull : ((1ull << (up - lo + 1u)) - 1ull)) << lo;
              }
            }
            if (wd + 64u > ndocs) bits &= wd >= ndocs ? 0ull : ((1ull << (ndocs - wd)) - 1ull);
            const uint32_t cnt = (uint32_t)__popcll(bits);
            uint32_t incl = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
              const uint32_t t = __shfl_up(incl, o, 64);
              if (lane >= o) incl += t;
            }
            n = __shfl(incl, 63, 64);
            if (n == 0) continue;
            uint32_t pos = incl - cnt;
            while (bits) {
              list[pos++] = (uint16_t)(lane * 64 + __builtin_ctzll(bits));
              bits &= bits - 1ull;
            }
            sb = hi + 4096u * (uint32_t)st;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          }
          for (uint32_t base = 0; base < n; base += 64) {
            const uint32_t i = base + (uint32_t)lane;
            const uint32_t doc = i < n ? sb + (arr ? cont_u16(pay + 2 * i) : (uint32_t)list[i]) : 0xffffffffu;
            const bool ok = doc < ndocs;
            matched += (unsigned long long)__popcll(__ballot(ok));
            if (ok) agg_doc(S, doc);
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
      continue;
    } else {
    const unsigned long long* bm = reinterpret_cast<const unsigned long long*>(S->fptr);  // 64 docs per word
    const int32_t wb = chunks[c].word_begin, we = chunks[c].word_end;
    const bool reg = S->sp_reg != 0;  // chunk-uniform: every wave of the workgroup walks the same chunks
    if (C > 0 && reg) {
      __syncthreads();
      conj_stage_sets(S, csets, threadIdx.x, kBlock);
      __syncthreads();
    }
    int32_t w = wb + wave * SW;
    unsigned long long nxt = (!reg && w + lane < we) ? bm[w + lane] : 0ull;
    for (; w < we; w += WAVES * SW) {
      unsigned long long bits;
      if (reg) {
        if constexpr (C > 0) bits = conj_step_word<C>(S, w, we, lane, csets);
        else bits = 0ull;  // not reached: the host picks C > 0 when a segment has register-direct leaves
      } else {
        bits = nxt;
        const int32_t wn = w + WAVES * SW;
        nxt = (wn + lane < we) ? bm[wn + lane] : 0ull;  // the next step's bitmap words are in flight meanwhile
      }
      const uint32_t d0 = (uint32_t)(w + lane) * 64u;
      if (d0 + 64u > ndocs) bits &= d0 >= ndocs ? 0ull : ((1ull << (ndocs - d0)) - 1ull);
      step(S, (uint32_t)w * 64u, bits);
    }
    }
  }
  // epilogue: one set of device atomics per wave, registers once per workgroup
  for (int j = 0; j < p.num_vals && j < kMaxVals; ++j) {
    const int64_t si = wave_sum_i64(isum[j]);
    const double sd = wave_sum_f64(dsum[j]);
    const int64_t mn = wave_min_i64(vmin[j]);
    const int64_t mx = wave_max_i64(vmax[j]);
    if (lane == 0) {
      const int ops = p.val_ops[j];
      if (ops & OPS_SUM) {
        if (p.val_is_int[j]) atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum[j]), (unsigned long long)si);
        else atomicAdd(reinterpret_cast<double*>(p.out_sum[j]), sd);
      }
      if ((ops & OPS_MIN) && mn != INT64_MAX) atomicMin(reinterpret_cast<long long*>(p.out_min[j]), (long long)mn);
      if ((ops & OPS_MAX) && mx != INT64_MIN) atomicMax(reinterpret_cast<long long*>(p.out_max[j]), (long long)mx);
    }
  }
  if (lane == 0 && matched) atomicAdd(&p.out_count[0], matched);
  __syncthreads();
  for (int i = threadIdx.x; i < p.num_hll * m; i += kBlock)
    if (lds_hll[i]) atomicMax(&p.out_hll[i], lds_hll[i]);
}

void launch_scan_agg(const KParams& p, int mode, int grid, size_t lds, hipStream_t s) {
  if (mode == MODE_AGG && p.agg_sparse) {
    auto go = [&](auto ex) {
      constexpr int EX = decltype(ex)::value;
      if (p.sparse_c > 4) {
        allow_lds(k_agg_sparse<EX, 8>, lds);
        hipLaunchKernelGGL((k_agg_sparse<EX, 8>), dim3(grid), dim3(kBlock), lds, s, p);
      } else if (p.sparse_c > 0) {  // (the hoisted narrow-leaf form, C = 2, measured slower here: 1.01 vs 0.86 ms
                                    // on SSB Q1.x -- its registers cost the gathers their occupancy)
        allow_lds(k_agg_sparse<EX, 4>, lds);
        hipLaunchKernelGGL((k_agg_sparse<EX, 4>), dim3(grid), dim3(kBlock), lds, s, p);
      } else if (p.agg_cont) {  // straight from the leaves' roaring containers
        allow_lds(k_agg_sparse<EX, -1>, lds);
        hipLaunchKernelGGL((k_agg_sparse<EX, -1>), dim3(grid), dim3(kBlock), lds, s, p);
      } else {  // bitmap leaves only
        allow_lds(k_agg_sparse<EX, 0>, lds);
        hipLaunchKernelGGL((k_agg_sparse<EX, 0>), dim3(grid), dim3(kBlock), lds, s, p);
      }
    };
    switch (p.num_vals == 1 ? p.val_op[0] : 0) {
      case PH_EXPR_MULT: go(std::integral_constant<int, PH_EXPR_MULT>{}); break;
      case PH_EXPR_SUB: go(std::integral_constant<int, PH_EXPR_SUB>{}); break;
      case PH_EXPR_ADD: go(std::integral_constant<int, PH_EXPR_ADD>{}); break;
      default: go(std::integral_constant<int, 0>{}); break;
    }
    return;
  }
  if (mode == MODE_COUNT) {
    launch_late<MODE_COUNT, 0, 0>(p, grid, lds, s);
  } else if (p.agg_fast) {  // one kernel per value-term form (the plain column keeps k_agg_lean's r2 code size)
    switch (p.val_op[0]) {
#define PH_LEAN_CASE(e)                                                       \
  case e:                                                                     \
    allow_lds(k_agg_lean<e>, lds);                                            \
    hipLaunchKernelGGL((k_agg_lean<e>), dim3(grid), dim3(kBlock), lds, s, p); \
    break;
      PH_LEAN_CASE(PH_EXPR_MULT) PH_LEAN_CASE(PH_EXPR_SUB) PH_LEAN_CASE(PH_EXPR_ADD)
      default: PH_LEAN_CASE(0)
#undef PH_LEAN_CASE
    }
  } else if (p.num_vals <= 1 && !p.val_op[0]) {
    launch_late<MODE_AGG, 0, 1>(p, grid, lds, s);  // ValCap 1
  } else if (p.num_vals <= 1) {
    launch_late<MODE_AGG, 0, 2>(p, grid, lds, s);  // ValCap 1 + a 2-operand expression
  } else {
    launch_late<MODE_AGG, 0, 0>(p, grid, lds, s);
  }
}

}  // namespace ph
