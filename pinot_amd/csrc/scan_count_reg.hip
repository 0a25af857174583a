// scan_count_reg.hip -- k_count_reg: COUNT(*) over one dictId RANGE scan leaf per segment (or ALL / sorted DOCRANGE) (BASELINE config 2: SVScanDocIdIterator
// + a RANGE predicate evaluator feeding FastFilteredCount-less AggregationOperator) in the
// register-direct form of reg_decode.h.  Each wave streams its tiles independently (no LDS, no barriers): the next
// tile's ceil(b/4) 16-byte loads per lane are issued before the current tile is decoded (two register sets), every
// value is one bfe (or alignbit + and), a subtract and an unsigned compare, and matches accumulate per lane.
#include "reg_decode.h"

namespace ph {

// DS (ph_filter_execute): each lane also stores its run's 32-bit match mask, word t.w0 * 2 + lane of the segment's doc
// bitmap -- the wave's 64 lanes write 256 contiguous bytes
template <int C, int DS>
__global__ void __launch_bounds__(kBlock) k_count_reg(const KParams p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  constexpr int32_t TW = kRegTileWords;
  constexpr int32_t round_words = kWaves * TW;
  const int64_t nch = p.chunk_end - p.chunk_begin;
  int32_t c = p.chunk_begin + (int32_t)(nch * blockIdx.x / gridDim.x), r = 0;
  const int32_t c_end = p.chunk_begin + (int32_t)(nch * (blockIdx.x + 1) / gridDim.x);
  struct Tile {
    SegPtr S;
    int32_t w0, ndoc;
  };
  auto next_tile = [&]() {
    Tile t{nullptr, 0, 0};
    if (c < c_end) {
      const int32_t cbeg = chunks[c].word_begin, cend = chunks[c].word_end;
      t.S = segs + chunks[c].seg;
      t.w0 = cbeg + r * round_words + wave * TW;
      const int32_t nw = min(TW, cend - t.w0);
      t.ndoc = nw > 0 ? min(nw * 64, t.S->num_docs - t.w0 * 64) : 0;
      if (cbeg + (r + 1) * round_words < cend) {
        ++r;
      } else {
        ++c;
        r = 0;
      }
    }
    return t;
  };
  auto load = [&](const Tile& t, u32x4 (&pool)[C]) {
    const bool tile = t.ndoc > 0 && t.S->fkind == FK_RANGE;  // ALL / DOCRANGE tiles count without data
    const int fs = p.f_stream;
    reg_load<C>(tile, tile && lane * 32 < t.ndoc, tile ? t.S->streams[fs].fwd : nullptr,
                tile ? t.S->streams[fs].bits : 0,
                tile ? ((int64_t)t.S->num_docs * t.S->streams[fs].bits + 7) / 8 : 0, t.w0 * 2, lane, pool);
  };
  uint32_t cnt = 0;
  auto count = [&](const Tile& t, const u32x4 (&pool)[C]) {
    if (t.ndoc <= 0) return;
    const int32_t nv = max(0, min(32, t.ndoc - lane * 32));
    const uint32_t flo = t.S->flo, flen = t.S->flen;
    const int fk = t.S->fkind;
    if constexpr (DS) {
      uint32_t m = nv >= 32 ? 0xffffffffu : ((1u << nv) - 1u);
      if (fk == FK_RANGE) {
        uint32_t pass = 0;
        reg_decode<C>(pool, t.S->streams[p.f_stream].bits, [&](auto j, uint32_t v) {
          pass |= ((v - flo) < flen ? 1u : 0u) << decltype(j)::value;
        });
        m &= pass;
      } else if (fk == FK_DOCRANGE) {
        const int64_t d0 = (int64_t)t.w0 * 64 + lane * 32;
        const int64_t lo = max<int64_t>(0, (int64_t)flo - d0), hi = min<int64_t>(32, (int64_t)flo + flen - d0);
        uint32_t dm = 0;
        if (hi > lo) dm = (hi >= 32 ? 0xffffffffu : ((1u << hi) - 1u)) & ~(lo <= 0 ? 0u : ((1u << lo) - 1u));
        m &= dm;
      }
      cnt += (uint32_t)__builtin_popcount(m);
      if (nv > 0) t.S->docset[(int64_t)t.w0 * 2 + lane] = m;
      return;
    }
    if (fk == FK_RANGE) {
      reg_decode<C>(pool, t.S->streams[p.f_stream].bits, [&](auto j, uint32_t v) {
        cnt += ((v - flo) < flen && (int32_t)decltype(j)::value < nv) ? 1u : 0u;
      });
    } else if (fk == FK_DOCRANGE) {  // docs [d0, d0 + nv) inside [flo, flo + flen)
      const int64_t d0 = (int64_t)t.w0 * 64 + lane * 32;
      const int64_t lo = max<int64_t>(d0, flo), hi = min<int64_t>(d0 + nv, (int64_t)flo + flen);
      cnt += hi > lo ? (uint32_t)(hi - lo) : 0u;
    } else {
      cnt += (uint32_t)nv;
    }
  };
  u32x4 pa[C], pb[C];
  Tile ta = next_tile();
  load(ta, pa);
  while (ta.S != nullptr) {  // wave-uniform: a tile, the next one in flight while this one is counted
    Tile tb = next_tile();
    load(tb, pb);
    count(ta, pa);
    if (tb.S == nullptr) break;
    ta = next_tile();
    load(ta, pa);
    count(tb, pb);
  }
  const int64_t tot = wave_sum_i64((int64_t)cnt);
  if (lane == 0 && tot) atomicAdd(&p.out_count[0], (unsigned long long)tot);
}

void launch_count_reg(const KParams& p, int grid, hipStream_t s) {
  switch (p.count_reg) {
#define PH_COUNT_CASE(n)                                                                                     \
  case n:                                                                                                    \
    if (p.docset) hipLaunchKernelGGL((k_count_reg<n, 1>), dim3(grid), dim3(kBlock), 0, s, p);               \
    else hipLaunchKernelGGL((k_count_reg<n, 0>), dim3(grid), dim3(kBlock), 0, s, p);                        \
    break;
    PH_COUNT_CASE(1) PH_COUNT_CASE(2) PH_COUNT_CASE(3) PH_COUNT_CASE(4)
    PH_COUNT_CASE(5) PH_COUNT_CASE(6) PH_COUNT_CASE(7) default: PH_COUNT_CASE(8)
#undef PH_COUNT_CASE
  }
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph
