// scan_partition_reg.hip -- kernel A of the partitioned group-by in its register-direct form (k_part_reg); kernel B
// and the LDS-staged forms are in scan_partition.hip.
#include "scan_partition.h"
#include "reg_decode.h"

#ifndef PH_PART_AB
#define PH_PART_AB 4
#endif

namespace ph {

// ------------------------------------------------------------------ kernel A, register-direct form (k_part_reg)
// The LDS-staged forms above stage every stream through LDS and decode each value with a ds_read2 (4 streams x 64
// docs = 16+ LDS cycles per word, ~35 VALU per word): at config 3 they are LDS- and issue-bound at 2.6 TB/s.  Here
// lane l of a wave owns the 32 CONSECUTIVE docs [32 l, 32 l + 32) of a 2048-doc tile, so its b-bit values of any
// stream are exactly b whole dwords at byte (tile run + l) * 4b -- read straight into registers with 16-byte buffer
// loads (ceil(b / 4) per stream per lane), byte-swapped once, and decoded with compile-time bit positions (one bfe,
// or one alignbit + and, per value) by a switch over the segment's width.  No staging LDS, no per-value LDS read:
// the LDS holds only the partition rings.  The next tile's loads are issued right after the decode and stay in
// flight through the append rounds.  Phases: keys (mixed radix), value offset, then the filter, which turns a
// missed or out-of-range doc's key into ~0u (partition index >= P: the append goes to the lane's scratch word).
template <int NG, int HASV, int CK, int CV>
__global__ void __launch_bounds__(kRegBlock) k_part_reg(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  uint32_t* pend = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  uint32_t* gpos = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
  uint32_t* lists = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off);  // [2][P] listed partitions
  uint32_t* lcnt = lists + 2 * p.num_parts;                            // [2] list lengths
  uint32_t* slots = reinterpret_cast<uint32_t*>(smem + p.pl_slot_off);
  for (int i = threadIdx.x; i < p.num_parts + 64; i += kRegBlock) pend[i] = 0;
  for (int i = threadIdx.x; i < p.num_parts; i += kRegBlock) gpos[i] = 0;
  if (threadIdx.x < 2) lcnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t par = 0;
  unsigned long long matched = 0;
  constexpr int32_t TW = kRegTileWords;
  constexpr int32_t round_words = kRegWaves * TW;
  const int64_t nch = p.chunk_end - p.chunk_begin;
  const int32_t c0 = p.chunk_begin + (int32_t)(nch * blockIdx.x / gridDim.x);
  int32_t c = c0, r = 0;
  const int32_t c_end = p.chunk_begin + (int32_t)(nch * (blockIdx.x + 1) / gridDim.x);
  struct Tile {
    SegPtr S;
    int32_t w0, ndoc;  // first word; docs of this tile the wave owns (<= 2048, clipped to the segment)
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
  u32x4 pf[CK], pk[NG][CK], pv[HASV ? CV : 1];
  auto load = [&](const Tile& t) {
    const bool tile = t.ndoc > 0;                        // wave-uniform
    const bool lane_live = tile && lane * 32 < t.ndoc;  // this lane's run holds docs of the tile
    const int32_t run0 = t.w0 * 2;
    SegPtr S = t.S;
    auto bytes = [&](int st) { return ((int64_t)S->num_docs * S->streams[st].bits + 7) / 8; };
    const bool rng = tile && S->fkind == FK_RANGE;
    const int fs = p.f_stream;
    reg_load<CK>(rng, lane_live, rng ? S->streams[fs].fwd : nullptr, rng ? S->streams[fs].bits : 0,
                 rng ? bytes(fs) : 0, run0, lane, pf);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int gs = p.g_stream[g];
      reg_load<CK>(tile, lane_live, tile ? S->streams[gs].fwd : nullptr, tile ? S->streams[gs].bits : 0,
                   tile ? bytes(gs) : 0, run0, lane, pk[g]);
    }
    if constexpr (HASV != 0) {
      const int vs = p.v_stream[0];
      reg_load<CV>(tile, lane_live, tile ? S->streams[vs].fwd : nullptr, tile ? S->streams[vs].bits : 0,
                   tile ? bytes(vs) : 0, run0, lane, pv);
    }
  };
  int32_t nrounds = 0;
  for (int32_t cc = c0; cc < c_end; ++cc) {
    const int32_t words = chunks[cc].word_end - chunks[cc].word_begin;
    nrounds += (words + round_words - 1) / round_words;
  }
  const uint32_t klo = (uint32_t)p.part_klo, kmask = (1u << klo) - 1u, vbits = (uint32_t)p.part_vbits;
  const uint32_t P = (uint32_t)p.num_parts;
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  constexpr uint32_t CH = 16;  // 32-bit records per 64-byte chunk
  constexpr int kAB = PH_PART_AB;  // records per lane whose rank atomics are in flight together
  const int halves = p.part_rounds == 2 ? 2 : 1;
  const bool swz = (p.part_variant & 1) != 0, masked = (p.part_variant & 2) != 0;
  const uint32_t dummy_word = P + (uint32_t)lane;           // scratch word / slot of a record-less lane
  const uint32_t dummy_slot = (P << cl) + (uint32_t)lane;
  Tile t0 = next_tile();
  load(t0);
  // per lane and doc j of the tile: X[j] = the 32-bit record ((key & kmask) << vbits | value offset); PB packs two
  // 16-bit partition indices per register (0xffff: a missed or out-of-range doc), so the append state between the
  // decode and the rounds is 48 registers, not 64
  uint32_t X[32], PB[16];
  for (int32_t it = 0; it < nrounds; ++it) {
    // ---- decode the tile (registers only): keys into X, then the filter reads the partition indices off them,
    // then the value phase turns each key into its record in place (peak: 48 registers + the loads)
    const int32_t nv = t0.ndoc > 0 ? max(0, min(32, t0.ndoc - lane * 32)) : 0;  // this lane's valid docs
    if (t0.ndoc > 0) {
      SegPtr S = t0.S;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const uint32_t st = (uint32_t)p.group_stride[g];
        if (g == 0) reg_decode<CK>(pk[g], S->streams[p.g_stream[g]].bits, [&](auto j, uint32_t v) { X[j] = __umul24(v, st); });
        else reg_decode<CK>(pk[g], S->streams[p.g_stream[g]].bits, [&](auto j, uint32_t v) { X[j] += __umul24(v, st); });
      }
      // filter + doc validity -> the partition index (0xffff: no record)
      auto put = [&](auto j, bool pass) {
        constexpr int J = decltype(j)::value;
        const uint32_t b = pass && J < nv ? (X[J] >> klo) : 0xffffu;
        if constexpr ((J & 1) == 0) PB[J >> 1] = b;
        else PB[J >> 1] |= b << 16;
      };
      const int fk = S->fkind;
      const uint32_t flo = S->flo, flen = S->flen;
      if (fk == FK_RANGE) {
        reg_decode<CK>(pf, S->streams[p.f_stream].bits, [&](auto j, uint32_t v) { put(j, (v - flo) < flen); });
      } else if (fk == FK_DOCRANGE) {
        const uint32_t d0 = (uint32_t)t0.w0 * 64u + (uint32_t)lane * 32u;
        static_for<0, 32>([&](auto j) { put(j, (d0 + (uint32_t)decltype(j)::value - flo) < flen); });
      } else {
        static_for<0, 32>([&](auto j) { put(j, true); });
      }
      if constexpr (HASV != 0) {
        const uint32_t vadd = (uint32_t)(S->vals[0].base - p.part_vbase);
        reg_decode<CV>(pv, S->streams[p.v_stream[0]].bits,
                       [&](auto j, uint32_t v) { X[j] = ((X[j] & kmask) << vbits) | (v + vadd); });
      } else {
        static_for<0, 32>([&](auto j) { X[j] &= kmask; });
      }
    } else {
      static_for<0, 16>([&](auto j) { PB[j] = 0xffffffffu; });
    }
    // timing experiments (PH_PART_DBG; results invalid): 2 = no appends, 8 = no append rounds at all
    const int dbg = p.part_dbg;
    if (dbg & 2) static_for<0, 16>([&](auto j) { PB[j] = 0xffffffffu; });
    // ---- the next tile's loads stay in flight through the append rounds
    t0 = next_tile();
    load(t0);
    if (dbg & 8) {
      unsigned long long x = 0;
      static_for<0, 16>([&](auto j) { x += PB[j] ^ X[2 * j] ^ X[2 * j + 1]; });
      if (x == 0x5bd1e9955bd1e995ull) matched += 1;  // keeps the decode alive
      continue;
    }
    // ---- append rounds: flush the chunks the previous round completed, then append this round's records
    auto append_round = [&](auto jb, auto je) {
      {
        const uint32_t prev = par ^ 1u;
        const uint32_t nl = lcnt[prev];
        if (threadIdx.x == 0) lcnt[par] = 0;
        part_flush_listed<0, kRegBlock, 1>(p, smem, lists + prev * P, nl, matched);
      }
      lds_barrier();
      uint32_t* fl = lists + par * P;
      uint32_t* fc = lcnt + par;
      static_for<decltype(jb)::value / kAB, decltype(je)::value / kAB>([&](auto u) {
        constexpr int j0 = decltype(u)::value * kAB;
        uint32_t bk[kAB], w[kAB], rec[kAB];
        static_for<0, kAB>([&](auto q) {
          constexpr int J = j0 + decltype(q)::value;
          bk[q] = (J & 1) ? (PB[J >> 1] >> 16) : (PB[J >> 1] & 0xffffu);
          rec[q] = X[J];
        });
        // append form (part_variant): record-less lanes either exec-masked (bit 1: no LDS operation) or sent to their
        // lane's scratch word / slot (branch-free); ring quarters XOR-swizzled by partition (bit 0) or not
        bool ovf = false, full = false;
        if (masked) {
          static_for<0, kAB>([&](auto q) {
            w[q] = C;
            if (bk[q] < P) w[q] = atomicAdd(&pend[bk[q]], 1u);
          });
          static_for<0, kAB>([&](auto q) {
            const bool h = bk[q] < P;
            ovf |= h & (w[q] >= C);
            full |= h & (w[q] == CH - 1u);
            if (h & (w[q] < C)) slots[(bk[q] << cl) + (w[q] ^ (swz ? ring_swizzle(bk[q], C) : 0u))] = rec[q];
          });
        } else {
          static_for<0, kAB>([&](auto q) { w[q] = atomicAdd(&pend[min(bk[q], dummy_word)], 1u); });
          static_for<0, kAB>([&](auto q) {
            const bool h = bk[q] < P;
            const bool ok = h & (w[q] < C);
            ovf |= h & (w[q] >= C);
            full |= h & (w[q] == CH - 1u);
            slots[ok ? (bk[q] << cl) + (w[q] ^ (swz ? ring_swizzle(bk[q], C) : 0u)) : dummy_slot] = rec[q];
          });
        }
        if (__ballot(full)) {
          static_for<0, kAB>([&](auto q) {
            if (bk[q] < P && w[q] == CH - 1u) fl[atomicAdd(fc, 1u)] = bk[q];
          });
        }
        if (__ballot(ovf)) {
          static_for<0, kAB>([&](auto q) {
            if (bk[q] < P && w[q] >= C) part_overflow<0>(p, bk[q], rec[q]);
          });
        }
      });
      lds_barrier();
      par ^= 1u;
    };
    if (halves == 2) {
      append_round(std::integral_constant<int, 0>{}, std::integral_constant<int, 16>{});
      append_round(std::integral_constant<int, 16>{}, std::integral_constant<int, 32>{});
    } else {
      append_round(std::integral_constant<int, 0>{}, std::integral_constant<int, 32>{});
    }
  }
  part_flush_listed<0, kRegBlock, 1>(p, smem, lists + (par ^ 1u) * P, lcnt[par ^ 1u], matched);
  lds_barrier();
  part_flush_final<0, kRegBlock, 1>(p, smem, matched);
  if (matched && p.matched_total) atomicAdd(p.matched_total, matched);
}

template <int NG, int HASV, int CK, int CV>
static void launch_part_reg_k(const KParams& p, int grid, size_t lds, hipStream_t s) {
  allow_lds(k_part_reg<NG, HASV, CK, CV>, lds);
  hipLaunchKernelGGL((k_part_reg<NG, HASV, CK, CV>), dim3(grid), dim3(kRegBlock), lds, s, p);
}

template <int NG>
static void launch_part_reg_ng(const KParams& p, int grid, size_t lds, hipStream_t s) {
  const bool hasv = p.num_vals > 0;
  if (p.part_ck == 3) {
    if (hasv) launch_part_reg_k<NG, 1, 3, 5>(p, grid, lds, s);
    else launch_part_reg_k<NG, 0, 3, 5>(p, grid, lds, s);
  } else {
    if (hasv) launch_part_reg_k<NG, 1, 4, 8>(p, grid, lds, s);
    else launch_part_reg_k<NG, 0, 4, 8>(p, grid, lds, s);
  }
}

void launch_part_reg(const KParams& p, int ng, int grid, size_t lds, hipStream_t s) {
  switch (ng) {
    case 1: launch_part_reg_ng<1>(p, grid, lds, s); break;
    case 2: launch_part_reg_ng<2>(p, grid, lds, s); break;
    default: launch_part_reg_ng<3>(p, grid, lds, s); break;
  }
}

// resident k_part_reg workgroups per CU at `lds` bytes of dynamic LDS (registers bound it, not only the LDS)
int part_reg_blocks_per_cu(const KParams& p, int ng, size_t lds) {
  const void* f = nullptr;
  const bool hasv = p.num_vals > 0;
#define PH_REG_FN(NG)                                                                                                 \
  f = p.part_ck == 3 ? (hasv ? (const void*)k_part_reg<NG, 1, 3, 5> : (const void*)k_part_reg<NG, 0, 3, 5>)          \
                     : (hasv ? (const void*)k_part_reg<NG, 1, 4, 8> : (const void*)k_part_reg<NG, 0, 4, 8>);
  if (ng == 1) { PH_REG_FN(1) } else if (ng == 2) { PH_REG_FN(2) } else { PH_REG_FN(3) }
#undef PH_REG_FN
  if (lds > 64 * 1024) PH_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int n = 0;
  PH_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, kRegBlock, lds));
  return std::max(1, n);
}

}  // namespace ph
