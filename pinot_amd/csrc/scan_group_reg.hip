// scan_group_reg.hip -- k_group_reg: the register-direct form of k_group_lds_lean (DefaultGroupByExecutor over a
// DictionaryBasedGroupKeyGenerator array holder, SURVEY 8(a10) / 8(a12): identity key remaps, at most one packed
// integer value column, ALL / RANGE / DOCRANGE filter leaves, a key space that fits LDS).
//
// Decode is reg_decode.h's: lane l of a wave owns 32 consecutive docs of a 2048-doc tile and holds each stream's
// b-bit values as b dwords, loaded one tile ahead with 16-byte buffer loads.  Per tile a lane folds the filter
// stream into a 32-bit match mask, the group streams into 32 keys, then walks the value stream issuing one LDS
// atomic per matched doc.
//
// The LDS table is LANE-INTERLEAVED: every key owns L (<= 32, a power of two) slots and lane l updates slot
// key * L + (l & (L - 1)).  With L = 32 the 64 lanes of one atomic hit 32 distinct bank pairs whatever their keys
// (lane l and l + 32 share one, which a 64-bit LDS op splits over two passes anyway), so the per-doc atomic runs
// conflict-free; the waves of a workgroup share the table through the atomics.  The L slots of a key are summed
// once at the end.  Slot state: COUNT << 40 | SUM of value offsets in one 64-bit word and the MIN, MAX offsets in a
// 32-bit pair; every doc of a tile issues its three atomics without a branch (missed docs go to a dummy row).
#include "reg_decode.h"

namespace ph {

template <int NG, int CF, int CG, int CV>
__global__ void __launch_bounds__(kBlock) k_group_reg(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  constexpr int32_t TW = kRegTileWords;
  constexpr int32_t round_words = kWaves * TW;
  const uint32_t G = (uint32_t)p.num_groups;
  const int lg = p.group_reg_lanes_log2;
  const uint32_t L = 1u << lg, GL = (G + 1) << lg;  // + the dummy row of missed docs
  unsigned long long* cs = reinterpret_cast<unsigned long long*>(smem);  // [(G + 1) * L] COUNT << 40 | SUM
  uint32_t* mm = reinterpret_cast<uint32_t*>(smem + (size_t)GL * 8);      // [(G + 1) * L][2] MIN, MAX offsets
  for (uint32_t i = threadIdx.x; i < GL; i += kBlock) {
    cs[i] = 0;
    mm[2 * i] = 0xffffffffu;
    mm[2 * i + 1] = 0u;
  }
  __syncthreads();
  const uint32_t lslot = (uint32_t)lane & (L - 1u);
  const int ops = CV ? p.val_ops[0] : 0;
  const bool want_min = (ops & OPS_MIN) != 0, want_max = (ops & OPS_MAX) != 0;
  uint32_t gstr[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) gstr[g] = (uint32_t)p.group_stride[g];

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
  struct Pool {
    u32x4 f[CF], g[NG][CG], v[CV > 0 ? CV : 1];
  };
  auto stream_bytes = [](SegPtr S, int s) { return ((int64_t)S->num_docs * S->streams[s].bits + 7) / 8; };
  auto load = [&](const Tile& t, Pool& pl) {
    const bool tile = t.ndoc > 0;
    const bool live = tile && lane * 32 < t.ndoc;
    const bool rng = tile && t.S->fkind == FK_RANGE;
    const int fs = p.f_stream;
    reg_load<CF>(rng, live, rng ? t.S->streams[fs].fwd : nullptr, rng ? t.S->streams[fs].bits : 0,
                 rng ? stream_bytes(t.S, fs) : 0, t.w0 * 2, lane, pl.f);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int gs = p.g_stream[g];
      reg_load<CG>(tile, live, tile ? t.S->streams[gs].fwd : nullptr, tile ? t.S->streams[gs].bits : 0,
                   tile ? stream_bytes(t.S, gs) : 0, t.w0 * 2, lane, pl.g[g]);
    }
    if constexpr (CV > 0) {
      const int vs = p.v_stream[0];
      reg_load<CV>(tile, live, tile ? t.S->streams[vs].fwd : nullptr, tile ? t.S->streams[vs].bits : 0,
                   tile ? stream_bytes(t.S, vs) : 0, t.w0 * 2, lane, pl.v);
    }
  };
  unsigned long long matched = 0;  // per lane
  // one register set of loads: a tile's streams are unpacked into the match mask, the 32 slot indices and the 32
  // value offsets, then the next tile's loads are issued and run under this tile's LDS atomics
  Pool pl;
  Tile t = next_tile();
  load(t, pl);
  while (t.S != nullptr) {  // wave-uniform
    const int32_t nv = max(0, min(32, t.ndoc - lane * 32));
    const uint32_t flo = t.S->flo, flen = t.S->flen;
    const int fk = t.S->fkind;
    uint32_t m = nv >= 32 ? 0xffffffffu : ((1u << nv) - 1u);  // docs of this lane's run that match
    uint32_t tmp[32];
    if (fk == FK_RANGE) {
      reg_unpack<CF>(pl.f, t.S->streams[p.f_stream].bits, tmp);
      uint32_t pass = 0;
#pragma unroll
      for (int j = 0; j < 32; ++j) pass |= ((tmp[j] - flo) < flen ? 1u : 0u) << j;
      m &= pass;
    } else if (fk == FK_DOCRANGE) {
      const int64_t d0 = (int64_t)t.w0 * 64 + lane * 32;
      const int64_t lo = max<int64_t>(0, (int64_t)flo - d0), hi = min<int64_t>(32, (int64_t)flo + flen - d0);
      uint32_t dm = 0;
      if (hi > lo) dm = (hi >= 32 ? 0xffffffffu : ((1u << hi) - 1u)) & ~(lo >= 32 ? 0xffffffffu : ((1u << lo) - 1u));
      m &= dm;
    }
    if (t.ndoc <= 0) m = 0;
    matched += (unsigned long long)__builtin_popcount(m);
    const bool any = __ballot(m != 0) != 0;
    uint32_t key[32];  // LDS slot of each doc: key * L + this lane's slot, or the dummy row's slot if it missed
    if (any) {
      reg_unpack<CG>(pl.g[0], t.S->streams[p.g_stream[0]].bits, key);
#pragma unroll
      for (int j = 0; j < 32; ++j) key[j] = __umul24(key[j], gstr[0]);
#pragma unroll
      for (int g = 1; g < NG; ++g) {
        reg_unpack<CG>(pl.g[g], t.S->streams[p.g_stream[g]].bits, tmp);
#pragma unroll
        for (int j = 0; j < 32; ++j) key[j] += __umul24(tmp[j], gstr[g]);
      }
#pragma unroll
      for (int j = 0; j < 32; ++j) key[j] = (((m >> j) & 1u) ? key[j] : G) << lg | lslot;
      if constexpr (CV > 0) {
        const uint32_t vadd = (uint32_t)(t.S->vals[0].base - p.part_vbase);
        reg_unpack<CV>(pl.v, t.S->streams[p.v_stream[0]].bits, tmp);
#pragma unroll
        for (int j = 0; j < 32; ++j) tmp[j] += vadd;
      }
    }
    t = next_tile();
    load(t, pl);
    // branch-free atomics: a missed doc updates the dummy row (key G), whose L slots are as conflict-free as any
    // key's, so no exec-mask juggling per doc; the atomics return nothing and never stall the wave
    if (any) {
      auto run = [&](auto mmode) {
        constexpr int MM = decltype(mmode)::value;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          const uint32_t slot = key[j];
          if constexpr (CV > 0) {
            const uint32_t vo = tmp[j];
            atomicAdd(&cs[slot], (1ull << 40) | (unsigned long long)vo);
            if constexpr (MM & 1) atomicMin(&mm[2 * slot], vo);
            if constexpr (MM & 2) atomicMax(&mm[2 * slot + 1], vo);
          } else {
            atomicAdd(&cs[slot], 1ull << 40);
          }
        }
      };
      const int mmode = (want_min ? 1 : 0) | (want_max ? 2 : 0);
      if (CV == 0 || mmode == 0) run(std::integral_constant<int, 0>{});
      else if (mmode == 1) run(std::integral_constant<int, 1>{});
      else if (mmode == 2) run(std::integral_constant<int, 2>{});
      else run(std::integral_constant<int, 3>{});
    }
  }
  const int64_t mt = wave_sum_i64((int64_t)matched);
  if (lane == 0 && mt && p.matched_total) atomicAdd(p.matched_total, (unsigned long long)mt);
  __syncthreads();
  // sum each key's L slots and add this workgroup's table into the dense result
  for (uint32_t k = threadIdx.x; k < G; k += kBlock) {
    unsigned long long n = 0, sum = 0;
    uint32_t vmin = 0xffffffffu, vmax = 0u;
    for (uint32_t s = 0; s < L; ++s) {
      const uint32_t i = (k << lg) | s;
      const unsigned long long x = cs[i];
      n += x >> 40;
      sum += x & ((1ull << 40) - 1ull);
      vmin = min(vmin, mm[2 * i]);
      vmax = max(vmax, mm[2 * i + 1]);
    }
    if (!n) continue;
    atomicAdd(&p.out_count[k], n);
    if (ops & OPS_SUM)
      atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum[0]) + k,
                (unsigned long long)((int64_t)sum + (int64_t)n * p.part_vbase));
    if (ops & OPS_MIN)
      atomicMin(reinterpret_cast<long long*>(p.out_min[0]) + k, (long long)(p.part_vbase + (int64_t)vmin));
    if (ops & OPS_MAX)
      atomicMax(reinterpret_cast<long long*>(p.out_max[0]) + k, (long long)(p.part_vbase + (int64_t)vmax));
  }
}

template <int NG, int CF, int CG>
static void launch_group_reg_v(const KParams& p, int grid, size_t lds, hipStream_t s) {
  switch (p.group_reg_cv) {
    case 0: hipLaunchKernelGGL((k_group_reg<NG, CF, CG, 0>), dim3(grid), dim3(kBlock), lds, s, p); break;
    case 4: hipLaunchKernelGGL((k_group_reg<NG, CF, CG, 4>), dim3(grid), dim3(kBlock), lds, s, p); break;
    default: hipLaunchKernelGGL((k_group_reg<NG, CF, CG, 8>), dim3(grid), dim3(kBlock), lds, s, p); break;
  }
}

template <int NG>
static void launch_group_reg_f(const KParams& p, int grid, size_t lds, hipStream_t s) {
  if (p.group_reg_cf <= 3) {
    if (p.group_reg_cg <= 2) launch_group_reg_v<NG, 3, 2>(p, grid, lds, s);
    else launch_group_reg_v<NG, 3, 4>(p, grid, lds, s);
  } else {
    if (p.group_reg_cg <= 2) launch_group_reg_v<NG, 8, 2>(p, grid, lds, s);
    else launch_group_reg_v<NG, 8, 4>(p, grid, lds, s);
  }
}

void launch_group_reg(const KParams& p, int ng, int grid, size_t lds, hipStream_t s) {
  // the host picks lds <= 40 KiB (four workgroups per CU): no dynamic-LDS attribute needed
  if (ng == 1) launch_group_reg_f<1>(p, grid, lds, s);
  else launch_group_reg_f<2>(p, grid, lds, s);
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph
