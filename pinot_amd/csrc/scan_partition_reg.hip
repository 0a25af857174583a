// scan_partition_reg.hip -- kernel A of the partitioned group-by in its register-direct form (k_part_reg); kernel B
// and the LDS-staged forms are in scan_partition.hip.
#include "scan_partition.h"
#include "part_tiles.h"

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
  uint32_t* pend = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  uint32_t* lists = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off);  // [2][P] listed partitions
  uint32_t* lcnt = lists + 2 * p.num_parts;                            // [2] list lengths
  uint32_t* slots = reinterpret_cast<uint32_t*>(smem + p.pl_slot_off);
  {
    uint32_t* gpos = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
    for (int i = threadIdx.x; i < p.num_parts + 64; i += kRegBlock) pend[i] = 0;
    for (int i = threadIdx.x; i < p.num_parts; i += kRegBlock) gpos[i] = 0;
    if (threadIdx.x < 2) lcnt[threadIdx.x] = 0;
  }
  __syncthreads();
  uint32_t par = 0;
  unsigned long long matched = 0;
  PartTiles<NG, HASV, CK, CV> tiles(p, wave, blockIdx.x, gridDim.x);
  const int32_t nrounds = tiles.rounds();
  const uint32_t P = (uint32_t)p.num_parts;
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  constexpr uint32_t CH = 16;  // 32-bit records per 64-byte chunk
  constexpr int kAB = PH_PART_AB;  // records per lane whose rank atomics are in flight together
  const int halves = p.part_rounds == 2 ? 2 : 1;
  const bool swz = (p.part_variant & 1) != 0, masked = (p.part_variant & 2) != 0;
  const uint32_t dummy_word = P + (uint32_t)lane;           // scratch word / slot of a record-less lane
  const uint32_t dummy_slot = (P << cl) + (uint32_t)lane;
  auto t0 = tiles.next();
  tiles.load(t0, lane);
  // per lane and doc j of the tile: X[j] = the 32-bit record ((key & kmask) << vbits | value offset); PB packs two
  // 16-bit partition indices per register (0xffff: a missed or out-of-range doc), so the append state between the
  // decode and the rounds is 48 registers, not 64
  uint32_t X[32], PB[16];
  for (int32_t it = 0; it < nrounds; ++it) {
    tiles.decode(t0, lane, X, PB);
    // timing experiments (PH_PART_DBG; results invalid): 2 = no appends, 8 = no append rounds at all
    const int dbg = p.part_dbg;
    if (dbg & 2) static_for<0, 16>([&](auto j) { PB[j] = 0xffffffffu; });
    // ---- the next tile's loads stay in flight through the append rounds
    t0 = tiles.next();
    tiles.load(t0, lane);
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
          bk[q] = part_of<J>(PB);
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
