// scan_partition_reg.hip -- kernel A of the partitioned group-by in its register-direct form (k_part_reg); kernel B
// and the LDS-staged forms are in scan_partition.hip.
#include <map>
#include <mutex>
#include <tuple>

#include "scan_partition.h"
#include "part_tiles.h"

namespace ph {

// records whose ring-rank atomics issue back to back before their stores (the stores need the ranks)
constexpr int kAppendGroup = 8;

// ------------------------------------------------------------------ kernel A, register-direct form (k_part_reg)
// The LDS-staged forms (scan_partition.hip) stage every stream through LDS and decode each value with a ds_read2
// (4 streams x 64 docs = 16+ LDS cycles per word, ~35 VALU per word): at config 3 they are LDS- and issue-bound at
// 2.6 TB/s.  Here lane l of a wave owns the 32 CONSECUTIVE docs [32 l, 32 l + 32) of a 2048-doc tile, so its b-bit
// values of any stream are exactly b whole dwords at byte (tile run + l) * 4b -- read straight into registers with
// 16-byte buffer loads (ceil(b / 4) per stream per lane), byte-swapped once, and decoded with compile-time bit
// positions (one bfe, or one alignbit + and, per value) by a switch over the segment's width.  No staging LDS, no
// per-value LDS read: the LDS holds only the partition rings.  The next tile's loads are issued right after the
// decode and stay in flight through the two append rounds.
//
// An append is straight-line per record: one returning LDS add on the record's ring word (the partition's pending
// count, or the lane's scratch word for a missed doc -- PartTiles::decode already chose it), one compare, one store
// (a missed doc's or a full ring's record to the lane's scratch slot).  r4 SQ counters on the previous form (runtime
// append variants, listed flush with per-record "chunk completed" checks): 64.5 VALU + 33 SALU per doc and the VALU
// busy 62 % of the kernel.  The flush is one thread per partition (part_flush_owner: pending >= 16 sends its whole
// 64-byte chunks out), so no append keeps a list.
// SETS: ring sets.  2 -- a round appends to one set while the owner threads send out the whole chunks the previous
// round completed in the other (one barrier per round); 1 -- flush, barrier, append, barrier (half the LDS: at
// config 3's 245 partitions the two sets' 76 KB hold kernel A at 2 workgroups per CU, one set's 41 KB allow the 3 its
// registers allow)
template <int NG, int HASV, int CK, int CV, int SETS>
__global__ void __launch_bounds__(kRegBlock) k_part_reg(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* pend = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  uint32_t* const pend0 = pend;
  uint32_t* const slots0 = reinterpret_cast<uint32_t*>(smem + p.pl_slot_off);
  const size_t SW = (size_t)p.part_set_words;
  uint32_t round = 0;
  {
    uint32_t* gpos = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
    // the lanes' scratch words start at 2^31 + 64: a scratch rank is then negative as an int, so the overflow test
    // below (0 <= rank - C as an int) never fires for a missed doc, without a per-record partition compare
    for (int i = threadIdx.x; i < SETS * (p.num_parts + 64); i += kRegBlock)
      pend[i] = (i % (p.num_parts + 64)) < p.num_parts ? 0u : 0x80000040u;
    for (int i = threadIdx.x; i < p.num_parts; i += kRegBlock) gpos[i] = 0;
  }
  __syncthreads();
  unsigned long long matched = 0;
  PartTiles<NG, HASV, CK, CV> tiles(p, wave, blockIdx.x, gridDim.x);
  const int32_t nrounds = tiles.rounds();
  const uint32_t P = (uint32_t)p.num_parts;
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  const uint32_t RS = (uint32_t)p.part_ring_stride;
  const uint32_t dummy_slot = P * RS + (uint32_t)lane;  // scratch slot of a record-less lane
  auto t0 = tiles.next();
  tiles.load(t0, lane);
  // per lane and doc j of the tile: X[j] = the 32-bit record; PB packs two 16-bit ring-word indices per register
  uint32_t X[32], PB[16];
  for (int32_t it = 0; it < nrounds; ++it) {
    tiles.decode(t0, lane, X, PB);
    // ---- the next tile's loads stay in flight through the append rounds
    t0 = tiles.next();
    tiles.load(t0, lane);
    // ---- two append rounds of 16 records per lane each
    auto append_round = [&](auto jb) {
      const int cur = SETS == 2 ? (int)(round & 1) : 0;
      if constexpr (SETS == 2) {
        if (round > 0) part_flush_owner<kRegBlock>(p, smem, matched, false, cur ^ 1);
      } else {
        if (round > 0) {  // the previous round's appends are complete (its barrier): flush, then append after a barrier
          part_flush_owner<kRegBlock>(p, smem, matched, false, 0);
          lds_barrier();
        }
      }
      uint32_t* pend = pend0 + (size_t)cur * (P + 64);
      uint32_t* slots = slots0 + (size_t)cur * SW;
      // groups of kAppendGroup: the group's rank atomics issue back to back, then its stores.  Branch-free and SGPR-free per record:
      // slot = min(b * RS + min(rank, C), scratch slot) -- a real partition's ring slot (rank C: the ring's padding
      // quarter, for a record that overflows), a missed doc's scratch slot; a full ring (skewed round) shows as
      // 0 <= (int)(rank - C) (scratch ranks are negative), ORed over the group into one sign test
      static_for<0, 16 / kAppendGroup>([&](auto u) {
        constexpr int J0 = decltype(jb)::value + kAppendGroup * decltype(u)::value;
        uint32_t b[kAppendGroup], w[kAppendGroup];
        static_for<0, kAppendGroup>([&](auto q) {
          b[q] = part_of<J0 + decltype(q)::value>(PB);
          w[q] = atomicAdd(&pend[b[q]], 1u);
        });
        uint32_t neg = 0xffffffffu;  // bit 31 stays set while no record overflowed
        static_for<0, kAppendGroup>([&](auto q) {
          neg &= w[q] - C;
          slots[min(__umul24(b[q], RS) + min(w[q], C), dummy_slot)] = X[J0 + decltype(q)::value];
        });
        if (__builtin_expect(__ballot((int32_t)neg >= 0) != 0ull, 0)) {
          static_for<0, kAppendGroup>([&](auto q) {
            if ((int32_t)(w[q] - C) >= 0) part_overflow<0>(p, b[q], X[J0 + decltype(q)::value]);
          });
        }
      });
      lds_barrier();
      ++round;
    };
    append_round(std::integral_constant<int, 0>{});
    append_round(std::integral_constant<int, 16>{});
  }
  if constexpr (SETS == 2) {
    // the last round's set still holds its whole chunks; every pending record of both sets then goes out (one owner
    // thread per partition writes both sets' leftovers, then the region count)
    if (round > 0) part_flush_owner<kRegBlock>(p, smem, matched, false, (int)((round - 1) & 1));
    lds_barrier();
    part_flush_owner<kRegBlock>(p, smem, matched, true, (int)(round & 1), false);
    part_flush_owner<kRegBlock>(p, smem, matched, true, (int)((round - 1) & 1), true);
  } else {
    part_flush_owner<kRegBlock>(p, smem, matched, true, 0, true);  // (the last round ended at a barrier)
  }
  if (matched && p.matched_total) atomicAdd(p.matched_total, matched);
}

template <int NG, int HASV, int CK, int CV>
static void launch_part_reg_k(const KParams& p, int grid, size_t lds, hipStream_t s) {
  if (p.part_sets == 1) {
    allow_lds(k_part_reg<NG, HASV, CK, CV, 1>, lds);
    hipLaunchKernelGGL((k_part_reg<NG, HASV, CK, CV, 1>), dim3(grid), dim3(kRegBlock), lds, s, p);
  } else {
    allow_lds(k_part_reg<NG, HASV, CK, CV, 2>, lds);
    hipLaunchKernelGGL((k_part_reg<NG, HASV, CK, CV, 2>), dim3(grid), dim3(kRegBlock), lds, s, p);
  }
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
#define PH_REG_FX(NG, FX)                                                                                             \
  f = p.part_ck == 3 ? (hasv ? (const void*)k_part_reg<NG, 1, 3, 5, FX> : (const void*)k_part_reg<NG, 0, 3, 5, FX>)  \
                     : (hasv ? (const void*)k_part_reg<NG, 1, 4, 8, FX> : (const void*)k_part_reg<NG, 0, 4, 8, FX>);
#define PH_REG_FN(NG)     \
  if (p.part_sets == 1) { \
    PH_REG_FX(NG, 1)      \
  } else {                \
    PH_REG_FX(NG, 2)      \
  }
  if (ng == 1) { PH_REG_FN(1) } else if (ng == 2) { PH_REG_FN(2) } else { PH_REG_FN(3) }
#undef PH_REG_FN
#undef PH_REG_FX
  // (the occupancy query and the attribute call cost tens of microseconds of host time per query: cached per
  // (kernel, LDS bytes, device))
  static std::mutex mu;
  static std::map<std::tuple<const void*, size_t, int>, int> cache;
  int dev = 0;
  PH_HIP_CHECK(hipGetDevice(&dev));
  const auto key = std::make_tuple(f, lds, dev);
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  if (lds > 64 * 1024) PH_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int n = 0;
  PH_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, kRegBlock, lds));
  n = std::max(1, n);
  std::lock_guard<std::mutex> lk(mu);
  cache[key] = n;
  return n;
}

}  // namespace ph
