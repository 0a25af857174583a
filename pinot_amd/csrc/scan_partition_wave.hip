// scan_partition_wave.hip -- kernel A of the partitioned group-by with WAVE-PRIVATE partition rings (k_part_wave).
//
// k_part_reg shares one set of per-partition LDS rings among the four waves of a workgroup, so every 1024-doc half
// tile ends in a flush round and two workgroup barriers: measured on config 3 (1e9 rows, P = 245), the rounds alone
// cost 0.5 ms and the appends another 1.1 ms on top of the 1.2 ms the streaming and decode need.  Here every wave owns
// its rings: cnt[b] (records pending in partition b's ring) and ring[b][16] (one 64-byte chunk), so a rank is a
// returning LDS add that only the wave's own lanes contend on, and the wave flushes its own completed chunks right
// after its batch of appends -- LDS operations of one wave execute in order, so no barrier is ever needed:
//  * a batch = kWB records per lane (kWB x 64 docs): rank w = atomicAdd(cnt[b], 1); w < 16 stores the record at
//    ring[b][w], w == 15 lists b (the chunk is complete), w >= 16 defers the record;
//  * the flush moves each listed chunk with four lanes (one 16-byte LDS read + one 16-byte store each) to the
//    partition's region of the WORKGROUP at a position reserved with one LDS add on gpos[b] (shared by the
//    workgroup's waves, once per chunk, not per record), then cnt[b] -= 16;
//  * the deferred records (a partition that took more than its ring's room in one batch: rare) then store at
//    w - 16, possibly completing the next chunk, and the flush repeats until none is left.
// Regions and the per-region counts are k_part_reg's (kernel B is unchanged); the last chunks (< 16 records per
// partition per wave) are stored record by record at the end.  LDS per wave = P x (64 + 8) bytes.
#include "scan_partition.h"
#include "part_tiles.h"

#ifndef PH_WAVE_BATCH
#define PH_WAVE_BATCH 8
#endif

namespace ph {

template <int NG, int HASV, int CK, int CV>
__global__ void __launch_bounds__(kRegBlock) k_part_wave(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t P = (uint32_t)p.num_parts;
  constexpr uint32_t CH = 16;  // 32-bit records per 64-byte chunk
  // LDS: gpos[P] (workgroup), then per wave: ring[P][16], cnt[P], list[P]
  uint32_t* gpos = reinterpret_cast<uint32_t*>(smem);
  const uint32_t wstride = P * (CH + 2);
  uint32_t* ring = reinterpret_cast<uint32_t*>(smem) + ((P + 3) & ~3u) + (size_t)wave * wstride;
  uint32_t* cnt = ring + P * CH;
  uint32_t* list = cnt + P;
  for (uint32_t i = threadIdx.x; i < P; i += kRegBlock) gpos[i] = 0;
  for (uint32_t i = lane; i < P; i += 64) cnt[i] = 0;
  __syncthreads();
  const uint32_t cap = (uint32_t)p.part_cap;
  uint32_t* region0 = reinterpret_cast<uint32_t*>(p.part_buf) + (size_t)blockIdx.x * P * cap;
  unsigned long long matched = 0;

  // flush the nl listed chunks (list[0, nl)): 4 lanes per chunk, 16 chunks per pass
  auto flush = [&](uint32_t nl) {
    for (uint32_t base = 0; base < nl; base += 16) {
      const uint32_t i = base + ((uint32_t)lane >> 2), q = (uint32_t)lane & 3u;
      const bool live = i < nl;
      uint32_t b = 0, g = 0;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (live) {
        b = list[i];
        v = *reinterpret_cast<const u32x4*>(ring + b * CH + q * 4u);
        if (q == 0) {
          g = atomicAdd(&gpos[b], CH);
          atomicSub(&cnt[b], CH);
        }
      }
      // the chunk's region position from its quad's first lane
      g = __builtin_amdgcn_mov_dpp(g, 0x00, 0xf, 0xf, false);  // quad_perm [0, 0, 0, 0]
      if (live) {
        uint32_t* dst = region0 + (size_t)b * cap;
        const uint32_t d = g + q * 4u;
        if (g + CH <= cap) {
          *reinterpret_cast<u32x4*>(dst + d) = v;
        } else {  // region full (skewed keys): record by record, beyond the capacity to the overflow table
          part_store<0>(p, b, d + 0, v[0]);
          part_store<0>(p, b, d + 1, v[1]);
          part_store<0>(p, b, d + 2, v[2]);
          part_store<0>(p, b, d + 3, v[3]);
        }
      }
    }
  };

  PartTiles<NG, HASV, CK, CV> tiles(p, wave, blockIdx.x, gridDim.x);
  const int32_t nrounds = tiles.rounds();
  auto t0 = tiles.next();
  tiles.load(t0, lane);
  uint32_t X[32], PB[16];
  constexpr int kWB = PH_WAVE_BATCH;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int32_t it = 0; it < nrounds; ++it) {
    tiles.decode(t0, lane, X, PB);
    t0 = tiles.next();
    tiles.load(t0, lane);  // the next tile's loads stay in flight through the appends
    static_for<0, 32 / kWB>([&](auto u) {
      constexpr int j0 = decltype(u)::value * kWB;
      uint32_t w[kWB];
      uint32_t nl = 0;  // listed chunks (wave-uniform)
      bool defer = false;
      static_for<0, kWB>([&](auto qq) {
        constexpr int J = j0 + decltype(qq)::value;
        const uint32_t b = part_of<J>(PB);
        w[qq] = 0xffffffffu;
        if (b < P) w[qq] = atomicAdd(&cnt[b], 1u);
      });
      static_for<0, kWB>([&](auto qq) {
        constexpr int J = j0 + decltype(qq)::value;
        const uint32_t b = part_of<J>(PB);
        const bool h = b < P;
        if (h && w[qq] < CH) ring[b * CH + w[qq]] = X[J];
        const unsigned long long full = __ballot(h && w[qq] == CH - 1u);
        if (h && w[qq] == CH - 1u) list[nl + (uint32_t)__popcll(full & below)] = b;
        nl += (uint32_t)__popcll(full);
        defer |= h && w[qq] >= CH && w[qq] != 0xffffffffu;
        matched += (unsigned long long)__popcll(__ballot(h));
      });
      flush(nl);
      // deferred records: ranks past the ring's chunk, stored once the chunk before them has left
      while (__ballot(defer)) {
        nl = 0;
        bool again = false;
        static_for<0, kWB>([&](auto qq) {
          constexpr int J = j0 + decltype(qq)::value;
          const uint32_t b = part_of<J>(PB);
          const bool d = b < P && w[qq] >= CH && w[qq] != 0xffffffffu;
          if (d) w[qq] -= CH;
          if (d && w[qq] < CH) ring[b * CH + w[qq]] = X[J];
          const unsigned long long full = __ballot(d && w[qq] == CH - 1u);
          if (d && w[qq] == CH - 1u) list[nl + (uint32_t)__popcll(full & below)] = b;
          nl += (uint32_t)__popcll(full);
          again |= d && w[qq] >= CH;
        });
        flush(nl);
        defer = again;
      }
    });
  }
  // the last partial chunks of this wave's rings
  for (uint32_t b = lane; b < P; b += 64) {
    const uint32_t n = cnt[b];
    if (n) {
      const uint32_t g = atomicAdd(&gpos[b], n);
      for (uint32_t i = 0; i < n; ++i) part_store<0>(p, b, g + i, ring[b * CH + i]);
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < P; b += kRegBlock)
    p.part_count[(size_t)b * gridDim.x + blockIdx.x] = gpos[b];  // records of region (b, blockIdx), may exceed cap
  if (lane == 0 && matched && p.matched_total) atomicAdd(p.matched_total, matched);
}

size_t part_wave_lds_bytes(int32_t num_parts) {
  const size_t P = (size_t)num_parts;
  return 4 * (((P + 3) & ~(size_t)3) + (size_t)kRegWaves * P * 18);
}

template <int NG, int HASV, int CK, int CV>
static const void* wave_fn() {
  return (const void*)k_part_wave<NG, HASV, CK, CV>;
}

template <int NG>
static const void* wave_fn_ng(const KParams& p) {
  const bool hasv = p.num_vals > 0;
  if (p.part_ck == 3) return hasv ? wave_fn<NG, 1, 3, 5>() : wave_fn<NG, 0, 3, 5>();
  return hasv ? wave_fn<NG, 1, 4, 8>() : wave_fn<NG, 0, 4, 8>();
}

static const void* part_wave_fn(const KParams& p, int ng) {
  return ng == 1 ? wave_fn_ng<1>(p) : (ng == 2 ? wave_fn_ng<2>(p) : wave_fn_ng<3>(p));
}

void launch_part_wave(const KParams& p, int ng, int grid, size_t lds, hipStream_t s) {
  const void* f = part_wave_fn(p, ng);
  if (lds > 64 * 1024) PH_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* args[] = {const_cast<KParams*>(&p)};
  PH_HIP_CHECK(hipLaunchKernel(f, dim3(grid), dim3(kRegBlock), args, lds, s));
}

int part_wave_blocks_per_cu(const KParams& p, int ng, size_t lds) {
  const void* f = part_wave_fn(p, ng);
  if (lds > 64 * 1024) PH_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int n = 0;
  PH_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, kRegBlock, lds));
  return std::max(1, n);
}

}  // namespace ph
