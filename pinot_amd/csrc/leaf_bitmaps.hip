// leaf_bitmaps.hip -- k_leaf_bitmaps: the doc bitmap of one dictId scan leaf (a RANGE [lo, lo + len) or a dictId set)
// per job, in the register-direct form of reg_decode.h: lane l of a wave owns the 32 consecutive docs [32 l, 32 l + 32)
// of a 2048-doc tile, decodes them with compile-time bit positions and writes their match bits as ONE 32-bit word --
// two lanes form the 64-doc word of the bitmap (doc d at bit d & 63 of word d >> 6), so the stores are coalesced.
// What the filter-statistic pass needs of the scan leaves (query.cpp: the leapfrog of ANDs of scans,
// k_scan_and_entries, and the host iterator simulation); HBM-bound like k_count_reg, against the generic per-doc
// program evaluation of k_filter_bitmaps.
#include "reg_decode.h"

namespace ph {

// G tiles per wave per batch (8 / C: the same registers whatever the width), the next batch's loads in flight while
// this one is tested; the set (if any) in dynamic LDS sized by the launch
template <int C, int G>
__global__ void __launch_bounds__(256) k_leaf_bitmaps(const LeafJob* __restrict__ jobs) {
  extern __shared__ uint32_t set_lds[];
  const LeafJob J = jobs[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const bool use_set = J.set != nullptr;
  if (use_set) {  // the dictId set, staged once per workgroup
    for (int i = threadIdx.x; i < J.set_words; i += 256) set_lds[i] = J.set[i];
    __syncthreads();
  }
  const int64_t ntiles = (J.ndocs + 2047) / 2048;
  const int64_t bytes = (J.ndocs * J.bits + 7) / 8;
  const int64_t stride = (int64_t)gridDim.x * 4 * G;  // tiles between a wave's batches
  auto load = [&](int64_t t0, u32x4 (&pool)[G][C]) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t t = t0 + g;
      const int32_t ndoc = t < ntiles ? (int32_t)min<int64_t>(2048, J.ndocs - t * 2048) : 0;
      reg_load<C>(t < ntiles, lane * 32 < ndoc, J.fwd, J.bits, bytes, (int32_t)((t * 2048) >> 5), lane, pool[g]);
    }
  };
  int64_t t0 = ((int64_t)blockIdx.x * 4 + wave) * G;
  u32x4 cur[G][C];
  load(t0, cur);
  for (; t0 < ntiles; t0 += stride) {
    u32x4 nxt[G][C];
    load(t0 + stride, nxt);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int64_t tile = t0 + g;
      if (tile >= ntiles) break;
      const int64_t d0 = tile * 2048;
      const int32_t ndoc = (int32_t)min<int64_t>(2048, J.ndocs - d0);
      const int32_t nv = max(0, min(32, ndoc - lane * 32));
      uint32_t v[32];
      reg_unpack<C>(cur[g], J.bits, v);
      uint32_t mask = 0;
      if (use_set) {
#pragma unroll
        for (int j = 0; j < 32; ++j)
          mask |= (v[j] < (uint32_t)J.card && ((set_lds[v[j] >> 5] >> (v[j] & 31)) & 1u) ? 1u : 0u) << j;
      } else {
#pragma unroll
        for (int j = 0; j < 32; ++j) mask |= ((v[j] - J.lo) < J.len ? 1u : 0u) << j;
      }
      if (nv < 32) mask &= nv > 0 ? (0xffffffffu >> (32 - nv)) : 0u;
      const int64_t wi = (d0 >> 5) + lane;  // this lane's 32-doc word (lanes past the end write the zero padding)
      if (wi < J.out_words) J.out[wi] = mask;
    }
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < C; ++i) cur[g][i] = nxt[g][i];
  }
}

void launch_leaf_bitmaps(const LeafJob* jobs, int32_t njobs, int64_t max_docs, int32_t max_bits, int32_t set_words,
                         hipStream_t s) {
  if (njobs <= 0 || max_docs <= 0) return;
  const int64_t tiles = (max_docs + 2047) / 2048;
  const size_t lds = (size_t)std::max(0, set_words) * 4;
  // ~8 tiles per wave, one tile of look-ahead (r4 on the SSB flight: one tile per wave 0.39 ms, this 0.33, batches of
  // 4 tiles with the next batch in flight 0.42 -- fewer waves resident)
  auto go = [&](auto c) {
    constexpr int CC = decltype(c)::value, G = 1;
    const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>((tiles + 32 - 1) / 32, 2048)), (unsigned)njobs);
    hipLaunchKernelGGL((k_leaf_bitmaps<CC, G>), grid, dim3(256), lds, s, jobs);
  };
  switch (max_bits <= 4 ? 1 : max_bits <= 8 ? 2 : max_bits <= 16 ? 4 : 8) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    default: go(std::integral_constant<int, 8>{}); break;
  }
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph
