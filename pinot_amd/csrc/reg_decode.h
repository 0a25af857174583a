// reg_decode.h -- register-direct decode of packed fixed-bit streams (k_part_reg, k_count_reg): lane l of a wave owns
// the 32 consecutive docs [32 l, 32 l + 32) of a 2048-doc tile, so its b-bit values of a stream are exactly b dwords,
// loaded with 16-byte buffer loads and decoded with compile-time bit positions by a switch over the width.
#pragma once
#include "scan_kernel.h"

namespace ph {

template <int B, int J, int N>
__device__ __forceinline__ uint32_t reg_value(const uint32_t (&W)[N]) {
  constexpr int s = J * B, k = s >> 5, o = s & 31;
  static_assert(k < N, "value beyond the lane's dwords");
  if constexpr (B == 32) {
    return W[k];
  } else if constexpr (o + B <= 32) {
    return (W[k] >> (32 - o - B)) & ((1u << B) - 1u);
  } else {
    static_assert(k + 1 < N, "value beyond the lane's dwords");
    return __builtin_amdgcn_alignbit(W[k], W[k + 1], 64 - o - B) & ((1u << B) - 1u);
  }
}

// the lane's 32 values of one stream (width `bits` <= 4 C, wave-uniform): f(j, value) for j = 0..31
template <int C, class F>
__device__ __forceinline__ void reg_decode(const u32x4 (&pool)[C], int bits, F&& f) {
  uint32_t W[4 * C];
#pragma unroll
  for (int k = 0; k < 4 * C; ++k) W[k] = __builtin_bswap32(pool[k >> 2][k & 3]);
  auto run = [&](auto bb) {
    constexpr int BB = decltype(bb)::value;
    if constexpr (BB <= 4 * C) static_for<0, 32>([&](auto j) { f(j, reg_value<BB, decltype(j)::value, 4 * C>(W)); });
  };
  switch (bits) {
#define PH_REG_CASE(n) \
  case n: run(std::integral_constant<int, n>{}); break;
    PH_REG_CASE(1) PH_REG_CASE(2) PH_REG_CASE(3) PH_REG_CASE(4) PH_REG_CASE(5) PH_REG_CASE(6) PH_REG_CASE(7)
    PH_REG_CASE(8) PH_REG_CASE(9) PH_REG_CASE(10) PH_REG_CASE(11) PH_REG_CASE(12) PH_REG_CASE(13) PH_REG_CASE(14)
    PH_REG_CASE(15) PH_REG_CASE(16) PH_REG_CASE(17) PH_REG_CASE(18) PH_REG_CASE(19) PH_REG_CASE(20)
    PH_REG_CASE(21) PH_REG_CASE(22) PH_REG_CASE(23) PH_REG_CASE(24) PH_REG_CASE(25) PH_REG_CASE(26)
    PH_REG_CASE(27) PH_REG_CASE(28) PH_REG_CASE(29) PH_REG_CASE(30) PH_REG_CASE(31) PH_REG_CASE(32)
#undef PH_REG_CASE
    default: break;
  }
}

// the lane's 32 values of one stream into registers (the switch over the width only moves bit fields; the caller's
// per-doc work is emitted once, after it, instead of once per width)
template <int C>
__device__ __forceinline__ void reg_unpack(const u32x4 (&pool)[C], int bits, uint32_t (&out)[32]) {
  reg_decode<C>(pool, bits, [&](auto j, uint32_t v) { out[decltype(j)::value] = v; });
}

// a lane's C 16-byte loads of one stream of the tile whose first 32-doc run is `run0`: lane l reads the b dwords
// of run run0 + l.  The descriptor is wave-uniform (`use`: the tile reads this stream; `bytes` covers the stream's
// packed bytes rounded up to dwords plus 16, inside the allocation's kFwdPadBytes pad); a lane past the tile's docs
// gets an out-of-range offset, which the hardware answers with zeros and no memory access.
template <int C>
__device__ __forceinline__ void reg_load(bool use, bool lane_live, const uint32_t* fwd, int32_t bits, int64_t bytes,
                                         int32_t run0, int lane, u32x4 (&pool)[C]) {
  // the descriptor's base and size are forced into SGPRs: a descriptor the compiler cannot prove wave-uniform (r5: the
  // size went through a 64-bit min in VGPRs) turns every buffer load into a readfirstlane waterfall loop
  const uint64_t nb64 = use ? (uint64_t)((bytes + 3) & ~(int64_t)3) + 16u : 0u;
  const uint32_t nb = __builtin_amdgcn_readfirstlane(nb64 > 0x7fffffffull ? 0x7fffffffu : (uint32_t)nb64);
  const uint64_t base = use ? (uint64_t)(uintptr_t)fwd : 0u;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>((uintptr_t)(((uint64_t)hi << 32) | lo)), 0, (int)nb, 0x00020000);
  const uint32_t vo = (use && lane_live) ? (uint32_t)(run0 + lane) * 4u * (uint32_t)bits : 0x80000000u;
#pragma unroll
  for (int k = 0; k < C; ++k)
    pool[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo + 16u * k, 0, 0));
}

}  // namespace ph
