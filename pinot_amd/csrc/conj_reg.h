// conj_reg.h -- the register-direct front end of the sparse kernels (k_group_sparse, k_agg_sparse) for a segment
// filtered by an AND of dictId scan leaves only (SSB on dictionary-encoded dimensions: `d_year = 1993 AND
// lo_discount BETWEEN 1 AND 3 AND lo_quantity < 25`, AndDocIdSet over ScanBasedFilterOperators).
//
// The streaming kernels decode every referenced column of every doc; at the 0.01-4 % selectivity of these ANDs the
// group and value columns are needed for few docs.  Here a wave step (64 doc words, 4096 docs) decodes only the
// leaves' streams, reg_decode.h-style: in each of two 2048-doc passes lane l owns the 32 consecutive docs of run
// 2w + 64 pass + l, loads its b dwords of every leaf's stream with 16-byte buffer loads (consecutive lanes read
// consecutive runs), tests each value against the leaf's dictId range or set (sets staged in LDS per chunk when they
// have <= kConjSetWords words, read from HBM otherwise) and ANDs the 32-bit masks; two lanes' masks then form the
// 64-doc word of lane w + j.  The kernels list the word's docs and gather the group keys and values of those only.
#pragma once
#include "reg_decode.h"

namespace ph {

// the leaves' sets into LDS (`sets`: [kMaxConj][kConjSetWords]); every thread of the workgroup calls it for the
// chunk's segment, between two barriers
__device__ __forceinline__ void conj_stage_sets(SegPtr S, uint32_t* sets, int tid, int nthreads) {
  for (int k = 0; k < S->sp_nscan; ++k) {
    if (!S->sp_set[k]) continue;
    const int words = (S->cols[S->sp_slot[k]].cardinality + 31) >> 5;
    if (words > kConjSetWords) continue;
    for (int i = tid; i < words; i += nthreads) sets[k * kConjSetWords + i] = S->sp_set[k][i];
  }
}

// the leaf's doc bitmap word of run `run` (32 docs), when the filter statistic wants it (conj_reg's leaf masks are
// the scan's own: the statistic's AND walk then reads no forward index again)
__device__ __forceinline__ void conj_leaf_out(SegPtr S, int k, int32_t run, uint32_t mask, int64_t ndocs) {
  uint32_t* out = S->sp_lbits[k];
  if (out != nullptr && (int64_t)run < (ndocs + 63) / 64 * 2) out[run] = mask;  // the last word's upper half too
}

// a leaf's test of the 32 values of one lane's run into a 32-bit mask
template <int C>
__device__ __forceinline__ uint32_t conj_leaf_mask(SegPtr S, int k, const u32x4 (&pool)[C], const uint32_t* sets) {
  ColRef col = S->cols[S->sp_slot[k]];
  uint32_t v[32];
  reg_unpack<C>(pool, col.bits, v);
  uint32_t pass = 0;
  const uint32_t* gset = S->sp_set[k];
  if (gset) {
    const uint32_t card = (uint32_t)col.cardinality;
    if (((card + 31) >> 5) <= (uint32_t)kConjSetWords) {
      const uint32_t* ls = sets + k * kConjSetWords;
#pragma unroll
      for (int j = 0; j < 32; ++j) pass |= (v[j] < card && ((ls[v[j] >> 5] >> (v[j] & 31)) & 1u) ? 1u : 0u) << j;
    } else {
#pragma unroll
      for (int j = 0; j < 32; ++j) pass |= (v[j] < card && ((gset[v[j] >> 5] >> (v[j] & 31)) & 1u) ? 1u : 0u) << j;
    }
  } else {
    const uint32_t lo = S->sp_lo[k], len = S->sp_len[k];
#pragma unroll
    for (int j = 0; j < 32; ++j) pass |= ((v[j] - lo) < len ? 1u : 0u) << j;
  }
  return pass;
}

// the AND of the leaves over doc word w + lane of the step at word w (words at or past `we`: 0).  One leaf of one
// pass at a time (C loads in flight, then the test): few registers, so the kernel's gather phase keeps its occupancy
// and the other waves hide the loads' latency
template <int C>
__device__ __forceinline__ unsigned long long conj_step_word(SegPtr S, int32_t w, int32_t we, int lane,
                                                             const uint32_t* sets) {
  const int n = S->sp_nscan;
  const int64_t ndocs = S->num_docs;
  uint32_t half[2];
  if constexpr (C <= 2) {
    // every leaf <= 8 bits (the host picks C = 2 then): all leaves' loads of both passes issued at once (2 x 32 B
    // per lane and leaf), then tested -- r4's one-leaf-at-a-time form kept one load per wave in flight
    u32x4 pool[2][kMaxConj][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int32_t run0 = 2 * w + 64 * h;
      const bool live = (int64_t)(run0 + lane) * 32 < ndocs;
#pragma unroll
      for (int k = 0; k < kMaxConj; ++k) {
        const bool use = k < n;
        ColRef col = S->cols[use ? S->sp_slot[k] : 0];
        reg_load<2>(use, live, use ? col.fwd : nullptr, use ? col.bits : 0, use ? (ndocs * col.bits + 7) / 8 : 0,
                    run0, lane, pool[h][k]);
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int32_t run = 2 * w + 64 * h + lane;
      const int64_t d0 = (int64_t)run * 32;
      const uint32_t valid = d0 >= ndocs ? 0u : (d0 + 32 <= ndocs ? 0xffffffffu : ((1u << (uint32_t)(ndocs - d0)) - 1u));
      uint32_t m = valid;
#pragma unroll
      for (int k = 0; k < kMaxConj; ++k)
        if (k < n) {
          const uint32_t lm = conj_leaf_mask<2>(S, k, pool[h][k], sets) & valid;
          conj_leaf_out(S, k, run, lm, ndocs);
          m &= lm;
        }
      half[h] = m;
    }
  } else {
    // leaf by leaf, both passes' loads of the leaf issued together, as many 16-byte units as its width needs (a
    // 3-bit column's 12 bytes per lane: one), not the widest leaf's
    const int32_t ra = 2 * w, rb = 2 * w + 64;
    const bool la = (int64_t)(ra + lane) * 32 < ndocs, lb = (int64_t)(rb + lane) * 32 < ndocs;
    auto valid = [&](int32_t run) -> uint32_t {
      const int64_t d0 = (int64_t)(run + lane) * 32;
      return d0 >= ndocs ? 0u : (d0 + 32 <= ndocs ? 0xffffffffu : ((1u << (uint32_t)(ndocs - d0)) - 1u));
    };
    half[0] = valid(ra);
    half[1] = valid(rb);
#pragma unroll 1
    for (int k = 0; k < n; ++k) {
      ColRef col = S->cols[S->sp_slot[k]];
      auto leaf = [&](auto cc) {
        constexpr int CC = decltype(cc)::value;
        u32x4 pa[CC], pb[CC];
        const int64_t bytes = (ndocs * col.bits + 7) / 8;
        reg_load<CC>(true, la, col.fwd, col.bits, bytes, ra, lane, pa);
        reg_load<CC>(true, lb, col.fwd, col.bits, bytes, rb, lane, pb);
        const uint32_t ma = conj_leaf_mask<CC>(S, k, pa, sets) & valid(ra);
        const uint32_t mb = conj_leaf_mask<CC>(S, k, pb, sets) & valid(rb);
        conj_leaf_out(S, k, ra + lane, ma, ndocs);
        conj_leaf_out(S, k, rb + lane, mb, ndocs);
        half[0] &= ma;
        half[1] &= mb;
      };
      if (col.bits <= 4) leaf(std::integral_constant<int, 1>{});
      else if (col.bits <= 8) leaf(std::integral_constant<int, 2>{});
      else if (C <= 4 || col.bits <= 16) leaf(std::integral_constant<int, (C < 4 ? C : 4)>{});
      else leaf(std::integral_constant<int, C>{});
    }
  }
  const int src = 2 * (lane & 31);
  const uint32_t x0 = __shfl(half[0], src), y0 = __shfl(half[0], src + 1);
  const uint32_t x1 = __shfl(half[1], src), y1 = __shfl(half[1], src + 1);
  const unsigned long long word = lane < 32 ? ((unsigned long long)y0 << 32 | x0) : ((unsigned long long)y1 << 32 | x1);
  return w + lane < we ? word : 0ull;
}

}  // namespace ph
