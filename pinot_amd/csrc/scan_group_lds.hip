// scan_group_lds.hip -- k_scan instantiations of the LDS-private dense group table plan (MODE_GROUP_LDS), and the
// lean form k_group_lds_lean.
#include "scan_kernel.h"

namespace ph {

// ------------------------------------------------------------------ lean MODE_GROUP_LDS
// k_group_lds_lean is k_scan<MODE_GROUP_LDS> for the common shape (DefaultGroupByExecutor over a
// DictionaryBasedGroupKeyGenerator array holder: identity key remaps, at most one packed integer value column,
// filter leaf ALL / RANGE / DOCRANGE).  Per matched doc:
//  * COUNT and SUM share one 64-bit LDS add when they fit (count << 40 | value - vmin: lds_pack), else a 32-bit
//    count add and a 64-bit sum add;
//  * MIN / MAX offsets live in the two halves of one 64-bit word that is READ first; an LDS atomic is issued only
//    when the value improves one of them (min only falls, max only rises: a stale read is safe), so after the
//    first few docs of each key the per-doc cost is one atomic and one read instead of four atomics;
//  * the table is replicated per wave when it fits (lds_copies), so waves on different SIMDs never contend for
//    one key's words; the copies are summed once at the end.
template <int NG, int FK, int PACK>
__device__ __forceinline__ void group_lds_tile(const KParams& p, SegPtr S, uint32_t wst_off, int lane, int32_t w0,
                                               int32_t nvalid, uint8_t* tbl, unsigned long long& matched) {
  const uint32_t ndocs = (uint32_t)S->num_docs;
  LaneStream fs = lane_stream(wst_off + (uint32_t)p.stage_soff[p.f_stream],
                              FK == FK_RANGE ? S->streams[p.f_stream].bits : 1, lane);
  const uint32_t flo = S->flo, flen = S->flen;
  LaneStream gs[NG];
  uint32_t gstr[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    gs[g] = lane_stream(wst_off + (uint32_t)p.stage_soff[p.g_stream[g]], S->streams[p.g_stream[g]].bits, lane);
    gstr[g] = (uint32_t)p.group_stride[g];
  }
  const bool hasv = p.num_vals > 0;
  LaneStream vs = fs;
  uint32_t vadd = 0;
  if (hasv) {
    vs = lane_stream(wst_off + (uint32_t)p.stage_soff[p.v_stream[0]], S->streams[p.v_stream[0]].bits, lane);
    vadd = (uint32_t)(S->vals[0].base - p.part_vbase);
  }
  const uint32_t G = (uint32_t)p.num_groups;
  unsigned long long* cs = reinterpret_cast<unsigned long long*>(tbl);            // [G] count<<40|sum or sum
  uint32_t* cnt = reinterpret_cast<uint32_t*>(tbl + (size_t)G * 8);               // [G] counts (!PACK)
  uint32_t* mm = reinterpret_cast<uint32_t*>(tbl + (size_t)G * (PACK ? 8 : 12));  // [G][2] min, max offsets
  const int ops = p.val_ops[0];
  const bool want_mm = hasv && (ops & (OPS_MIN | OPS_MAX));
  uint32_t doc = (uint32_t)w0 * 64u + (uint32_t)lane;
  uint32_t tcnt = 0;
  for (int u = 0; u < nvalid; u += 2) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      bool hh = (u + q < nvalid) & (doc < ndocs);
      if constexpr (FK == FK_RANGE) hh &= (lds_value(fs.off, fs.rsh, fs.mask) - flo) < flen;
      if constexpr (FK == FK_DOCRANGE) hh &= (doc - flo) < flen;
      uint32_t key = 0;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        key += __umul24(lds_value(gs[g].off, gs[g].rsh, gs[g].mask), gstr[g]);
        gs[g].off += gs[g].step;
      }
      const uint32_t vo = hasv ? lds_value(vs.off, vs.rsh, vs.mask) + vadd : 0u;
      if (hasv) vs.off += vs.step;
      if (FK == FK_RANGE) fs.off += fs.step;
      doc += 64u;
      tcnt += (uint32_t)__popcll(__ballot(hh));
      if (hh) {
        if (PACK) {
          atomicAdd(&cs[key], (1ull << 40) | (unsigned long long)vo);
        } else {
          atomicAdd(&cnt[key], 1u);
          if (hasv) atomicAdd(&cs[key], (unsigned long long)vo);
        }
        if (want_mm) {
          const unsigned long long cur = *reinterpret_cast<const unsigned long long*>(mm + 2 * key);
          if ((ops & OPS_MIN) && vo < (uint32_t)cur) atomicMin(&mm[2 * key], vo);
          if ((ops & OPS_MAX) && vo > (uint32_t)(cur >> 32)) atomicMax(&mm[2 * key + 1], vo);
        }
      }
    }
  }
  matched += tcnt;
}

template <int NG, int PACK>
__global__ void __launch_bounds__(kBlock) k_group_lds_lean(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NL = kPrefetchOther;
  constexpr int WAVES = kWaves;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  uint8_t* wst = smem + p.stage_off + (size_t)wave * p.stage_stride;
  const uint32_t wst_off = lds_addr(wst);
  const uint32_t G = (uint32_t)p.num_groups;
  const size_t copy_bytes = (size_t)p.lds_copy_bytes;
  const int copies = p.lds_copies;
  uint8_t* tbl0 = smem + p.lds_cnt_off;
  // init every copy: sums / counts 0, min offset ~0, max offset 0
  for (uint32_t i = threadIdx.x; i < (uint32_t)copies * G; i += kBlock) {
    uint8_t* t = tbl0 + (size_t)(i / G) * copy_bytes;
    const uint32_t k = i % G;
    reinterpret_cast<unsigned long long*>(t)[k] = 0;
    if (!PACK) reinterpret_cast<uint32_t*>(t + (size_t)G * 8)[k] = 0;
    uint32_t* mm = reinterpret_cast<uint32_t*>(t + (size_t)G * (PACK ? 8 : 12));
    mm[2 * k] = 0xffffffffu;
    mm[2 * k + 1] = 0u;
  }
  __syncthreads();
  uint8_t* tbl = tbl0 + (size_t)(wave % copies) * copy_bytes;
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
    if (cnvalid > 0) {
      const int fk = cs->fkind;
      if (fk == FK_RANGE) group_lds_tile<NG, FK_RANGE, PACK>(p, cs, wst_off, lane, cw0, cnvalid, tbl, matched);
      else if (fk == FK_DOCRANGE) group_lds_tile<NG, FK_DOCRANGE, PACK>(p, cs, wst_off, lane, cw0, cnvalid, tbl, matched);
      else group_lds_tile<NG, FK_ALL, PACK>(p, cs, wst_off, lane, cw0, cnvalid, tbl, matched);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0 && matched && p.matched_total) atomicAdd(p.matched_total, matched);
  __syncthreads();
  // merge the copies and add this workgroup's table into the dense result
  const int ops = p.num_vals ? p.val_ops[0] : 0;
  for (uint32_t k = threadIdx.x; k < G; k += kBlock) {
    unsigned long long n = 0, sum = 0;
    uint32_t vmin = 0xffffffffu, vmax = 0u;
    for (int cp = 0; cp < copies; ++cp) {
      const uint8_t* t = tbl0 + (size_t)cp * copy_bytes;
      const unsigned long long x = reinterpret_cast<const unsigned long long*>(t)[k];
      if (PACK) {
        n += x >> 40;
        sum += x & ((1ull << 40) - 1ull);
      } else {
        n += reinterpret_cast<const uint32_t*>(t + (size_t)G * 8)[k];
        sum += x;
      }
      const uint32_t* mm = reinterpret_cast<const uint32_t*>(t + (size_t)G * (PACK ? 8 : 12));
      vmin = min(vmin, mm[2 * k]);
      vmax = max(vmax, mm[2 * k + 1]);
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

template <int NG>
static void launch_lds_lean(const KParams& p, int grid, size_t lds, hipStream_t s) {
  if (p.lds_pack) {
    allow_lds(k_group_lds_lean<NG, 1>, lds);
    hipLaunchKernelGGL((k_group_lds_lean<NG, 1>), dim3(grid), dim3(kBlock), lds, s, p);
  } else {
    allow_lds(k_group_lds_lean<NG, 0>, lds);
    hipLaunchKernelGGL((k_group_lds_lean<NG, 0>), dim3(grid), dim3(kBlock), lds, s, p);
  }
}

void launch_scan_group_lds(const KParams& p, int ng, int grid, size_t lds, hipStream_t s) {
  if (p.lds_fast) {
    switch (ng) {
      case 1: launch_lds_lean<1>(p, grid, lds, s); break;
      case 2: launch_lds_lean<2>(p, grid, lds, s); break;
      case 3: launch_lds_lean<3>(p, grid, lds, s); break;
      default: launch_lds_lean<4>(p, grid, lds, s); break;
    }
    return;
  }
  launch_mode<MODE_GROUP_LDS>(p, ng, value_variant(p), grid, lds, s);
}

}  // namespace ph
