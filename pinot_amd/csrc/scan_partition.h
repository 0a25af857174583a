// scan_partition.h -- device helpers shared by the partitioned group-by's kernel A forms (scan_partition.hip: the
// LDS-staged k_part_scan / k_part_scan2; scan_partition_reg.hip: the register-direct k_part_reg): the listed flush of
// the per-partition LDS rings and the final flush.
#pragma once
#include "scan_kernel.h"

namespace ph {

// Flush of the lean kernel's rings, listed partitions only: a partition enters the round's list when an append
// completes its first whole 64-byte chunk, so the flush touches ~(round records / 16) partitions instead of all P.
// Per listed partition (8 lanes of one wave) the whole chunks go to the partition's region at its flushed
// position with 16-byte stores, and the < 16 leftovers move to the front of the ring.  Every lane reads before
// any lane of its wave writes (LDS ops of a wave execute in order), so a leftover never overwrites a record still
// to be stored.  `matched` gains the appends that went to the overflow table (a full ring).
template <int REC64, int BLOCK>
__device__ __forceinline__ void part_flush_listed(const KParams& p, uint8_t* smem, const uint32_t* flist, uint32_t nlisted,
                                  unsigned long long& matched) {
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  constexpr uint32_t CH = 64 / sizeof(Rec);  // records per 64-byte chunk
  constexpr uint32_t PQ = 16 / sizeof(Rec);  // records per 16-byte quarter
  Rec* slots = reinterpret_cast<Rec*>(smem + p.pl_slot_off);
  uint32_t* pend = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  uint32_t* gpos = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  const uint32_t cap = (uint32_t)p.part_cap;
  const uint32_t total = nlisted * 8u;
  for (uint32_t t = threadIdx.x; t < total; t += BLOCK) {
    const uint32_t b = flist[t >> 3], i = t & 7u;
    const uint32_t raw = pend[b];
    const uint32_t n = min(raw, C);  // records beyond C went to the overflow table
    const uint32_t out = n & ~(CH - 1u), left = n - out;
    const uint32_t g = gpos[b];
    Rec* ring = slots + ((size_t)b << cl);
    // reads: quarters i and i + 8 of the outgoing records (C / PQ <= 16), leftovers i and i + 8 (< CH <= 16)
    u32x4 q0 = {0u, 0u, 0u, 0u}, q1 = {0u, 0u, 0u, 0u};
    const uint32_t r0 = i * PQ, r1 = (i + 8u) * PQ;
    if (r0 < out) q0 = *reinterpret_cast<const u32x4*>(ring + r0);
    if (r1 < out) q1 = *reinterpret_cast<const u32x4*>(ring + r1);
    Rec l0 = 0, l1 = 0;
    if (i < left) l0 = ring[out + i];
    if (i + 8u < left) l1 = ring[out + i + 8u];
    // writes
    Rec* region = reinterpret_cast<Rec*>(p.part_buf) + part_region(p, b, blockIdx.x) * (size_t)cap;
    if (r0 < out) {
      if (g + r0 + PQ <= cap) {
        *reinterpret_cast<u32x4*>(region + g + r0) = q0;
      } else {
        const Rec* e = reinterpret_cast<const Rec*>(&q0);
        for (uint32_t k = 0; k < PQ; ++k) part_store<REC64>(p, b, g + r0 + k, e[k]);
      }
    }
    if (r1 < out) {
      if (g + r1 + PQ <= cap) {
        *reinterpret_cast<u32x4*>(region + g + r1) = q1;
      } else {
        const Rec* e = reinterpret_cast<const Rec*>(&q1);
        for (uint32_t k = 0; k < PQ; ++k) part_store<REC64>(p, b, g + r1 + k, e[k]);
      }
    }
    if (i < left) ring[i] = l0;
    if (i + 8u < left) ring[i + 8u] = l1;
    if (i == 0) {
      pend[b] = left;
      gpos[b] = g + out;
      matched += raw - n;
    }
  }
}

// Final flush of the lean kernel (after the last listed flush): every partition's < 16 pending records, the
// region record counts, and the matched docs = the regions' records (overflow appends counted already).
template <int REC64, int BLOCK>
__device__ __forceinline__ void part_flush_final(const KParams& p, uint8_t* smem, unsigned long long& matched) {
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  const Rec* slots = reinterpret_cast<const Rec*>(smem + p.pl_slot_off);
  const uint32_t* pend = reinterpret_cast<const uint32_t*>(smem + p.pl_lcnt_off);
  const uint32_t* gpos = reinterpret_cast<const uint32_t*>(smem + p.pl_bcnt_off);
  const int cl = p.part_slot_log2;
  const uint32_t total = (uint32_t)p.num_parts * 16u;
  for (uint32_t t = threadIdx.x; t < total; t += BLOCK) {
    const uint32_t b = t >> 4, i = t & 15u;
    const uint32_t n = pend[b], g = gpos[b];  // n < 16 after the listed flushes
    if (i < n) part_store<REC64>(p, b, g + i, slots[((size_t)b << cl) + i]);
    if (i == 0) {
      p.part_count[(size_t)b * gridDim.x + blockIdx.x] = g + n;  // records of region (b, blockIdx)
      matched += g + n;
    }
  }
}

// The register-direct kernel A's flush (k_part_reg), one thread per partition: a partition with a whole pending 64-byte
// chunk writes its whole chunks to its region with 16-byte stores (each thread a whole chunk: the 4 stores of a chunk
// merge in L2 into one 64-byte write) and copies the partial chunk to the front of its ring.  One LDS word read per
// partition and round decides; r5 SQ counters: the 8-lanes-per-partition sweep over all partitions issued ~20 VALU per
// doc, this form ~2.  `final`: every pending record goes out (< 16 after the last round's flush), the region counts
// are written.
template <int BLOCK>
__device__ __forceinline__ void part_flush_owner(const KParams& p, uint8_t* smem, unsigned long long& matched,
                                                 bool final, int set = 0, bool count = true) {
  uint32_t* slots = reinterpret_cast<uint32_t*>(smem + p.pl_slot_off) + (size_t)set * p.part_set_words;
  uint32_t* pend = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off) + (size_t)set * (p.num_parts + 64);
  uint32_t* gpos = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  const uint32_t cap = (uint32_t)p.part_cap;
  const uint32_t P = (uint32_t)p.num_parts;
  for (uint32_t b = threadIdx.x; b < P; b += BLOCK) {
    const uint32_t raw = pend[b];
    if (!final && raw < 16u) continue;
    const uint32_t n = min(raw, C);  // records beyond C went to the overflow table
    const uint32_t out = final ? n : (n & ~15u), left = n - out;
    const uint32_t g = gpos[b];
    uint32_t* ring = slots + (size_t)b * (uint32_t)p.part_ring_stride;
    uint32_t* region = reinterpret_cast<uint32_t*>(p.part_buf) + part_region(p, b, blockIdx.x) * (size_t)cap;
    for (uint32_t k = 0; k < out; k += 16u) {
      u32x4 q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) q[e] = *reinterpret_cast<const u32x4*>(ring + k + 4 * e);
      if (g + k + 16u <= cap) {
#pragma unroll
        for (int e = 0; e < 4; ++e) *reinterpret_cast<u32x4*>(region + g + k + 4 * e) = q[e];  // (final: past n unread)
      } else {
        const uint32_t m = min(16u, out - k);
        for (uint32_t e = 0; e < m; ++e) part_store<0>(p, b, g + k + e, ring[k + e]);  // region full (skew)
      }
    }
    if (left) {  // the partial chunk to the front of the ring (whole 16-byte quarters; past `left` is garbage)
      u32x4 q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) q[e] = *reinterpret_cast<const u32x4*>(ring + out + 4 * e);
#pragma unroll
      for (int e = 0; e < 4; ++e) *reinterpret_cast<u32x4*>(ring + 4 * e) = q[e];
    }
    pend[b] = left;
    gpos[b] = g + out;
    matched += raw - n;
    if (final && count) {
      p.part_count[(size_t)b * gridDim.x + blockIdx.x] = g + out;  // records of region (b, blockIdx)
      matched += g + out;
    }
  }
}

}  // namespace ph
