// scan_partition.hip -- the partitioned group-by (MODE_PARTITION): kernel A (k_scan instantiations that append records
// to per-(partition, workgroup) regions) and kernel B (k_part_agg), plus the overflow-table merge.
#include "scan_partition.h"

namespace ph {

size_t partition_lds_bytes(KParams& p, int ring_log2) {
  const size_t rec = p.part_vbits + p.part_klo > 32 ? 8 : 4;
  size_t o = 0;
  auto place = [&](int32_t& dst, size_t bytes) {
    dst = (int32_t)o;
    o = (o + bytes + 15) / 16 * 16;
  };
  int32_t stage_off = 0;
  place(stage_off, (size_t)kPartWaves * p.stage_stride);
  p.stage_off = stage_off;
  // ring slots per partition: a whole 64-byte chunk of leftovers (< 16 records) plus one round's appends
  // (~ round records / P, Poisson) must fit or records take the overflow-table path
  int cl = std::max(3, std::min(7, ring_log2));  // (<= 7: a partition's flush lanes stay in one wave)
  while (cl > 4 && (size_t)(p.num_parts << cl) * rec > 48 * 1024) --cl;
  // the lean kernel's flush moves a partition's records with 16 lanes, one 16-byte quarter each
  if (p.part_fast) cl = std::min(cl, rec == 4 ? 6 : 5);
  // (r5: 128-byte flush chunks from 64-slot rings measured the same as 64-byte ones, 2.751 vs 2.754 ms at klo 13)
  p.part_slot_log2 = cl;
  // k_part_reg pads each ring by one 16-byte quarter: with 128-byte rings the owner threads of 16 consecutive
  // partitions would read / write the same 16 bytes of their rings in ONE bank quad (r5: bank conflicts 72 % of the
  // kernel's LDS cycles); a 144-byte stride puts them on 16 distinct quads
  p.part_ring_stride = p.part_reg ? (1 << cl) + 4 : (1 << cl);
  // + one scratch slot and one scratch word per lane: k_part_scan appends misses there (branch-free); k_part_reg has
  // two ring sets (a round appends to one while the other's completed chunks go out)
  const int sets = p.part_reg ? (p.part_sets == 1 ? 1 : 2) : 1;
  p.part_set_words = (int32_t)((size_t)p.num_parts * p.part_ring_stride + 64);
  place(p.pl_slot_off, (size_t)sets * p.part_set_words * rec);
  // generic kernel: (flushed / CH << 16 | pending) per partition; lean kernel: pending per partition
  place(p.pl_lcnt_off, 4 * ((size_t)p.num_parts + 64) * sets);
  place(p.pl_bcnt_off, 4 * (size_t)p.num_parts);  // lean kernel: records flushed per partition (region position)
  // lean kernel: two lists (round parity) of the partitions whose ring reached a whole chunk, + their counts
  place(p.pl_misc_off, 8 * (size_t)p.num_parts + 16);
  return o;
}

// ------------------------------------------------------------------ kernel A, lean form
// k_part_scan is k_scan<MODE_PARTITION> for the common shapes (no gathers: identity key remaps, a packed value
// stream; filter leaf ALL / RANGE / DOCRANGE) written for issue efficiency:
//  * per group of 4 words the filter, key and value decodes of every lane are straight-line; each stream keeps
//    one per-lane LDS byte offset that advances by the stream's 8*b bytes per word (one add per value);
//  * keys are 24-bit multiply-adds;
//  * a partition's ring holds only its pending records, from slot 0 (the flush writes the whole 64-byte chunks
//    and moves the < 16 leftovers to the front), so a record's slot is its partition's pending count: one
//    returning LDS add, one compare, one shift-add.  The 4 rank atomics issue back to back, a miss increments
//    its lane's scratch word and stores to its lane's scratch slot instead of branching.
// r2 SQ counters on the generic form: 61 VALU + 44 SALU per 64-doc word and 51 % of wave cycles waiting.
template <int NG, int REC64, int HASV, int FK>
__device__ __forceinline__ void part_tile(const KParams& p, SegPtr S, uint8_t* smem, uint32_t wst_off, int lane,
                                          int32_t w0, int32_t nvalid, uint32_t* flist, uint32_t* fcnt) {
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  constexpr uint32_t CH = 64 / sizeof(Rec);
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
  LaneStream vs = fs;
  uint32_t vadd = 0;
  if (HASV) {
    vs = lane_stream(wst_off + (uint32_t)p.stage_soff[p.v_stream[0]], S->streams[p.v_stream[0]].bits, lane);
    vadd = (uint32_t)(S->vals[0].base - p.part_vbase);  // record value = packed offset + (base - vmin)
  }
  const uint32_t klo = (uint32_t)p.part_klo, kmask = (1u << klo) - 1u, vbits = (uint32_t)p.part_vbits;
  const int cl = p.part_slot_log2;
  const uint32_t C = 1u << cl;
  uint32_t* pend = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  Rec* slots = reinterpret_cast<Rec*>(smem + p.pl_slot_off);
  const uint32_t dummy_word = (uint32_t)p.num_parts + (uint32_t)lane;
  const uint32_t dummy_slot = ((uint32_t)p.num_parts << cl) + (uint32_t)lane;
  uint32_t doc = (uint32_t)w0 * 64u + (uint32_t)lane;
  for (int u = 0; u < nvalid; u += 4) {
    bool h[4];
    uint32_t widx[4], bk[4];
    Rec rec[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bool hh = (u + q < nvalid) & (doc < ndocs);
      if constexpr (FK == FK_RANGE) hh &= (lds_value(fs.off, fs.rsh, fs.mask) - flo) < flen;
      if constexpr (FK == FK_DOCRANGE) hh &= (doc - flo) < flen;
      uint32_t key = 0;
#pragma unroll
      for (int g = 0; g < NG; ++g) key += __umul24(lds_value(gs[g].off, gs[g].rsh, gs[g].mask), gstr[g]);  // keys < 2^22
      const uint32_t vo = HASV ? lds_value(vs.off, vs.rsh, vs.mask) + vadd : 0u;
#pragma unroll
      for (int g = 0; g < NG; ++g) gs[g].off += gs[g].step;
      if (HASV) vs.off += vs.step;
      if (FK == FK_RANGE) fs.off += fs.step;
      doc += 64u;
      h[q] = hh;
      bk[q] = key >> klo;
      rec[q] = REC64 ? (Rec)(((unsigned long long)(key & kmask) << 32) | vo) : (Rec)(((key & kmask) << vbits) | vo);
      widx[q] = hh ? bk[q] : dummy_word;
    }
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) w[q] = atomicAdd(&pend[widx[q]], 1u);
    bool ovf = false, full = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool ok = h[q] & (w[q] < C);
      ovf |= h[q] & (w[q] >= C);
      full |= h[q] & (w[q] == CH - 1u);
      slots[ok ? (bk[q] << cl) + w[q] : dummy_slot] = rec[q];
    }
    if (__ballot(full)) {  // this record completed its partition's first whole chunk of the round: list it
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (h[q] && w[q] == CH - 1u) flist[atomicAdd(fcnt, 1u)] = bk[q];
    }
    if (__ballot(ovf)) {  // a skewed round filled a ring: those records aggregate into the overflow table
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (h[q] && w[q] >= C) part_overflow<REC64>(p, bk[q], rec[q]);
    }
  }
}

template <int NG, int REC64, int HASV>
__global__ void __launch_bounds__(kPartBlock) k_part_scan(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NL = kPrefetchPartition;
  constexpr int WAVES = kPartWaves;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  uint8_t* wst = smem + p.stage_off + (size_t)wave * p.stage_stride;
  const uint32_t wst_off = lds_addr(wst);
  uint32_t* words = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  uint32_t* gpos = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
  uint32_t* lists = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off);  // [2][P] listed partitions
  uint32_t* lcnt = lists + 2 * p.num_parts;                            // [2] list lengths
  for (int i = threadIdx.x; i < p.num_parts + 64; i += kPartBlock) words[i] = 0;
  for (int i = threadIdx.x; i < p.num_parts; i += kPartBlock) gpos[i] = 0;
  if (threadIdx.x < 2) lcnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t par = 0;  // round parity: this round appends to list par, the flush reads list par ^ 1

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
    const bool load_first = p.part_load_first;
    if (load_first && c < c_end) tile_load<NL>(S, w0, nvalid, lane, pf);
    // flush the chunks completed in the previous round; the prefetch goes first (its loads get the flush's time
    // to arrive; the flush's stores, issued after them, complete under the decode)
    {
      const uint32_t prev = par ^ 1u;
      const uint32_t nl = lcnt[prev];
      if (threadIdx.x == 0) lcnt[par] = 0;  // read by nobody now; this round's appends fill it
      part_flush_listed<REC64, kPartBlock>(p, smem, lists + prev * p.num_parts, nl, matched);
    }
    lds_barrier();  // ring words are final before anyone appends again
    if (!load_first && c < c_end) tile_load<NL>(S, w0, nvalid, lane, pf);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (cnvalid > 0) {
      const int fk = cs->fkind;
      uint32_t* fl = lists + par * p.num_parts;
      uint32_t* fc = lcnt + par;
      if (fk == FK_RANGE) part_tile<NG, REC64, HASV, FK_RANGE>(p, cs, smem, wst_off, lane, cw0, cnvalid, fl, fc);
      else if (fk == FK_DOCRANGE) part_tile<NG, REC64, HASV, FK_DOCRANGE>(p, cs, smem, wst_off, lane, cw0, cnvalid, fl, fc);
      else part_tile<NG, REC64, HASV, FK_ALL>(p, cs, smem, wst_off, lane, cw0, cnvalid, fl, fc);
    }
    lds_barrier();  // this round's appends are complete before the next round's flush
    par ^= 1u;
  }
  part_flush_listed<REC64, kPartBlock>(p, smem, lists + (par ^ 1u) * p.num_parts, lcnt[par ^ 1u], matched);
  lds_barrier();
  part_flush_final<REC64, kPartBlock>(p, smem, matched);  // also writes the region record counts
  if (matched && p.matched_total) atomicAdd(p.matched_total, matched);
}

// Kernel A with a two-deep load pipeline (PH_PART_DEPTH=2): the same rounds, rings and flushes as k_part_scan, but
// a wave's loads run two tiles ahead in two register sets (tile_load_fixed), so each wave keeps two tiles of HBM
// reads in flight instead of one (r2: kernel A streamed at 2.6 TB/s with one 12-word tile in flight per wave, its
// occupancy held at 16 waves per CU by the rings + staging LDS).  In a round the flush stores go out BEFORE the
// prefetch loads, so the wait before a set is consumed (vmcnt(NL): the other set still in flight) covers them.
template <int NG, int REC64, int HASV>
__global__ void __launch_bounds__(kPartBlock) k_part_scan2(const KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NL = kPrefetchPartition;
  constexpr int WAVES = kPartWaves;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  SegPtr segs = (SegPtr)p.segs;
  const PH_CONST Chunk* chunks = (const PH_CONST Chunk*)p.chunks;
  uint8_t* wst = smem + p.stage_off + (size_t)wave * p.stage_stride;
  const uint32_t wst_off = lds_addr(wst);
  uint32_t* words = reinterpret_cast<uint32_t*>(smem + p.pl_lcnt_off);
  uint32_t* gpos = reinterpret_cast<uint32_t*>(smem + p.pl_bcnt_off);
  uint32_t* lists = reinterpret_cast<uint32_t*>(smem + p.pl_misc_off);  // [2][P] listed partitions
  uint32_t* lcnt = lists + 2 * p.num_parts;                            // [2] list lengths
  for (int i = threadIdx.x; i < p.num_parts + 64; i += kPartBlock) words[i] = 0;
  for (int i = threadIdx.x; i < p.num_parts; i += kPartBlock) gpos[i] = 0;
  if (threadIdx.x < 2) lcnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t par = 0;
  unsigned long long matched = 0;
  const int32_t tw = p.tile_words;
  const int32_t round_words = WAVES * tw;
  const int64_t nch = p.chunk_end - p.chunk_begin;
  const int32_t c0 = p.chunk_begin + (int32_t)(nch * blockIdx.x / gridDim.x);
  int32_t c = c0, r = 0;
  const int32_t c_end = p.chunk_begin + (int32_t)(nch * (blockIdx.x + 1) / gridDim.x);
  // the round iterator (c, r) names the NEXT tile to load; t0 / t1 are the two tiles in flight (t0 older)
  struct Tile {
    SegPtr S;
    int32_t w0, nvalid;
    bool live;
  };
  auto next_tile = [&]() {
    Tile t{nullptr, 0, 0, false};
    if (c < c_end) {
      const int32_t cbeg = chunks[c].word_begin, cend = chunks[c].word_end;
      t.S = segs + chunks[c].seg;
      t.w0 = cbeg + r * round_words + wave * tw;
      t.nvalid = min(tw, cend - t.w0);
      t.live = true;
      if (cbeg + (r + 1) * round_words < cend) {
        ++r;
      } else {
        ++c;
        r = 0;
      }
    }
    return t;
  };
  Prefetch<NL> pa, pb;
  Tile t0 = next_tile();
  tile_load_fixed<NL>(t0.live && t0.nvalid > 0, t0.S, t0.w0, t0.nvalid, lane, pa);
  Tile t1 = next_tile();
  tile_load_fixed<NL>(t1.live && t1.nvalid > 0, t1.S, t1.w0, t1.nvalid, lane, pb);
  // one round on the tile in `cur` (its loads the older set); the tile two ahead reloads `cur`
  auto round = [&](Prefetch<NL>& cur) {
    if (t0.live) tile_store_nowait<NL>(t0.S, t0.nvalid, wst, lane, cur);
    {
      const uint32_t prev = par ^ 1u;
      const uint32_t nl = lcnt[prev];
      if (threadIdx.x == 0) lcnt[par] = 0;
      part_flush_listed<REC64, kPartBlock>(p, smem, lists + prev * p.num_parts, nl, matched);
    }
    lds_barrier();  // ring words are final before anyone appends again; this wave's staging is written
    const Tile t2 = next_tile();
    tile_load_fixed<NL>(t2.live && t2.nvalid > 0, t2.S, t2.w0, t2.nvalid, lane, cur);  // always NL loads
    if (t0.live && t0.nvalid > 0) {
      const int fk = t0.S->fkind;
      uint32_t* fl = lists + par * p.num_parts;
      uint32_t* fc = lcnt + par;
      if (fk == FK_RANGE) part_tile<NG, REC64, HASV, FK_RANGE>(p, t0.S, smem, wst_off, lane, t0.w0, t0.nvalid, fl, fc);
      else if (fk == FK_DOCRANGE) part_tile<NG, REC64, HASV, FK_DOCRANGE>(p, t0.S, smem, wst_off, lane, t0.w0, t0.nvalid, fl, fc);
      else part_tile<NG, REC64, HASV, FK_ALL>(p, t0.S, smem, wst_off, lane, t0.w0, t0.nvalid, fl, fc);
    }
    lds_barrier();  // this round's appends are complete before the next round's flush; staging read
    par ^= 1u;
    t0 = t1;
    t1 = t2;
  };
  // rounds are workgroup-uniform (every wave of a workgroup walks the same chunk range), so the barriers match.
  // The round count is padded to even (a last round without a tile stages nothing and appends nothing): the loop
  // body is then the unconditional pair round(pa); round(pb), whose load / consume order the waitcnt pass can
  // follow (with a conditional exit between the two rounds it waited for the younger set as well: vmcnt(0))
  int32_t nrounds = 0;
  for (int32_t cc = c0; cc < c_end; ++cc) {
    const int32_t words = chunks[cc].word_end - chunks[cc].word_begin;
    nrounds += (words + round_words - 1) / round_words;
  }
  for (int32_t i = 0; i < nrounds; i += 2) {
    round(pa);
    round(pb);
  }
  part_flush_listed<REC64, kPartBlock>(p, smem, lists + (par ^ 1u) * p.num_parts, lcnt[par ^ 1u], matched);
  lds_barrier();
  part_flush_final<REC64, kPartBlock>(p, smem, matched);
  if (matched && p.matched_total) atomicAdd(p.matched_total, matched);
}

template <int NG, int REC64, int HASV>
static void launch_part_fast(const KParams& p, int grid, size_t lds, hipStream_t s) {
  if (p.part_depth == 2) {
    allow_lds(k_part_scan2<NG, REC64, HASV>, lds);
    hipLaunchKernelGGL((k_part_scan2<NG, REC64, HASV>), dim3(grid), dim3(kPartBlock), lds, s, p);
    return;
  }
  allow_lds(k_part_scan<NG, REC64, HASV>, lds);
  hipLaunchKernelGGL((k_part_scan<NG, REC64, HASV>), dim3(grid), dim3(kPartBlock), lds, s, p);
}

template <int NG>
static void launch_part_fast_ng(const KParams& p, int rec64, int grid, size_t lds, hipStream_t s) {
  const int hasv = p.num_vals > 0;
  if (rec64) {
    if (hasv) launch_part_fast<NG, 1, 1>(p, grid, lds, s);
    else launch_part_fast<NG, 1, 0>(p, grid, lds, s);
  } else {
    if (hasv) launch_part_fast<NG, 0, 1>(p, grid, lds, s);
    else launch_part_fast<NG, 0, 0>(p, grid, lds, s);
  }
}

void launch_scan_partition(const KParams& p, int ng, int rec64, int grid, size_t lds, hipStream_t s) {
  if (p.part_reg) {
    launch_part_reg(p, ng, grid, lds, s);
    return;
  }
  if (!p.part_fast) {
    launch_mode<MODE_PARTITION>(p, ng, rec64, grid, lds, s);
    return;
  }
  switch (ng) {
    case 1: launch_part_fast_ng<1>(p, rec64, grid, lds, s); break;
    case 2: launch_part_fast_ng<2>(p, rec64, grid, lds, s); break;
    case 3: launch_part_fast_ng<3>(p, rec64, grid, lds, s); break;
    default: launch_part_fast_ng<4>(p, rec64, grid, lds, s); break;
  }
}

// ------------------------------------------------------------------ kernel B: partition aggregation
// One workgroup per (partition, slice): every record of the slice's regions goes through an LDS table of the
// partition's keys, then the workgroup merges its key range into the dense result table (one slice: the
// range has exactly one owner, plain read-modify-write; more slices: coalesced device atomics).  Region fill
// levels are read once into LDS; each wave keeps 4 regions' 16-byte-per-lane record loads in flight.  Per key
// the LDS table holds COUNT and the value-offset SUM in one 64-bit word (count << 40 | sum, pack_cs) and
// MIN / MAX offsets in the two halves of a second 64-bit word.  A record reads that min/max word first and
// issues an LDS atomic only when it improves one of them: over a key's records in random order that is
// O(log n) atomics instead of 2 per record (min only falls and max only rises, so a stale read is safe).  A lane
// handles its 16 records of a step together: the count/sum atomics, then all 16 min/max reads before the first
// wait (r3: one read and one wait per record left kernel B latency-bound), then the improving atomics.
template <int REC64>
__global__ void __launch_bounds__(1024) k_part_agg(const PartAggParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int part = blockIdx.x / p.slices;
  const int slice = blockIdx.x - part * p.slices;
  const uint32_t KP = 1u << p.part_klo;
  const int R = p.regions;
  // this slice's regions [r0, r1)
  const int r0 = (int)((int64_t)R * slice / p.slices), r1 = (int)((int64_t)R * (slice + 1) / p.slices);
  const int NR = r1 - r0;
  // LDS layout: [count u32 | count<<40|sum u64] [sum u64] [min|max u32 pairs] [region fill u32 x NR]
  size_t off = 0;
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem);
  unsigned long long* cs = reinterpret_cast<unsigned long long*>(smem);
  const size_t KT = (size_t)KP + 64;  // + one dummy key per lane for padding records (no same-address atomics)
  off += p.pack_cs ? 8 * KT : 4 * KT;
  off = (off + 7) / 8 * 8;
  unsigned long long* sum = reinterpret_cast<unsigned long long*>(smem + off);
  off += (p.has_sum && !p.pack_cs) ? 8 * KT : 0;
  uint32_t* mm = reinterpret_cast<uint32_t*>(smem + off);
  off += (p.has_min | p.has_max) ? 8 * KT : 0;
  uint32_t* fill = reinterpret_cast<uint32_t*>(smem + off);
  for (uint32_t k = threadIdx.x; k < (uint32_t)KT; k += blockDim.x) {
    if (p.pack_cs) cs[k] = 0; else cnt[k] = 0;
    if (p.has_sum && !p.pack_cs) sum[k] = 0;
    if (p.has_min | p.has_max) {
      mm[2 * k] = 0xffffffffu;
      mm[2 * k + 1] = 0u;
    }
  }
  for (int i = threadIdx.x; i < NR; i += blockDim.x) {
    const uint32_t c = p.part_count[(size_t)part * R + r0 + i];
    fill[i] = c < (uint32_t)p.part_cap ? c : (uint32_t)p.part_cap;
  }
  __syncthreads();
  const uint32_t vmask = p.part_vbits ? ((p.part_vbits >= 32) ? 0xffffffffu : ((1u << p.part_vbits) - 1u)) : 0u;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nwaves = blockDim.x >> 6;
  constexpr int RPW = 4;                          // regions per wave per step
  constexpr int PER = REC64 ? 2 : 4;              // records per 16-byte lane load
  constexpr uint32_t SPAN = 64 * PER;             // records per wave-load
  using Rec = typename std::conditional<REC64 != 0, unsigned long long, uint32_t>::type;
  const Rec* buf = reinterpret_cast<const Rec*>(p.part_buf);
  // the wave's steps: regions [b0, b0 + RPW) x record offsets `base` of them; the next step's loads are issued before
  // this step's atomics, so they are in flight while the LDS work runs (r5: half of kernel B's wave cycles waited)
  struct Step {
    int b0;
    uint32_t base, maxn;
    uint32_t nn[RPW];
  };
  auto regions_at = [&](Step& t, int b0) {
    for (; b0 < NR; b0 += nwaves * RPW) {  // the first group of regions with records
      t.b0 = b0;
      t.base = 0;
      t.maxn = 0;
#pragma unroll
      for (int q = 0; q < RPW; ++q) {
        t.nn[q] = (b0 + q < NR) ? (uint32_t)__builtin_amdgcn_readfirstlane(fill[b0 + q]) : 0u;  // (uniform: SGPRs)
        t.maxn = t.nn[q] > t.maxn ? t.nn[q] : t.maxn;
      }
      if (t.maxn) return;
    }
    t.b0 = NR;  // no step left
  };
  auto advance = [&](Step& t) {
    t.base += SPAN;
    if (t.base >= t.maxn) regions_at(t, t.b0 + nwaves * RPW);
  };
  // RPW buffer loads per step on every path (a region's own descriptor; a lane past the region's fill, or a step
  // past the last, gets an out-of-range offset: zeros, no access), so the compiler's wait for a step's loads can
  // leave the next step's in flight -- with the loads under branches the minimum over paths was no load at all
  auto load = [&](const Step& t, u32x4 (&v)[RPW]) {
    const bool live = t.b0 < NR;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const uint64_t base = (uint64_t)(uintptr_t)(buf + (live ? ((size_t)(r0 + t.b0 + q) * p.num_parts + part) *
                                                                    (size_t)p.part_cap : 0));
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          reinterpret_cast<void*>((uintptr_t)(((uint64_t)hi << 32) | (uint64_t)lo)), 0,
          __builtin_amdgcn_readfirstlane(p.part_cap * (int)sizeof(Rec)), 0x00020000);
      const uint32_t i0 = t.base + lane * PER;
      const uint32_t vo = (live && i0 < t.nn[q]) ? i0 * (uint32_t)sizeof(Rec) : 0x80000000u;
      v[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, vo, 0, 0));
    }
  };
  auto process = [&](const Step& t, const u32x4 (&v)[RPW]) {
    const uint32_t base = t.base;
    const uint32_t* nn = t.nn;
    // the step's RPW * PER records of this lane: key and value offset; a record past its region's fill goes to
    // the lane's dummy key KP + lane, so the atomics below run without per-record branches
    uint32_t rk[RPW * PER], rv[RPW * PER];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const uint32_t i0 = base + lane * PER;
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const unsigned long long r = REC64 ? ((unsigned long long)v[q][2 * e + 1] << 32) | v[q][2 * e]
                                           : (unsigned long long)v[q][e];
        uint32_t k, x;
        if (REC64) {
          k = (uint32_t)(r >> 32);
          x = (uint32_t)r;
        } else {
          k = (uint32_t)r >> p.part_vbits;
          x = (uint32_t)r & vmask;
        }
        rk[q * PER + e] = (i0 + e < nn[q]) ? k : KP + (uint32_t)lane;
        rv[q * PER + e] = x;
      }
    }
    constexpr int NREC = RPW * PER;
#pragma unroll
    for (int i = 0; i < NREC; ++i) {
      if (p.pack_cs) {
        atomicAdd(&cs[rk[i]], (1ull << 40) | (unsigned long long)rv[i]);
      } else {
        atomicAdd(&cnt[rk[i]], 1u);
        if (p.has_sum) atomicAdd(&sum[rk[i]], (unsigned long long)rv[i]);
      }
    }
    if (p.has_min | p.has_max) {
      if (p.mm_blind) {  // every record issues its MIN / MAX atomics (no return: nothing waits)
#pragma unroll
        for (int i = 0; i < NREC; ++i) {
          if (p.has_min) atomicMin(&mm[2 * rk[i]], rv[i]);
          if (p.has_max) atomicMax(&mm[2 * rk[i] + 1], rv[i]);
        }
      } else {
        // read the step's (min, max) words together; a record that improves one is rare after a key's first few
        // records (O(log n) of a key's n), but issuing its atomic in the record's own slot made the wave issue one
        // min and one max instruction for nearly every slot (some lane of 64 needs it: r5 SQ, 5.3 LDS instructions
        // per record against 2).  The lane's improving records go to a bitmask instead, and the wave issues one
        // atomicMin / atomicMax round per pending record of its busiest lane.
        unsigned long long cur[NREC];
#pragma unroll
        for (int i = 0; i < NREC; ++i) cur[i] = *reinterpret_cast<const unsigned long long*>(mm + 2 * rk[i]);
        uint32_t pmin = 0, pmax = 0;
#pragma unroll
        for (int i = 0; i < NREC; ++i) {
          if (p.has_min && rv[i] < (uint32_t)cur[i]) pmin |= 1u << i;
          if (p.has_max && rv[i] > (uint32_t)(cur[i] >> 32)) pmax |= 1u << i;
        }
        while (__ballot((pmin | pmax) != 0u)) {
          const uint32_t pm = pmin ? pmin : pmax;
          const int i = pm ? __builtin_ctz(pm) : 0;
          uint32_t key = 0, val = 0;
#pragma unroll
          for (int t = 0; t < NREC; ++t)  // register-indexed select (no dynamic register indexing)
            if (t == i) {
              key = rk[t];
              val = rv[t];
            }
          if (pmin) {
            atomicMin(&mm[2 * key], val);
            pmin &= pmin - 1u;
          } else if (pmax) {
            atomicMax(&mm[2 * key + 1], val);
            pmax &= pmax - 1u;
          }
        }
      }
    }
  };
  Step ta, tb;
  u32x4 va[RPW], vb[RPW];
  regions_at(ta, wave * RPW);
  load(ta, va);
  while (ta.b0 < NR) {  // wave-uniform
    tb = ta;
    advance(tb);
    load(tb, vb);
    process(ta, va);
    if (tb.b0 >= NR) break;
    ta = tb;
    advance(ta);
    load(ta, va);
    process(tb, vb);
  }
  __syncthreads();
  const bool shared_range = p.slices > 1;
  for (uint32_t k = threadIdx.x; k < KP; k += blockDim.x) {
    uint32_t c;
    int64_t s = 0;
    if (p.pack_cs) {
      const unsigned long long x = cs[k];
      c = (uint32_t)(x >> 40);
      s = (int64_t)(x & ((1ull << 40) - 1ull));
    } else {
      c = cnt[k];
      if (p.has_sum) s = (int64_t)sum[k];
    }
    if (!c) continue;
    const int64_t g = ((int64_t)part << p.part_klo) | k;
    if (g >= p.num_groups) continue;
    const int64_t vs = s + (int64_t)c * p.part_vbase;
    const int64_t vmin = p.part_vbase + (int64_t)mm[2 * k], vmax = p.part_vbase + (int64_t)mm[2 * k + 1];
    if (shared_range) {
      atomicAdd(&p.out_count[g], (unsigned long long)c);
      if (p.has_sum) atomicAdd(reinterpret_cast<unsigned long long*>(p.out_sum) + g, (unsigned long long)vs);
      if (p.has_min) atomicMin(reinterpret_cast<long long*>(p.out_min) + g, (long long)vmin);
      if (p.has_max) atomicMax(reinterpret_cast<long long*>(p.out_max) + g, (long long)vmax);
    } else {
      p.out_count[g] += c;  // this block owns keys [part << klo, (part + 1) << klo)
      if (p.has_sum) p.out_sum[g] += vs;
      if (p.has_min && vmin < p.out_min[g]) p.out_min[g] = vmin;
      if (p.has_max && vmax > p.out_max[g]) p.out_max[g] = vmax;
    }
  }
}

size_t part_agg_lds_bytes(const PartAggParams& p) {
  const size_t KP = ((size_t)1 << p.part_klo) + 64;  // + the per-lane dummy keys
  size_t o = p.pack_cs ? 8 * KP : 4 * KP;
  o = (o + 7) / 8 * 8;
  o += (p.has_sum && !p.pack_cs) ? 8 * KP : 0;
  o += (p.has_min | p.has_max) ? 8 * KP : 0;
  return o + 4 * (size_t)((p.regions + p.slices - 1) / p.slices);
}

void launch_part_agg(const PartAggParams& p, size_t lds, hipStream_t s) {
  const dim3 grid((unsigned)(p.num_parts * p.slices));
  if (p.rec64) {
    allow_lds(k_part_agg<1>, lds);
    hipLaunchKernelGGL(k_part_agg<1>, grid, dim3(1024), lds, s, p);
  } else {
    allow_lds(k_part_agg<0>, lds);
    hipLaunchKernelGGL(k_part_agg<0>, grid, dim3(1024), lds, s, p);
  }
  PH_HIP_CHECK(hipGetLastError());
}

__global__ void k_merge_overflow(const MergeParams p) {
  for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < p.n; g += (int64_t)gridDim.x * blockDim.x) {
    const unsigned long long c = p.ovf_count[g];
    if (!c) continue;
    p.out_count[g] += c;
    if (p.out_sum) p.out_sum[g] += p.ovf_sum[g];
    if (p.out_min && p.ovf_min[g] < p.out_min[g]) p.out_min[g] = p.ovf_min[g];
    if (p.out_max && p.ovf_max[g] > p.out_max[g]) p.out_max[g] = p.ovf_max[g];
  }
}

void launch_merge_overflow(const MergeParams& p, hipStream_t s) {
  const int grid = (int)std::min<int64_t>((p.n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_merge_overflow, dim3(grid), dim3(256), 0, s, p);
  PH_HIP_CHECK(hipGetLastError());
}


}  // namespace ph
