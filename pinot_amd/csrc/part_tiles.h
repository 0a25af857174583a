// part_tiles.h -- the register-direct tile reader of the partitioned group-by's kernel A (k_part_reg,
// scan_partition_reg.hip).
//
// A workgroup walks its share of the launch's chunks in rounds; in a round each of its waves takes one tile of
// kRegTileWords 64-doc words (2048 docs) and lane l owns the 32 CONSECUTIVE docs [32 l, 32 l + 32) of it, so its b-bit
// values of any stream are exactly b whole dwords: ceil(b / 4) 16-byte buffer loads per stream straight into registers
// (reg_load), decoded with compile-time bit positions (reg_decode).  decode() turns the tile into one 32-bit record
// per doc -- (key << (32 - klo)) + value offset -- and the doc's ring-word index (key >> klo, or the lane's scratch
// word P + lane for a missed or out-of-range doc), packed two per register.
#pragma once
#include "reg_decode.h"

namespace ph {

template <int NG, int HASV, int CK, int CV>
struct PartTiles {
  struct Tile {
    SegPtr S;
    int32_t w0, ndoc;  // first word; docs of this tile the wave owns (<= 2048, clipped to the segment)
  };
  const KParams& p;
  const PH_CONST Chunk* chunks;
  SegPtr segs;
  int32_t c, r, c_end, wave;
  u32x4 pf[CK], pk[NG][CK], pv[HASV ? CV : 1];  // the tile's loads (filter, keys, value)

  __device__ PartTiles(const KParams& kp, int wv, int32_t blk, int32_t nblk) : p(kp), wave(wv) {
    chunks = (const PH_CONST Chunk*)p.chunks;
    segs = (SegPtr)p.segs;
    const int64_t nch = p.chunk_end - p.chunk_begin;
    c = p.chunk_begin + (int32_t)(nch * blk / nblk);
    c_end = p.chunk_begin + (int32_t)(nch * (blk + 1) / nblk);
    r = 0;
  }

  // rounds of this workgroup (every wave runs all of them; a wave past its chunk's words gets an empty tile)
  __device__ __forceinline__ int32_t rounds() const {
    constexpr int32_t round_words = kRegWaves * kRegTileWords;
    int32_t n = 0;
    for (int32_t cc = c; cc < c_end; ++cc) n += (chunks[cc].word_end - chunks[cc].word_begin + round_words - 1) / round_words;
    return n;
  }

  __device__ __forceinline__ Tile next() {
    constexpr int32_t round_words = kRegWaves * kRegTileWords;
    Tile t{nullptr, 0, 0};
    if (c < c_end) {
      const int32_t cbeg = chunks[c].word_begin, cend = chunks[c].word_end;
      t.S = segs + chunks[c].seg;
      t.w0 = cbeg + r * round_words + wave * kRegTileWords;
      const int32_t nw = min(kRegTileWords, cend - t.w0);
      t.ndoc = nw > 0 ? min(nw * 64, t.S->num_docs - t.w0 * 64) : 0;
      if (cbeg + (r + 1) * round_words < cend) {
        ++r;
      } else {
        ++c;
        r = 0;
      }
    }
    return t;
  }

  // issue the tile's loads (they stay in flight until decode)
  __device__ __forceinline__ void load(const Tile& t, int lane) {
    load_keys(t, lane);
    load_value(t, lane);
  }
  __device__ __forceinline__ void load_keys(const Tile& t, int lane) {
    const bool tile = t.ndoc > 0;                        // wave-uniform
    const bool lane_live = tile && lane * 32 < t.ndoc;  // this lane's run holds docs of the tile
    const int32_t run0 = t.w0 * 2;
    SegPtr S = t.S;
    auto bytes = [&](int st) { return ((int64_t)S->num_docs * S->streams[st].bits + 7) / 8; };
    const bool rng = tile && S->fkind == FK_RANGE;
    const int fs = p.f_stream;
    reg_load<CK>(rng, lane_live, rng ? S->streams[fs].fwd : nullptr, rng ? S->streams[fs].bits : 0,
                 rng ? bytes(fs) : 0, run0, lane, pf);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int gs = p.g_stream[g];
      reg_load<CK>(tile, lane_live, tile ? S->streams[gs].fwd : nullptr, tile ? S->streams[gs].bits : 0,
                   tile ? bytes(gs) : 0, run0, lane, pk[g]);
    }
  }
  __device__ __forceinline__ void load_value(const Tile& t, int lane) {
    const bool tile = t.ndoc > 0;
    const bool lane_live = tile && lane * 32 < t.ndoc;
    const int32_t run0 = t.w0 * 2;
    SegPtr S = t.S;
    auto bytes = [&](int st) { return ((int64_t)S->num_docs * S->streams[st].bits + 7) / 8; };
    if constexpr (HASV != 0) {
      const int vs = p.v_stream[0];
      reg_load<CV>(tile, lane_live, tile ? S->streams[vs].fwd : nullptr, tile ? S->streams[vs].bits : 0,
                   tile ? bytes(vs) : 0, run0, lane, pv);
    }
  }

  // decode the loaded tile: keys into X (mixed radix), the filter turns each into its 16-bit ring-word index in PB
  // (the partition key >> klo, or the lane's scratch word P + lane for a missed doc), then the value phase turns each
  // key into its record in place, (key << (32 - klo)) + value offset: the shift drops the partition bits, and kernel B
  // reads the key as record >> (32 - klo) (peak: 48 registers + the loads)
  __device__ __forceinline__ void decode(const Tile& t, int lane, uint32_t (&X)[32], uint32_t (&PB)[16]) const {
    const uint32_t klo = (uint32_t)p.part_klo, rsh = 32u - klo;
    const uint32_t dummy = (uint32_t)p.num_parts + (uint32_t)lane;
    if (t.ndoc <= 0) {
      static_for<0, 16>([&](auto j) { PB[j] = dummy | (dummy << 16); });
      return;
    }
    SegPtr S = t.S;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const uint32_t st = (uint32_t)p.group_stride[g];
      if (g == 0) reg_decode<CK>(pk[g], S->streams[p.g_stream[g]].bits, [&](auto j, uint32_t v) { X[j] = __umul24(v, st); });
      else reg_decode<CK>(pk[g], S->streams[p.g_stream[g]].bits, [&](auto j, uint32_t v) { X[j] += __umul24(v, st); });
    }
    auto put = [&](auto j, bool pass) {
      constexpr int J = decltype(j)::value;
      const uint32_t b = pass ? (X[J] >> klo) : dummy;
      if constexpr ((J & 1) == 0) PB[J >> 1] = b;
      else PB[J >> 1] |= b << 16;
    };
    const int fk = S->fkind;
    const uint32_t flo = S->flo, flen = S->flen;
    if (fk == FK_RANGE) {
      reg_decode<CK>(pf, S->streams[p.f_stream].bits, [&](auto j, uint32_t v) { put(j, (v - flo) < flen); });
    } else if (fk == FK_DOCRANGE) {
      const uint32_t d0 = (uint32_t)t.w0 * 64u + (uint32_t)lane * 32u;
      static_for<0, 32>([&](auto j) { put(j, (d0 + (uint32_t)decltype(j)::value - flo) < flen); });
    } else {
      static_for<0, 32>([&](auto j) { put(j, true); });
    }
    if (t.ndoc < 64 * kRegTileWords) {  // a segment's last tile (wave-uniform): docs past its end append nothing
      const int32_t nv = t.ndoc - lane * 32;
      static_for<0, 32>([&](auto j) {
        constexpr int J = decltype(j)::value;
        if (J >= nv) PB[J >> 1] = (J & 1) ? ((PB[J >> 1] & 0xffffu) | (dummy << 16)) : ((PB[J >> 1] & 0xffff0000u) | dummy);
      });
    }
    if constexpr (HASV != 0) {
      const uint32_t vadd = (uint32_t)(S->vals[0].base - p.part_vbase);
      reg_decode<CV>(pv, S->streams[p.v_stream[0]].bits, [&](auto j, uint32_t v) { X[j] = (X[j] << rsh) + (v + vadd); });
    } else {
      static_for<0, 32>([&](auto j) { X[j] <<= rsh; });
    }
  }
};

// the partition index of record j of a lane (PB packs two 16-bit indices per register)
template <int J>
__device__ __forceinline__ uint32_t part_of(const uint32_t (&PB)[16]) {
  return (J & 1) ? (PB[J >> 1] >> 16) : (PB[J >> 1] & 0xffffu);
}

}  // namespace ph
