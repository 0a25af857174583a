// and_walk.h -- the chunked walks of an AND of SV scans' leap-frog (scan_and_walk.hip runs them on the device,
// filter_sim.cpp on the host for the CPU tests); the algorithm and its reference citations are in scan_and_walk.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ph {

constexpr int kWalkHead = 16;  // candidates a walker logs from its start
constexpr int kWalkTail = 16;  // candidates it logs at or past the next chunk
struct AndWalkJob {
  const unsigned long long* bits;  // k leaf doc bitmaps, leaf-major, nwords words each (bits past ndocs zero)
  int64_t nwords, ndocs;
  int32_t k, slot;                 // scans; the sum accumulates into out[slot]
  int32_t shift;                   // chunk = 1 << shift docs
  int64_t nchunks;
  int32_t* pos;                    // [kWalkHead + kWalkTail][nchunks] logged candidates (entry-major: the walkers
                                   // of a wave store one entry to consecutive addresses)
  unsigned long long* cum;         // their running sums, same layout
  uint32_t* cnt;                   // [nchunks] head count | tail count << 16
};

// index of log entry e (head: 0 .. kWalkHead - 1, tail: kWalkHead + i) of walker c
__host__ __device__ inline int64_t walk_slot(const AndWalkJob& J, int64_t c, int e) { return (int64_t)e * J.nchunks + c; }

// first set bit of bitmap `w` at or after x (x < nwords * 64), or -1
__host__ __device__ inline int64_t walk_next_set(const unsigned long long* w, int64_t nwords, int64_t x) {
  int64_t wi = x >> 6;
  unsigned long long v = w[wi] & (~0ull << (x & 63));
  while (!v) {
    if (++wi >= nwords) return -1;
    v = w[wi];
  }
  return wi * 64 + __builtin_ctzll(v);
}

// walker c: a fresh epoch at doc c << shift, logging as described in scan_and_walk.hip
__host__ __device__ inline void and_walk_chunk(const AndWalkJob& J, int64_t c) {
  const int64_t N = J.ndocs;
  const int k = J.k;
  const int64_t end = (c + 1) << J.shift;
  const int64_t thr = end < N ? end : N;  // the tail starts at the next chunk (the last walker's: the end)
  int64_t M = c << J.shift;
  int j = -1, hn = 0, tn = 0;
  unsigned long long cum = 0;
  for (;;) {
    bool term = false;
    int64_t nxt = 0;
    int jn = -1;
    if (M >= N) {  // scan 1's advance(numDocs) returns EOF at once
      cum += 1;
      term = true;
    } else {
      const int64_t wi = M >> 6;
      const unsigned long long bit = 1ull << (M & 63);
      int f = 0;
      while (f < k && (J.bits[(int64_t)f * J.nwords + wi] & bit)) ++f;
      if (f == k) {  // a match: k advance() calls (k - 1 after a move), minus the match
        cum += (unsigned long long)(k - 1 - (j >= 0 ? 1 : 0));
        nxt = M + 1;
      } else {
        cum += (unsigned long long)(f + 1 - ((j >= 0 && j < f) ? 1 : 0));
        nxt = walk_next_set(J.bits + (int64_t)f * J.nwords, J.nwords, M);
        term = nxt < 0 || nxt >= N;
        jn = f;
      }
    }
    const int32_t P = term ? (int32_t)N : (int32_t)M;  // the end is logged as candidate numDocs
    if (hn < kWalkHead) {
      J.pos[walk_slot(J, c, hn)] = P;
      J.cum[walk_slot(J, c, hn)] = cum;
      ++hn;
    }
    if (P >= thr) {
      J.pos[walk_slot(J, c, kWalkHead + tn)] = P;
      J.cum[walk_slot(J, c, kWalkHead + tn)] = cum;
      ++tn;
    }
    if (term || tn == kWalkTail) break;
    M = nxt;
    j = jn;
  }
  J.cnt[c] = (uint32_t)hn | ((uint32_t)tn << 16);
}

// where walker b's tail log meets walker b + 1's head log (the first common candidate): the index pair, or false
__host__ __device__ inline bool and_walk_meet(const AndWalkJob& J, int64_t b, int& ti, int& hi) {
  const int tn = (int)(J.cnt[b] >> 16), hn = (int)(J.cnt[b + 1] & 0xffff);
  int x = 0, y = 0;
  while (x < tn && y < hn) {
    const int32_t a = J.pos[walk_slot(J, b, kWalkHead + x)], h = J.pos[walk_slot(J, b + 1, y)];
    if (a == h) {
      ti = x;
      hi = y;
      return true;
    }
    if (a < h) ++x;
    else ++y;
  }
  return false;
}

// walker c's share of the true walk, cum_c(q_{c+1}) - cum_c(q_c); false when the walks do not meet in order
__host__ __device__ inline bool and_merge_chunk(const AndWalkJob& J, int64_t c, unsigned long long& part) {
  int64_t qc = -1, qn = -1;
  unsigned long long lo = 0, hi = 0;
  int ti = 0, h = 0;
  if (c > 0) {  // q_c: the true walk joins walker c
    if (!and_walk_meet(J, c - 1, ti, h)) return false;
    qc = J.pos[walk_slot(J, c, h)];
    lo = J.cum[walk_slot(J, c, h)];
  }
  if (c + 1 < J.nchunks) {  // q_{c+1}: walker c + 1 takes over
    if (!and_walk_meet(J, c, ti, h)) return false;
    qn = J.pos[walk_slot(J, c, kWalkHead + ti)];
    hi = J.cum[walk_slot(J, c, kWalkHead + ti)];
  } else {  // the last walker runs to the end: its tail holds the end alone
    const int tn = (int)(J.cnt[c] >> 16);
    if (tn < 1) return false;
    qn = J.pos[walk_slot(J, c, kWalkHead + tn - 1)];
    hi = J.cum[walk_slot(J, c, kWalkHead + tn - 1)];
  }
  if (qn < qc) return false;
  part = hi - lo;
  return true;
}

}  // namespace ph
