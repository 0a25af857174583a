// and_walk.h -- numEntriesScannedInFilter of an AND of SV scans only, as a composition of per-chunk transition tables
// of the AND's leap-frog (scan_and_walk.hip runs it on the device, filter_sim.cpp on the host for the CPU tests).
//
// AndDocIdSet.iterator returns AndDocIdIterator(scan_1 .. scan_k) for such an AND (AndDocIdSet.java:180-183), and
// DocIdSetOperator drains it with next().  AndDocIdIterator.next() (AndDocIdIterator.java:40-67) keeps a candidate M
// (maxDocId) and calls advance(M) on the scans in order, skipping the one that set M; a scan's advance(t)
// (SVScanDocIdIterator.java:101-112) examines the docs t .. its next match (or the rest of the segment at EOF).  So one
// "epoch" at candidate M that scan j set (j = -1 right after a match, or at the start) costs
//   calls(M, j) = f + 1 - [0 <= j < f]   advance() calls, f = the first scan without M, and moves M to scan f's next
//                                        match after M (or ends the segment: that call returns EOF);
//   calls(M, j) = k - [j >= 0]           when every scan has M (a match): the next epoch is M + 1 with j = -1;
//   1                                    for M = numDocs (scan 1's advance returns EOF at once),
// and the docs the calls examine telescope to  entries = numDocs - 1 + sum over the epochs of (calls - [match]).
//
// The walk as a finite automaton over chunks of L docs.  The true walk enters chunk [c0, c1) in one of k + 1 ways: a
// fresh epoch at c0 (type -1: the previous chunk ended with a match at c0 - 1, or c0 = 0), or a jump by scan i that
// found no match of its own in the previous chunk (type i: the epoch at scan i's first match >= c0, set by i --
// because scan i had no match in [M_prev, c0), its next match after M_prev IS its first match >= c0).  From an entry
// the walk inside the chunk is fixed, and it leaves the chunk in one of the same k + 1 ways.  So every chunk is a
// table  type -> (exit type, sum of (calls - [match]) of its epochs),  the tables compose associatively, and the
// segment's sum is the composition applied to type -1 at doc 0, plus 1 if it ends in type -1 (the epoch at numDocs).
// No speculation, no logs, no reruns: exact for every input.  A chunk computes its table with one full walk (type -1)
// whose first kDfaHist candidates it remembers; the other types' walks stop at the first of those they reach (the
// candidate sequence depends on M only -- the setter changes only an epoch's call count -- so two walks that share a
// candidate agree from there on) and take the rest from the remembered running sums.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace ph {

constexpr int kDfaChunkWords = 4;  // default chunk = 4 words of 64 docs = 256 docs (and_dfa_chunk_words())
constexpr int kDfaHist = 8;        // candidates of the type -1 walk a chunk remembers

struct AndWalkJob {
  const unsigned long long* bits;  // k leaf doc bitmaps, leaf-major, nwords words each (bits past ndocs zero)
  int64_t nwords, ndocs;
  int32_t k, slot;                 // scans; the sum goes to out[slot]
  int64_t nchunks;                 // chunks of kDfaChunkWords words
  int32_t ngroups;                 // workgroup tables (chunks composed per workgroup on the device)
  int32_t pad;
  uint32_t* gdelta;                // [k + 1][ngroups] the workgroups' composed sums (row = entry type + 1)
  uint8_t* gexit;                  // [k + 1][ngroups] their exit types + 1
};

// One chunk's walker: the k scans' words through get(i, w) (absolute word index inside the chunk [c0, c1)).  The k
// words of the current candidate's 64-doc word stay in registers (read at compile-time indices only: the device keeps
// them in VGPRs), so an epoch inside the word is register work; a candidate in another word reloads them.  Doc
// positions are 32-bit (a segment's docIds are Java ints), which halves the walk's integer work on the device.
template <int K, class Get>
struct DfaWalker {
  int k;
  int32_t c1;
  Get get;
  int32_t cw = -1;          // word held in Wc
  unsigned long long Wc[K];
  unsigned long long Pc[K];  // prefix ANDs Wc[0] & .. & Wc[i]: bit b of Pc[i] = scans 0..i all have doc b
  __host__ __device__ void hold(int32_t w) {
    if (w == cw) return;
    cw = w;
    unsigned long long a = ~0ull;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      Wc[i] = i < k ? get(i, w) : ~0ull;
      a &= Wc[i];
      Pc[i] = a;
    }
  }
  // scan i's first match in [x, c1), or -1
  __host__ __device__ int32_t next_set(int i, int32_t x) {
    if (x >= c1) return -1;
    int32_t w = x >> 6;
    const int32_t wl = (c1 - 1) >> 6;
    unsigned long long v = 0;
    if (w == cw) {
#pragma unroll
      for (int y = 0; y < K; ++y)
        if (y == i) v = Wc[y];
    } else {
      v = get(i, w);
    }
    v &= ~0ull << (x & 63);
    while (v == 0ull) {
      if (++w > wl) return -1;
      v = get(i, w);
    }
    const int32_t m = w * 64 + (int32_t)__builtin_ctzll(v);
    return m < c1 ? m : -1;
  }
  // one epoch at M set by scan j (-1: none): returns its (calls - [match]) and sets the next candidate (-1: the walk
  // leaves the chunk) and its setter
  __host__ __device__ uint32_t epoch(int32_t M, int j, int32_t& nxt, int& jn) {
    hold(M >> 6);
    const int b = (int)(M & 63);
    // first scan without doc M (k: every scan has it) = how many of the nested prefix ANDs still hold doc M
    int f = 0;
#pragma unroll
    for (int i = 0; i < K; ++i)
      if (i < k) f += (int)((Pc[i] >> b) & 1ull);
    const uint32_t skip = (j >= 0) ? 1u : 0u;
    if (f == k) {
      nxt = M + 1 < c1 ? M + 1 : -1;
      jn = -1;
      return (uint32_t)k - 1u - skip;
    }
    nxt = next_set(f, M + 1);
    jn = f;
    return (uint32_t)f + 1u - ((skip != 0u && j < f) ? 1u : 0u);
  }
};

// One chunk's table: delta[e + 1] / ext[e + 1] for entry type e = -1 .. k - 1 (ext = exit type + 1).
template <int K, class Get>
__host__ __device__ inline void dfa_chunk(int k, int64_t c0, int64_t c1, Get&& get, uint32_t (&delta)[K + 1],
                                          uint8_t (&ext)[K + 1]) {
  DfaWalker<K, Get&> W{k, (int32_t)c1, get};
  // type -1: the full walk from c0, remembering its first kDfaHist candidates and the running sums around their
  // epochs (hcum[q]: before candidate q's epoch, hcum[q + 1]: after it)
  int32_t hpos[kDfaHist];
  uint32_t hcum[kDfaHist + 1];
  int nh = 0;
  uint32_t total = 0;
  uint8_t ext0 = 0;
  {
    int32_t M = (int32_t)c0;
    int j = -1;
    // (register arrays written and read at compile-time indices only: the device keeps them in VGPRs)
    for (;;) {
      const uint32_t before = total;
      int32_t nxt = -1;
      int jn = -1;
      total += W.epoch(M, j, nxt, jn);
      if (nh < kDfaHist) {  // (a branch: past the first kDfaHist epochs the wave skips the selects)
#pragma unroll
        for (int h = 0; h < kDfaHist; ++h)
          if (h == nh) {
            hpos[h] = M;
            hcum[h] = before;
            hcum[h + 1] = total;
          }
        nh += 1;
      }
      if (nxt < 0) {
        ext0 = (uint8_t)(jn + 1);
        break;
      }
      M = nxt;
      j = jn;
    }
  }
  delta[0] = total;
  ext[0] = ext0;
  // types 0 .. k - 1: from scan e's first match, until a remembered candidate of the type -1 walk
  for (int e = 0; e < K; ++e) {
    if (e >= k) break;
    uint32_t de = 0;
    uint8_t xe = (uint8_t)(e + 1);
    int32_t M = W.next_set(e, (int32_t)c0);
    if (M >= 0) {  // else: no match of scan e in the chunk, the jump passes through
      int j = e;
      for (;;) {
        int32_t nxt = -1;
        int jn = -1;
        const uint32_t d = W.epoch(M, j, nxt, jn);
        uint32_t after = 0;
        bool joined = false;
#pragma unroll
        for (int h = 0; h < kDfaHist; ++h)
          if (h < nh && hpos[h] == M) {
            joined = true;
            after = total - hcum[h + 1];
          }
        if (joined) {  // joined the type -1 walk at one of its remembered candidates: its epochs after it follow
          de += d + after;
          xe = ext0;
          break;
        }
        de += d;
        if (nxt < 0) {
          xe = (uint8_t)(jn + 1);
          break;
        }
        M = nxt;
        j = jn;
      }
    }
#pragma unroll
    for (int y = 1; y <= K; ++y)
      if (y == e + 1) {
        delta[y] = de;
        ext[y] = xe;
      }
  }
}

// One 64-doc word's table (the device form for ANDs of <= 4 scans, r6): the same automaton with the word as the
// chunk, so a chunk's table is its words' tables composed in order.  Every walk stays inside the k scans' words in
// registers (no word switches, no LDS); W[i] for k <= i < K are all-ones fillers (never the first scan without a doc),
// bits at or past c1 (the docs of the word) are zero.  The type -1 walk only marks its candidates (V) and the epochs
// whose setter is skipped (S): an epoch's (calls - [match]) is f + 1 - skip, or k - 1 - skip for a match, and f is
// the number of nested prefix ANDs holding the doc, so the sum of any run of its epochs is a handful of masked
// popcounts.  Another type's walk that reaches one of its candidates M takes the rest as that sum above M (the walks
// agree after a shared candidate).
template <int K>
__host__ __device__ inline void dfa_word(int k, const unsigned long long (&W)[K], int32_t c1, uint32_t (&delta)[K + 1],
                                         uint8_t (&ext)[K + 1]) {
  static_assert(K <= 4, "ANDs of at most 4 scans");
  unsigned long long P[K];
  {
    unsigned long long a = ~0ull;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      a &= W[i];
      P[i] = a;
    }
  }
  // the first scan without doc M (>= k: a match; fillers only add to it past k)
  auto level = [&](int32_t M) {
    int f = 0;
#pragma unroll
    for (int i = 0; i < K; ++i) f += (int)((P[i] >> M) & 1ull);
    return f;
  };
  // scan f's next match after M, or -1
  auto seek = [&](int f, int32_t M) -> int32_t {
    unsigned long long v = 0;
#pragma unroll
    for (int y = 0; y < K; ++y)
      if (y == f) v = W[y];
    v &= (~0ull << M) << 1;
    return v ? (int32_t)__builtin_ctzll(v) : -1;
  };
  // the type -1 walk from doc 0 of the word
  unsigned long long V = 0, S = 0;
  uint8_t x0 = 0;
  {
    int32_t M = 0;
    int j = -1;
    for (;;) {  // (branch-free body: the match and seek successors are both computed, then selected)
      const int f = level(M);
      const unsigned long long bit = 1ull << M;
      V |= bit;
      S |= (j >= 0 && j < f) ? bit : 0ull;  // (j < k <= f for a match: skipped whenever a scan set M)
      const bool match = f >= k;
      const int32_t sk = seek(match ? 0 : f, M);
      const int32_t nm = M + 1 < c1 ? M + 1 : -1;
      const int32_t nxt = match ? nm : sk;
      j = match ? -1 : f;
      if (nxt < 0) {
        x0 = (uint8_t)(j + 1);
        break;
      }
      M = nxt;
    }
  }
  // the type -1 epochs' sum over the candidates in `sel`: sum of (f + 1) - 2 per match - skips
  auto run_sum = [&](unsigned long long sel) -> uint32_t {
    const unsigned long long v = V & sel;
    uint32_t t = (uint32_t)__builtin_popcountll(v) - (uint32_t)__builtin_popcountll(S & sel);
    unsigned long long last = 0;
#pragma unroll
    for (int i = 0; i < K; ++i)
      if (i < k) {
        t += (uint32_t)__builtin_popcountll(v & P[i]);
        last = P[i];
      }
    return t - 2u * (uint32_t)__builtin_popcountll(v & last);
  };
  delta[0] = run_sum(~0ull);
  ext[0] = x0;
#pragma unroll
  for (int e = 0; e < K; ++e) {
    uint32_t de = 0;
    uint8_t xe = (uint8_t)(e + 1);
    if (e < k && W[e] != 0ull) {  // else the jump passes through the word
      int32_t M = (int32_t)__builtin_ctzll(W[e]);
      int j = e;
      int32_t joined = -1;
      for (;;) {  // (branch-free body, as the type -1 walk's)
        const int f = level(M);
        const uint32_t skip = (j >= 0 && j < f) ? 1u : 0u;
        const bool match = f >= k;
        de += (match ? (uint32_t)k - 2u : (uint32_t)f) + 1u - skip;
        const int32_t sk = seek(match ? 0 : f, M);
        const int32_t nm = M + 1 < c1 ? M + 1 : -1;
        const int32_t nxt = match ? nm : sk;
        const int jn = match ? -1 : f;
        if ((V >> M) & 1ull) {  // a type -1 candidate: its epochs after M follow
          joined = M;
          break;
        }
        if (nxt < 0) {
          xe = (uint8_t)(jn + 1);
          break;
        }
        M = nxt;
        j = jn;
      }
      if (joined >= 0) {
        de += run_sum((~0ull << joined) << 1);
        xe = x0;
      }
    }
    delta[e + 1] = de;
    ext[e + 1] = xe;
  }
}

// compose table b after table a (both k + 1 entries): out[e] = b applied to a's exit of e
template <int K>
__host__ __device__ inline void dfa_compose(int k, const uint32_t (&ad)[K + 1], const uint8_t (&ax)[K + 1],
                                            const uint32_t (&bd)[K + 1], const uint8_t (&bx)[K + 1],
                                            uint32_t (&od)[K + 1], uint8_t (&ox)[K + 1]) {
  for (int e = 0; e <= K; ++e) {
    if (e > k) break;
    const int x = ax[e];
    uint32_t d = 0;
    uint8_t t = 0;
    for (int y = 0; y <= K; ++y)  // register-indexed select (no dynamic register indexing on the device)
      if (y == x) {
        d = bd[y];
        t = bx[y];
      }
    od[e] = ad[e] + d;
    ox[e] = t;
  }
}

// the segment's entries from its composed table: entry type -1 at doc 0, + 1 for an end in type -1 (the epoch at
// numDocs), over numDocs - 1
inline int64_t dfa_entries(int64_t num_docs, uint32_t delta_m1, uint8_t exit_m1) {
  return num_docs - 1 + (int64_t)delta_m1 + (exit_m1 == 0 ? 1 : 0);
}

}  // namespace ph
