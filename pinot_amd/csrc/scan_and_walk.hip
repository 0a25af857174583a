// scan_and_walk.hip -- numEntriesScannedInFilter of an AND of SV scans only, as chunked walks of the AND's leap-frog.
//
// AndDocIdSet.iterator returns AndDocIdIterator(scan_1 .. scan_k) for such an AND (AndDocIdSet.java:180-183), and
// DocIdSetOperator drains it with next().  AndDocIdIterator.next() (AndDocIdIterator.java:40-67) keeps a candidate M
// (maxDocId) and calls advance(M) on the scans in order, skipping the one that set M; a scan's advance(t)
// (SVScanDocIdIterator.java:101-112) examines the docs t .. its next match (or the rest of the segment at EOF).  So one
// "epoch" at candidate M that the scan j set (j = -1 right after a match, or at the start) costs
//   calls(M, j) = f + 1 - [0 <= j < f]   advance() calls, f = the first scan without M, and moves M to scan f's next
//                                        match after M (or ends the segment: that call returns EOF);
//   calls(M, j) = k - [j >= 0]           when every scan has M (a match): the next epoch is M + 1 with j = -1;
//   1                                    for M = numDocs (scan 1's advance returns EOF at once),
// and the docs the calls examine telescope to  entries = numDocs - |matches| + calls - 1  =  numDocs - 1 + sum over the
// epochs of (calls - [match]).  The candidate sequence M_0 = 0, M_1, ... is a walk whose next step depends on M only
// (f and the next match do; the setter only changes an epoch's call count), so two walks that meet at one candidate
// agree from there on.  That makes the sum parallel:
//   k_and_walk   -- walker c starts a fresh epoch at doc c * L (one thread per chunk of L docs) and logs its first
//                   kWalkHead candidates and the first kWalkTail candidates at or past the next chunk (each with its running
//                   sum, the epoch included), stopping there or at the end (candidate numDocs);
//   k_and_merge  -- the true walk (walker 0's) meets walker c at q_c = the first candidate of walker c-1's tail log
//                   that walker c's head log holds; walker c owns the true epochs after q_c up to q_{c+1}:
//                   sum = cum_0(q_1) + sum_c (cum_c(q_{c+1}) - cum_c(q_c)).  A chunk whose walks do not meet inside the
//                   logs (or meet out of order) marks the job: the host reruns it with L x 4 (L >= numDocs is one
//                   walker: always exact).
// Algorithmic bytes: the k leaf bitmaps (k * numDocs / 8), read once per walk plus the logs; the host checks these
// sums against the iterator simulation in the parity tests (filter_sim.cpp, oracle.filter_entries).
#include "ph_internal.h"

namespace ph {

// and_walk_chunk with the k leaves' words of the walk's current 64-doc word AND of the next one held in registers: a
// step inside the word is register work (the first scan without M, the next match of scan f), a candidate that moves
// on to the next word swaps the next word's set in and issues the loads of the one after (waited on only when that
// word is reached: r4's one-word form stalled the wave on a reload in most iterations, some lane always crossing a
// word), and only a jump of two words or more loads on the spot.  Up to K leaves (the padding leaves read as
// all-ones, so they never fail); the logs are the same as and_walk_chunk's (the host version the CPU tests run).
template <int K>
__global__ void __launch_bounds__(256) k_and_walk(const AndWalkJob* __restrict__ jobs) {
  const AndWalkJob J = jobs[blockIdx.y];
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= J.nchunks) return;
  const int64_t N = J.ndocs, nwords = J.nwords;
  const int k = J.k;
  const int64_t end = (c + 1) << J.shift;
  const int64_t thr = end < N ? end : N;
  int64_t M = c << J.shift;
  int j = -1, hn = 0, tn = 0;
  unsigned long long cum = 0;
  unsigned long long W[K], X[K];  // words cw and cw + 1 of every leaf
  int64_t cw = M >> 6;
  auto load = [&](int64_t w, unsigned long long (&R)[K]) {
#pragma unroll
    for (int i = 0; i < K; ++i) R[i] = i >= k ? ~0ull : (w < nwords ? J.bits[(int64_t)i * nwords + w] : 0ull);
  };
  if (M < N) {
    load(cw, W);
    load(cw + 1, X);
  }
  for (;;) {
    bool term = false;
    int64_t nxt = 0;
    int jn = -1;
    if (M >= N) {
      cum += 1;
      term = true;
    } else {
      const int b = (int)(M & 63);
      int f = K;
#pragma unroll
      for (int i = K - 1; i >= 0; --i)
        if (!((W[i] >> b) & 1ull)) f = i;
      if (f == K) {
        cum += (unsigned long long)(k - 1 - (j >= 0 ? 1 : 0));
        nxt = M + 1;
      } else {
        cum += (unsigned long long)(f + 1 - ((j >= 0 && j < f) ? 1 : 0));
        unsigned long long v = 0, vx = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
          v = i == f ? W[i] : v;
          vx = i == f ? X[i] : vx;
        }
        v &= ~0ull << b;
        int64_t wi = cw;
        if (!v) {  // the next word from registers, then memory
          v = vx;
          ++wi;
          const unsigned long long* bf = J.bits + (int64_t)f * nwords;
          while (!v && ++wi < nwords) v = bf[wi];
        }
        nxt = (v && wi < nwords) ? wi * 64 + __builtin_ctzll(v) : N;
        term = nxt >= N;
        jn = f;
      }
    }
    const int32_t P = term ? (int32_t)N : (int32_t)M;
    if (hn < kWalkHead) {  // entry-major logs: the wave's walkers store to consecutive addresses
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
    const int64_t mw = M >> 6;
    if (mw != cw && M < N) {
      if (mw == cw + 1) {
#pragma unroll
        for (int i = 0; i < K; ++i) W[i] = X[i];
      } else {
        load(mw, W);
      }
      cw = mw;
      load(cw + 1, X);
    }
  }
  J.cnt[c] = (uint32_t)hn | ((uint32_t)tn << 16);
}

__global__ void __launch_bounds__(256) k_and_merge(const AndWalkJob* __restrict__ jobs, unsigned long long* out,
                                                   uint32_t* bad) {
  const AndWalkJob J = jobs[blockIdx.y];
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  unsigned long long part = 0;
  const bool fail = c < J.nchunks && !and_merge_chunk(J, c, part);
  for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
  const unsigned long long anyfail = __ballot(fail);
  if ((threadIdx.x & 63) == 0) {
    if (part) atomicAdd(out + J.slot, part);
    if (anyfail) atomicOr(bad + J.slot, 1u);
  }
}

void launch_and_walk(const AndWalkJob* jobs, int32_t njobs, int64_t max_chunks, int32_t max_k, unsigned long long* out,
                     uint32_t* bad, hipStream_t s) {
  if (njobs <= 0 || max_chunks <= 0) return;
  if (max_k > kMaxFbProgs) fail(PH_ERR_DEVICE, "AND walk wider than kMaxFbProgs scans");
  const dim3 grid((unsigned)((max_chunks + 255) / 256), (unsigned)njobs);
  // the widest AND of the launch picks the register set (ST_SCANAND: at most kMaxFbProgs scans)
  if (max_k <= 4) hipLaunchKernelGGL(k_and_walk<4>, grid, dim3(256), 0, s, jobs);
  else if (max_k <= 8) hipLaunchKernelGGL(k_and_walk<8>, grid, dim3(256), 0, s, jobs);
  else hipLaunchKernelGGL(k_and_walk<kMaxFbProgs>, grid, dim3(256), 0, s, jobs);
  PH_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_and_merge, grid, dim3(256), 0, s, jobs, out, bad);
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph
