// scan_and_walk.hip -- numEntriesScannedInFilter of an AND of SV scans only: the leap-frog of AndDocIdIterator as a
// composition of per-chunk transition tables (the algorithm and its reference citations are in and_walk.h).
//
//   k_and_dfa      -- one thread per 512-doc chunk: the chunk's k leaf bitmap words are staged in LDS by the
//                     workgroup (coalesced), the thread computes the chunk's table (dfa_chunk: one full walk and the
//                     other entry types' walks up to where they join it), and the workgroup composes its chunks'
//                     tables in a tree into one table per workgroup;
//   k_and_compose  -- one wave per job composes the job's workgroup tables in order, from entry type -1 at doc 0.
// Exact for every input (no speculative walks, no reruns).  Algorithmic bytes: the k leaf bitmaps (k * numDocs / 8),
// read once.  The host runs the same dfa_chunk over the same tables (filter_sim.cpp, phx_and_walk_entries) and the
// parity tests check both against the iterator simulation and the oracle's restatement.
#include "scan_kernel.h"

namespace ph {

// the workgroup's chunk tables composed in order, thread 0 storing the workgroup's table: a butterfly of shuffles
// inside each wave (r6; r5 ran all 7 levels through LDS with a barrier each), then thread 0 over the waves' tables
template <int K, int BLOCK>
__device__ __forceinline__ void dfa_group_compose(const AndWalkJob& J, int64_t g, uint32_t (&d)[K + 1],
                                                  uint8_t (&x)[K + 1], unsigned char* smem) {
  constexpr int NW = BLOCK / 64;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    uint32_t bd[K + 1];
    uint8_t bx[K + 1];
#pragma unroll
    for (int e = 0; e <= K; ++e) {
      bd[e] = (uint32_t)__shfl_down((int)d[e], s, 64);
      bx[e] = (uint8_t)__shfl_down((int)x[e], s, 64);
    }
    if ((lane & (2 * s - 1)) == 0) {  // lane + s < 64: the next run of lanes, in chunk order
      uint32_t od[K + 1];
      uint8_t ox[K + 1];
      dfa_compose<K>(K, d, x, bd, bx, od, ox);
#pragma unroll
      for (int e = 0; e <= K; ++e) {
        d[e] = od[e];
        x[e] = ox[e];
      }
    }
  }
  uint32_t* td = reinterpret_cast<uint32_t*>(smem);                           // [NW][K + 1]
  uint8_t* tx = reinterpret_cast<uint8_t*>(smem + (size_t)NW * (K + 1) * 4);  // [NW][K + 1]
  if (lane == 0)
#pragma unroll
    for (int e = 0; e <= K; ++e) {
      td[wave * (K + 1) + e] = d[e];
      tx[wave * (K + 1) + e] = x[e];
    }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < NW; ++w) {
      uint32_t bd[K + 1], od[K + 1];
      uint8_t bx[K + 1], ox[K + 1];
#pragma unroll
      for (int e = 0; e <= K; ++e) {
        bd[e] = td[w * (K + 1) + e];
        bx[e] = tx[w * (K + 1) + e];
      }
      dfa_compose<K>(K, d, x, bd, bx, od, ox);
#pragma unroll
      for (int e = 0; e <= K; ++e) {
        d[e] = od[e];
        x[e] = ox[e];
      }
    }
    for (int e = 0; e <= J.k; ++e) {
      J.gdelta[(int64_t)e * J.ngroups + g] = d[e];
      J.gexit[(int64_t)e * J.ngroups + g] = x[e];
    }
  }
}

template <int K, int BLOCK, int CW>
__global__ void __launch_bounds__(BLOCK) k_and_dfa(const AndWalkJob* __restrict__ jobs) {
  constexpr int ST = CW + 1;  // chunk words in LDS with one word of padding (bank spread)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long* words = reinterpret_cast<unsigned long long*>(smem);  // [K][BLOCK * ST]
  const AndWalkJob& J = jobs[blockIdx.y];
  const int64_t g = blockIdx.x;
  if (g >= J.ngroups) return;  // uniform over the workgroup
  const int k = J.k;
  const int64_t N = J.ndocs, nwords = J.nwords;
  const int64_t w0 = g * (int64_t)BLOCK * CW;  // the workgroup's first word
  for (int i = 0; i < k; ++i) {
    const unsigned long long* src = J.bits + (int64_t)i * nwords;
    for (int idx = threadIdx.x; idx < BLOCK * CW; idx += BLOCK) {
      const int64_t w = w0 + idx;
      words[(size_t)i * BLOCK * ST + (idx / CW) * ST + idx % CW] = w < nwords ? src[w] : 0ull;
    }
  }
  __syncthreads();
  const int64_t c = g * BLOCK + threadIdx.x;
  uint32_t d[K + 1];
  uint8_t x[K + 1];
  if (c < J.nchunks) {
    const int64_t c0 = c * CW * 64, c1 = c0 + CW * 64 < N ? c0 + CW * 64 : N;
    const unsigned long long* mine = words + (size_t)threadIdx.x * ST;
    const int32_t cwb = (int32_t)(c * CW);  // the chunk's first word (32-bit: docIds are Java ints)
    auto get = [&](int i, int32_t w) { return mine[i * (BLOCK * ST) + (w - cwb)]; };
    dfa_chunk<K>(k, c0, c1, get, d, x);
  } else {  // past the job's last chunk: the identity
#pragma unroll
    for (int e = 0; e <= K; ++e) {
      d[e] = 0;
      x[e] = (uint8_t)e;
    }
  }
  __syncthreads();  // the words are consumed: their LDS holds the tables now
  dfa_group_compose<K, BLOCK>(J, g, d, x, smem);
}

// ANDs of <= 4 scans (every SSB query; r6): one thread per chunk of CW words, the chunk's k x CW words loaded straight
// into registers (consecutive lanes read consecutive 8 * CW-byte runs), each word's table from dfa_word (walks inside
// registers only) composed in order into the chunk's table, then the workgroup tree.  K = the launch's widest AND
// (2..4): narrower jobs fill with all-ones scans.
template <int K, int BLOCK, int CW>
__global__ void __launch_bounds__(BLOCK) k_and_dfa_reg(const AndWalkJob* __restrict__ jobs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const AndWalkJob& J = jobs[blockIdx.y];
  const int64_t g = blockIdx.x;
  if (g >= J.ngroups) return;  // uniform over the workgroup
  const int k = J.k;
  const int64_t N = J.ndocs, nwords = J.nwords;
  const int64_t c = g * BLOCK + threadIdx.x;
  uint32_t d[K + 1];
  uint8_t x[K + 1];
#pragma unroll
  for (int e = 0; e <= K; ++e) {
    d[e] = 0;
    x[e] = (uint8_t)e;
  }
  if (c < J.nchunks) {
    unsigned long long Wall[K][CW];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
      for (int q = 0; q < CW; ++q) {
        const int64_t w = c * CW + q;
        Wall[i][q] = i >= k ? ~0ull : (w < nwords ? J.bits[(int64_t)i * nwords + w] : 0ull);
      }
#pragma unroll
    for (int q = 0; q < CW; ++q) {
      const int64_t c0 = (c * CW + q) * 64;
      if (c0 < N) {  // (lanes differ only in the job's last chunk)
        const int32_t c1 = N - c0 < 64 ? (int32_t)(N - c0) : 64;
        unsigned long long Wq[K];
#pragma unroll
        for (int i = 0; i < K; ++i)
          Wq[i] = (c1 < 64 && i < k) ? Wall[i][q] & ((1ull << c1) - 1ull) : Wall[i][q];
        uint32_t wd[K + 1];
        uint8_t wx[K + 1];
        dfa_word<K>(k, Wq, c1, wd, wx);
        if (q == 0) {
#pragma unroll
          for (int e = 0; e <= K; ++e) {
            d[e] = wd[e];
            x[e] = wx[e];
          }
        } else {
          uint32_t od[K + 1];
          uint8_t ox[K + 1];
          dfa_compose<K>(K, d, x, wd, wx, od, ox);
#pragma unroll
          for (int e = 0; e <= K; ++e) {
            d[e] = od[e];
            x[e] = ox[e];
          }
        }
      }
    }
  }
  dfa_group_compose<K, BLOCK>(J, g, d, x, smem);
}

// one wave per job: lane l composes its slice of the workgroup tables for every entry type (the k + 1 chains' loads
// interleaved), then lane 0 runs entry type -1 at doc 0 through the 64 slice tables in LDS.  (r5: one thread walking
// all ~300 tables of a 10M-doc segment serially was 50-70 us per query.)
__global__ void __launch_bounds__(64) k_and_compose(const AndWalkJob* __restrict__ jobs, unsigned long long* out) {
  constexpr int K = kMaxFbProgs;
  __shared__ unsigned long long sd[64][K + 1];
  __shared__ uint8_t sx[64][K + 1];
  const AndWalkJob& J = jobs[blockIdx.x];
  const int lane = threadIdx.x, k = J.k;
  const int64_t G = J.ngroups;
  const int64_t g0 = G * lane / 64, g1 = G * (lane + 1) / 64;
  unsigned long long acc[K + 1];
  int t[K + 1];
#pragma unroll
  for (int e = 0; e <= K; ++e) {
    acc[e] = 0;
    t[e] = e;
  }
  for (int64_t g = g0; g < g1; ++g) {
#pragma unroll
    for (int e = 0; e <= K; ++e)
      if (e <= k) {
        acc[e] += (unsigned long long)(int64_t)(int32_t)J.gdelta[(int64_t)t[e] * G + g];  // (< 0 only for k = 1)
        t[e] = J.gexit[(int64_t)t[e] * G + g];
      }
  }
#pragma unroll
  for (int e = 0; e <= K; ++e) {
    sd[lane][e] = acc[e];
    sx[lane][e] = (uint8_t)t[e];
  }
  __syncthreads();
  if (lane == 0) {
    int e = 0;  // entry type -1 at doc 0
    unsigned long long a = 0;
    for (int l = 0; l < 64; ++l) {
      a += sd[l][e];
      e = sx[l][e];
    }
    out[J.slot] = a + (e == 0 ? 1ull : 0ull);  // + the epoch at numDocs when the walk ends after a match
  }
}

template <int K, int BLOCK, int CW>
static void launch_dfa_cw(const AndWalkJob* jobs, int32_t njobs, int64_t max_groups, hipStream_t s) {
  constexpr size_t lds_words = (size_t)K * BLOCK * (CW + 1) * 8;
  constexpr size_t lds_tabs = (size_t)BLOCK * (K + 1) * 5;
  constexpr size_t lds = lds_words > lds_tabs ? lds_words : lds_tabs;
  allow_lds(k_and_dfa<K, BLOCK, CW>, lds);
  hipLaunchKernelGGL((k_and_dfa<K, BLOCK, CW>), dim3((unsigned)max_groups, (unsigned)njobs), dim3(BLOCK), lds, s, jobs);
}

template <int K, int BLOCK>
static void launch_dfa(const AndWalkJob* jobs, int32_t njobs, int64_t max_groups, hipStream_t s) {
  switch (and_dfa_chunk_words()) {
    case 2: launch_dfa_cw<K, BLOCK, 2>(jobs, njobs, max_groups, s); break;
    case 8: launch_dfa_cw<K, BLOCK, 8>(jobs, njobs, max_groups, s); break;
    default: launch_dfa_cw<K, BLOCK, 4>(jobs, njobs, max_groups, s); break;
  }
}


// chunks per workgroup of the launch k_and_dfa would use for an AND of k scans (the host sizes the tables with it):
// 128 threads (r5 at 256 threads and 8-word chunks, 44 % of wave cycles waited on the LDS word reads)
int and_dfa_block(int32_t max_k) { return max_k <= 4 ? 128 : max_k <= 8 ? 128 : 64; }

void launch_and_walk(const AndWalkJob* jobs, int32_t njobs, int64_t max_groups, int32_t max_k, unsigned long long* out,
                     hipStream_t s) {
  if (njobs <= 0 || max_groups <= 0) return;
  if (max_k > kMaxFbProgs) fail(PH_ERR_DEVICE, "AND walk wider than kMaxFbProgs scans");
  // the widest AND of the launch picks the register set (ST_SCANAND: at most kMaxFbProgs scans); LDS = K x 18 KiB
  if (max_k <= 4 && and_dfa_chunk_words() == 4) {
    constexpr size_t lds = (size_t)128 * 5 * 5;
    if (max_k <= 2) {
      allow_lds(k_and_dfa_reg<2, 128, 4>, lds);
      hipLaunchKernelGGL((k_and_dfa_reg<2, 128, 4>), dim3((unsigned)max_groups, (unsigned)njobs), dim3(128), lds, s, jobs);
    } else if (max_k == 3) {
      allow_lds(k_and_dfa_reg<3, 128, 4>, lds);
      hipLaunchKernelGGL((k_and_dfa_reg<3, 128, 4>), dim3((unsigned)max_groups, (unsigned)njobs), dim3(128), lds, s, jobs);
    } else {
      allow_lds(k_and_dfa_reg<4, 128, 4>, lds);
      hipLaunchKernelGGL((k_and_dfa_reg<4, 128, 4>), dim3((unsigned)max_groups, (unsigned)njobs), dim3(128), lds, s, jobs);
    }
  } else if (max_k <= 4) launch_dfa<4, 128>(jobs, njobs, max_groups, s);
  else if (max_k <= 8) launch_dfa<8, 128>(jobs, njobs, max_groups, s);
  else launch_dfa<kMaxFbProgs, 64>(jobs, njobs, max_groups, s);
  PH_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_and_compose, dim3((unsigned)njobs), dim3(64), 0, s, jobs, out);
  PH_HIP_CHECK(hipGetLastError());
}

}  // namespace ph

// test hook: the chunk size (words of 64 docs) k_and_dfa runs with
extern "C" int32_t phx_and_dfa_chunk_words() { return ph::and_dfa_chunk_words(); }

// test hook (not part of the product boundary, include/pinot_hip.h): one AND-of-scans job on the current device over
// host leaf bitmaps (leaf-major, k x ceil(n / 64) words); the entries, or -1 on a device error.  `gtab` (optional,
// (k + 1) x 2 x groups words) receives the workgroup tables (delta, exit + 1) for diagnosis.
extern "C" int64_t phx_and_walk_entries_device(const uint64_t* bits, int32_t k, int64_t num_docs, uint32_t* gtab) {
  using namespace ph;
  try {
    if (num_docs <= 0) return 0;
    const int64_t nwords = (num_docs + 63) / 64;
    AndWalkJob J{};
    J.nwords = nwords;
    J.ndocs = num_docs;
    J.k = k;
    J.slot = 0;
    J.nchunks = (num_docs + and_dfa_chunk_words() * 64 - 1) / (and_dfa_chunk_words() * 64);
    const int block = and_dfa_block(k);
    J.ngroups = (int32_t)((J.nchunks + block - 1) / block);
    DeviceBuffer b, d, x, jb, o;
    int dev = 0;
    PH_HIP_CHECK(hipGetDevice(&dev));
    b.alloc(8 * (size_t)k * nwords, dev);
    d.alloc(4 * (size_t)(k + 1) * J.ngroups, dev);
    x.alloc((size_t)(k + 1) * J.ngroups, dev);
    jb.alloc(sizeof(AndWalkJob), dev);
    o.alloc(8, dev);
    PH_HIP_CHECK(hipMemcpy(b.ptr, bits, 8 * (size_t)k * nwords, hipMemcpyHostToDevice));
    J.bits = b.as<unsigned long long>();
    J.gdelta = d.as<uint32_t>();
    J.gexit = x.as<uint8_t>();
    PH_HIP_CHECK(hipMemcpy(jb.ptr, &J, sizeof J, hipMemcpyHostToDevice));
    launch_and_walk(jb.as<AndWalkJob>(), 1, J.ngroups, k, o.as<unsigned long long>(), nullptr);
    PH_HIP_CHECK(hipDeviceSynchronize());
    unsigned long long out = 0;
    PH_HIP_CHECK(hipMemcpy(&out, o.ptr, 8, hipMemcpyDeviceToHost));
    if (gtab) {
      std::vector<uint8_t> hx((size_t)(k + 1) * J.ngroups);
      PH_HIP_CHECK(hipMemcpy(gtab, d.ptr, 4 * (size_t)(k + 1) * J.ngroups, hipMemcpyDeviceToHost));
      PH_HIP_CHECK(hipMemcpy(hx.data(), x.ptr, hx.size(), hipMemcpyDeviceToHost));
      for (size_t i = 0; i < hx.size(); ++i) gtab[(size_t)(k + 1) * J.ngroups + i] = hx[i];
    }
    return num_docs - 1 + (int64_t)out;
  } catch (...) {
    return -1;
  }
}
