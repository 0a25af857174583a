// mbench.hip -- standalone bandwidth probes for the scan's access pattern (development tool, not product).
//   hipcc --offload-arch=gfx950 -O3 -o tools/mbench tools/mbench.hip && ./tools/mbench
// (a) grid-stride 16 B/lane read + xor reduce   (the chip's streaming ceiling for this pattern)
// (b) per-wave contiguous tiles of T KiB, chunked like k_scan (persistent grid, chunk = 40 KiB)
// (c) (b) + register prefetch one tile ahead + LDS staging (k_scan's data movement without the decode)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                       \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_grid_stride(const u32x4* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    u32x4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// each wave reads tiles of L x 1 KiB; a chunk = 4 waves x R rounds x tile
template <int L>
__global__ void __launch_bounds__(256) k_tiles(const uint8_t* __restrict__ p, size_t bytes, size_t chunk_bytes,
                                               uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t nchunks = bytes / chunk_bytes;
  const size_t tile = (size_t)L * 1024;
  uint32_t acc = 0;
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    for (size_t t = wave * tile; t < chunk_bytes; t += 4 * tile) {
      const uint8_t* src = p + c * chunk_bytes + t;
      u32x4 v[L];
#pragma unroll
      for (int k = 0; k < L; ++k) v[k] = *reinterpret_cast<const u32x4*>(src + k * 1024 + lane * 16);
#pragma unroll
      for (int k = 0; k < L; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int L>
__global__ void __launch_bounds__(256) k_tiles_pf(const uint8_t* __restrict__ p, size_t bytes, size_t chunk_bytes,
                                                  uint32_t* out) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t nchunks = bytes / chunk_bytes;
  const size_t tile = (size_t)L * 1024;
  uint8_t* wst = smem + wave * L * 1024;
  uint32_t acc = 0;
  size_t c = blockIdx.x, t = wave * tile;
  u32x4 v[L];
  if (c < nchunks) {
#pragma unroll
    for (int k = 0; k < L; ++k) v[k] = *reinterpret_cast<const u32x4*>(p + c * chunk_bytes + t + k * 1024 + lane * 16);
  }
  while (c < nchunks) {
#pragma unroll
    for (int k = 0; k < L; ++k) *reinterpret_cast<u32x4*>(wst + k * 1024 + lane * 16) = v[k];
    t += 4 * tile;
    if (t >= chunk_bytes) {
      t = wave * tile;
      c += gridDim.x;
    }
    if (c < nchunks) {
#pragma unroll
      for (int k = 0; k < L; ++k)
        v[k] = *reinterpret_cast<const u32x4*>(p + c * chunk_bytes + t + k * 1024 + lane * 16);
    }
    __builtin_amdgcn_wave_barrier();
    // consume: 2 dwords per lane per 64-doc word, 32 words
    const uint32_t* w = reinterpret_cast<const uint32_t*>(wst);
    for (int u = 0; u < L * 1024 / 160; ++u) acc += __builtin_amdgcn_alignbit(w[u * 40 + lane / 2], w[u * 40 + lane / 2 + 1], lane & 31);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// 4 separate streams (b = 10, 10, 10, 20 bits): each wave reads the same 16-word tile span of every stream
// (1280, 1280, 1280, 2560 bytes), like the partitioned group-by scan; optional workgroup barrier per round.
template <int BAR>
__global__ void __launch_bounds__(256) k_4streams(const uint8_t* __restrict__ s0, const uint8_t* __restrict__ s1,
                                                  const uint8_t* __restrict__ s2, const uint8_t* __restrict__ s3,
                                                  size_t words, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t tiles = words / 16;
  const size_t t0 = tiles * blockIdx.x / gridDim.x, t1 = tiles * (blockIdx.x + 1) / gridDim.x;
  uint32_t acc = 0;
  for (size_t t = t0 + wave; t < t1 + 4; t += 4) {
    u32x4 v[9];
    const bool ok = t < t1;
    if (ok) {
      const size_t w0 = t * 16;
      const uint8_t* srcs[3] = {s0 + w0 * 80, s1 + w0 * 80, s2 + w0 * 80};
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        v[2 * s] = *reinterpret_cast<const u32x4*>(srcs[s] + lane * 16);
        if (1024 + lane * 16 < 1288) v[2 * s + 1] = *reinterpret_cast<const u32x4*>(srcs[s] + 1024 + lane * 16);
        else v[2 * s + 1] = u32x4{0, 0, 0, 0};
      }
      const uint8_t* d = s3 + w0 * 160;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (k * 1024 + lane * 16 < 2568) v[6 + k] = *reinterpret_cast<const u32x4*>(d + k * 1024 + lane * 16);
        else v[6 + k] = u32x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (BAR) __syncthreads();
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)2560 << 20;  // 2.5 GiB
  uint8_t* d;
  uint32_t* out;
  CK(hipMalloc(&d, bytes + 65536));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(d, 1, bytes));
  hipEvent_t a, b, b_ev;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  b_ev = b;
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 10;
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    printf("%-44s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  for (int bpc : {4, 8}) {
    char nm[64];
    snprintf(nm, sizeof nm, "grid-stride x4 grid=%d/CU", bpc);
    run(nm, [&] { hipLaunchKernelGGL(k_grid_stride, dim3(256 * bpc), dim3(256), 0, 0, (const u32x4*)d, bytes / 16, out); });
  }
  const size_t chunk = 40960;
  for (int bpc : {4, 7, 8}) {
    char nm[64];
    snprintf(nm, sizeof nm, "tiles L=1 chunk=40K %d/CU", bpc);
    run(nm, [&] { hipLaunchKernelGGL(k_tiles<1>, dim3(256 * bpc), dim3(256), 0, 0, d, bytes, (size_t)16384, out); });
    snprintf(nm, sizeof nm, "tiles L=2 chunk=32K %d/CU", bpc);
    run(nm, [&] { hipLaunchKernelGGL(k_tiles<2>, dim3(256 * bpc), dim3(256), 0, 0, d, bytes, (size_t)32768, out); });
    snprintf(nm, sizeof nm, "tiles L=5 chunk=40K %d/CU", bpc);
    run(nm, [&] { hipLaunchKernelGGL(k_tiles<5>, dim3(256 * bpc), dim3(256), 0, 0, d, bytes, chunk, out); });
    snprintf(nm, sizeof nm, "tiles L=8 chunk=64K %d/CU", bpc);
    run(nm, [&] { hipLaunchKernelGGL(k_tiles<8>, dim3(256 * bpc), dim3(256), 0, 0, d, bytes, (size_t)65536, out); });
    snprintf(nm, sizeof nm, "tiles+prefetch+LDS L=5 chunk=40K %d/CU", bpc);
    run(nm, [&] {
      hipLaunchKernelGGL(k_tiles_pf<5>, dim3(256 * bpc), dim3(256), 4 * 5 * 1024, 0, d, bytes, chunk, out);
    });
  }
  {
    // 1e9 docs: streams of 1.25, 1.25, 1.25, 2.5 GB in 4 allocations
    const size_t words = 1000000000 / 64;
    uint8_t* b[4];
    for (int i = 0; i < 4; ++i) {
      const size_t n = words * (i == 3 ? 160 : 80) + 65536;
      CK(hipMalloc(&b[i], n));
      CK(hipMemset(b[i], 1, n));
    }
    const double tot = words * 400.0;
    for (int bpc : {3, 4, 8}) {
      for (int bar : {0, 1}) {
        auto launch = [&] {
          if (bar) hipLaunchKernelGGL(k_4streams<1>, dim3(256 * bpc), dim3(256), 0, 0, b[0], b[1], b[2], b[3], words, out);
          else hipLaunchKernelGGL(k_4streams<0>, dim3(256 * bpc), dim3(256), 0, 0, b[0], b[1], b[2], b[3], words, out);
        };
        for (int i = 0; i < 2; ++i) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int i = 0; i < 5; ++i) launch();
        CK(hipEventRecord(b_ev));
        CK(hipEventSynchronize(b_ev));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b_ev));
        ms /= 5;
        printf("4 streams %d/CU barrier=%d                   %8.3f ms  %7.0f GB/s\n", bpc, bar, ms, tot / ms / 1e6);
      }
    }
  }
  return 0;
}
