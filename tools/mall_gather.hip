// mall_gather.hip — microbenchmark: random gathers of S-byte aligned pieces from a table of
// T bytes (L2 / Infinity Cache / HBM), as the mismatch Gram kernel's posting-line loads do.
// Prints one JSON line per (T, S, D) point: pieces/s, GB/s of piece bytes.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mall_gather tools/mall_gather.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// G lanes (16 B each) per piece of S = 16 G bytes; D pieces in flight per lane group.
template <int G, int D>
__global__ __launch_bounds__(256) void gather_kernel(const uint4 *__restrict__ tab, uint32_t npieces,
                                                     uint32_t iters, uint32_t seed,
                                                     uint32_t *__restrict__ sink) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t grp = tid / G, gl = tid % G;
  uint32_t acc = 0;
  for (uint32_t it = 0; it < iters; it += D) {
    uint4 v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const uint32_t p = hash32(grp * 0x9E3779B1u + (it + d) * 0x85EBCA77u + seed) % npieces;
      v[d] = tab[(size_t)p * G + gl];
    }
#pragma unroll
    for (int d = 0; d < D; ++d) acc += v[d].x ^ v[d].y ^ v[d].z ^ v[d].w;
  }
  if (acc == 0x12345678u) sink[tid] = acc;  // keeps the loads live; (almost) never stores
}

template <int G, int D>
double run(const uint4 *tab, size_t table_bytes, uint32_t *sink, int blocks, uint32_t iters) {
  const uint32_t npieces = (uint32_t)(table_bytes / (16 * G));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL((gather_kernel<G, D>), dim3(blocks), dim3(256), 0, 0, tab, npieces, iters, 1u, sink);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  const int reps = 3;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((gather_kernel<G, D>), dim3(blocks), dim3(256), 0, 0, tab, npieces, iters,
                       (uint32_t)(r + 2), sink);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double pieces = (double)blocks * 256 / G * iters * reps;
  const double s = ms / 1e3;
  printf("{\"table_MB\": %.1f, \"piece_B\": %d, \"inflight_per_group\": %d, \"blocks\": %d, "
         "\"ms\": %.3f, \"Gpieces_per_s\": %.2f, \"GBps\": %.1f}\n",
         table_bytes / 1e6, 16 * G, D, blocks, ms / reps, pieces / s / 1e9, pieces * 16 * G / s / 1e9);
  fflush(stdout);
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return pieces / s;
}

int main(int argc, char **argv) {
  const size_t maxT = (size_t)512 << 20;
  uint4 *tab = nullptr;
  uint32_t *sink = nullptr;
  CK(hipMalloc(&tab, maxT));
  CK(hipMalloc(&sink, (size_t)4096 * 256 * 4));
  CK(hipMemset(tab, 0x5A, maxT));
  const size_t tables[] = {(size_t)3 << 20, (size_t)38 << 20, (size_t)75 << 20, (size_t)150 << 20,
                           (size_t)226 << 20, (size_t)512 << 20};
  const int blocks = 4096;
  for (size_t T : tables) {
    run<4, 4>(tab, T, sink, blocks, 64);     // 64 B
    run<8, 4>(tab, T, sink, blocks, 64);     // 128 B
    run<8, 8>(tab, T, sink, blocks, 64);     // 128 B, deeper
    run<16, 4>(tab, T, sink, blocks, 64);    // 256 B
    run<32, 4>(tab, T, sink, blocks, 64);    // 512 B
    run<64, 4>(tab, T, sink, blocks, 64);    // 1 KiB
  }
  CK(hipFree(tab));
  CK(hipFree(sink));
  return 0;
}
