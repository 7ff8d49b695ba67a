// LDS add throughput microbenchmark (gfx950): 1024-thread workgroups (one a CU at a time:
// the 80 KB accumulator), an int32 accumulator of W words, each lane issuing R LDS
// operations over addresses from a register hash (a few VALU each, no memory traffic).
// Reports ns per wave-instruction per CU and the kernel time.
//   mode 0: ds_add_u32, uniformly random words
//   mode 1: ds_write_b32, the same addresses
//   mode 2: ds_add_u32, lane l's word = base + l (conflict-free, consecutive)
//   mode 3: ds_add_u32, a lane's 15 consecutive adds within 255 words of a random base
//           (the packed neighbourhood-list pieces)
//   mode 4: ds_add_rtn_u32, uniformly random
//   mode 5: none (address hashing only: the VALU floor of the loop)
// hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_bench.hip -o /tmp/lds_atomic_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int W = 20000, R = 4096;

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(1024) void bench(uint32_t seed, int *out) {
  __shared__ int acc[W + 256];
  for (int i = threadIdx.x; i < W + 256; i += 1024) acc[i] = 0;
  __syncthreads();
  const uint32_t t = blockIdx.x * 1024u + threadIdx.x;
  int sink = 0;
  uint32_t base = hsh(t ^ seed) % (W - 256);
  for (int r = 0; r < R; r += 15) {
    if (MODE == 3) base = hsh(t * 7919u + r + seed) % (W - 256);
#pragma unroll
    for (int u = 0; u < 15; ++u) {
      const uint32_t h = hsh(t * 131u + (uint32_t)(r + u) * 0x9e3779b9u + seed);
      uint32_t a;
      if (MODE == 2) a = (uint32_t)(((r + u) * 64 + (threadIdx.x & 63) + (threadIdx.x >> 6) * 1024) % W);
      else if (MODE == 3) a = base + (h & 0xFFu) % 255u;
      else a = h % (uint32_t)W;
      if (MODE == 0 || MODE == 2 || MODE == 3) atomicAdd(&acc[a], 2);
      else if (MODE == 1) acc[a] = (int)h;
      else if (MODE == 4) sink += atomicAdd(&acc[a], 2);
      else sink += (int)a;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = acc[(blockIdx.x * 7) % W] + sink;
}

int main() {
  const int blocks = 256 * 4;
  int *o;
  hipMalloc(&o, blocks * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[] = {"ds_add random", "ds_write random", "ds_add consecutive",
                         "ds_add packed-piece", "ds_add_rtn random", "address hash only"};
  for (int mode = 0; mode < 6; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      switch (mode) {
        case 0: hipLaunchKernelGGL(bench<0>, dim3(blocks), dim3(1024), 0, 0, 1u + rep, o); break;
        case 1: hipLaunchKernelGGL(bench<1>, dim3(blocks), dim3(1024), 0, 0, 1u + rep, o); break;
        case 2: hipLaunchKernelGGL(bench<2>, dim3(blocks), dim3(1024), 0, 0, 1u + rep, o); break;
        case 3: hipLaunchKernelGGL(bench<3>, dim3(blocks), dim3(1024), 0, 0, 1u + rep, o); break;
        case 4: hipLaunchKernelGGL(bench<4>, dim3(blocks), dim3(1024), 0, 0, 1u + rep, o); break;
        default: hipLaunchKernelGGL(bench<5>, dim3(blocks), dim3(1024), 0, 0, 1u + rep, o); break;
      }
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    // wave-instructions per CU: blocks / 256 workgroups x 16 waves x (R rounded to 15s)
    const double instr = (double)blocks / 256 * 16 * ((R + 14) / 15 * 15);
    printf("{\"mode\": %d, \"name\": \"%s\", \"ms\": %.4f, \"ns_per_wave_instr_per_cu\": %.3f}\n", mode,
           names[mode], best, best * 1e6 / instr);
  }
  return 0;
}
