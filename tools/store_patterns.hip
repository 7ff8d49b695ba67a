// store_patterns.hip — microbenchmark: write an N x N int32 / float64 matrix (row-major,
// ld = N) with the store shapes of the Gram kernels, to separate the write pattern from
// the kernels' compute.  One JSON line per (pattern, dtype).
//   rows1024 : one 1024-thread block per row, 16 B per lane, a wave covers 1 KB (spectrum)
//   tile8x128: 256 x 256 tiles, 8 waves; each store instruction = 8 rows x 128 B
//              (the dense kernel's 32 x 32 sub-tile epilogue)
//   tile1x1k : 256 x 256 tiles, 8 waves; each store instruction = 1 row x 1 KB
//   tile2x512: 256 x 256 tiles, 8 waves; each store instruction = 2 rows x 512 B
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_patterns tools/store_patterns.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st16(void *p, v4i v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, (v4i *)p);
  else
    *(v4i *)p = v;
}

// ESZ bytes per element; one block per row
template <int ESZ, bool NT>
__global__ __launch_bounds__(1024) void rows_kernel(char *out, int64_t n) {
  const int64_t i = blockIdx.x;
  char *row = out + i * n * ESZ;
  const int64_t bytes = n * ESZ;
  for (int64_t b = (int64_t)threadIdx.x * 16; b < bytes; b += 1024 * 16)
    st16<NT>(row + b, (v4i){(int)i, (int)b, 1, 2});
}

// rows1024 with a compute phase before the stores (SLEEP x 127 x 64 clocks), as the
// spectrum kernel's gather phase
template <int ESZ, bool NT, int SLEEP>
__global__ __launch_bounds__(1024) void rows_delay_kernel(char *out, int64_t n) {
  for (int s = 0; s < SLEEP; ++s) __builtin_amdgcn_s_sleep(127);
  const int64_t i = blockIdx.x;
  char *row = out + i * n * ESZ;
  const int64_t bytes = n * ESZ;
  for (int64_t b = (int64_t)threadIdx.x * 16; b < bytes; b += 1024 * 16)
    st16<NT>(row + b, (v4i){(int)i, (int)b, 1, 2});
}

// rows1024 through buffer stores with cache-policy bits AUX (1 sc0, 2 nt, 16 sc1)
template <int ESZ, int AUX>
__global__ __launch_bounds__(1024) void rows_buf_kernel(char *out, int64_t n) {
  const int64_t i = blockIdx.x;
  const int64_t bytes = n * ESZ;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out + i * bytes, 0, (int)bytes, 0x00020000);
  for (int b = threadIdx.x * 16; b < bytes; b += 1024 * 16)
    __builtin_amdgcn_raw_buffer_store_b128((v4i){(int)i, b, 1, 2}, rsrc, b, 0, AUX);
}

// grid-stride, U stores in flight per thread: iteration it covers [it*G*16*U, ...), thread
// t writes 16 B at t*16 + u*G*16 (every instruction of a wave contiguous)
template <int U, int TPB>
__global__ __launch_bounds__(TPB) void stride_kernel(char *out, int64_t bytes) {
  const int64_t G = (int64_t)gridDim.x * TPB;
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  for (int64_t base = 0; base < bytes; base += G * 16 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t b = base + (t + u * G) * 16;
      if (b + 16 <= bytes) st16<true>(out + b, (v4i){(int)b, u, 1, 2});
    }
  }
}

// persistent: G blocks, block b writes rows b, b + G, ... (G rows in flight)
template <int ESZ, bool NT>
__global__ __launch_bounds__(1024) void rows_persist_kernel(char *out, int64_t n) {
  const int64_t bytes = n * ESZ;
  for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
    char *row = out + i * bytes;
    for (int64_t b = (int64_t)threadIdx.x * 16; b < bytes; b += 1024 * 16)
      st16<NT>(row + b, (v4i){(int)i, (int)b, 1, 2});
  }
}

// flat grid-stride: 16 KB chunks, chunk c = block + k * grid (all blocks in one window)
template <bool NT>
__global__ __launch_bounds__(1024) void linear_kernel(char *out, int64_t bytes) {
  for (int64_t c = (int64_t)blockIdx.x * 16384; c < bytes; c += (int64_t)gridDim.x * 16384) {
    const int64_t b = c + (int64_t)threadIdx.x * 16;
    if (b + 16 <= bytes) st16<NT>(out + b, (v4i){(int)c, (int)b, 1, 2});
  }
}

// 256 x 256 tiles, XCD-major order (consecutive tiles of a row band on one XCD);
// RPI rows per wave store instruction, each row 1024 / RPI bytes
template <int ESZ, int RPI, bool NT>
__global__ __launch_bounds__(512) void tile_kernel(char *out, int64_t n, int tiles_n, int64_t ntiles) {
  const int64_t per_xcd = ((int64_t)gridDim.x + 7) >> 3;
  const int64_t t = (int64_t)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (t >= ntiles) return;
  const int tm = (int)(t / tiles_n), tn = (int)(t % tiles_n);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int SEG = 1024 / RPI;           // bytes per row per instruction
  constexpr int LPR = SEG / 16;             // lanes per row
  constexpr int TB = 256 * ESZ;             // tile row bytes
  constexpr int SEGS = TB / SEG;            // segments per tile row
  // the tile = 256 rows x SEGS segments; wave w takes segment columns round robin
  const int r_in = lane / LPR, c_in = lane % LPR;
  for (int sc = 0; sc < SEGS; ++sc) {
    for (int rb = wave * RPI; rb < 256; rb += 8 * RPI) {
      const int64_t r = (int64_t)tm * 256 + rb + r_in;
      const int64_t cb = (int64_t)tn * TB + (int64_t)sc * SEG + c_in * 16;
      if (r < n && cb + 16 <= n * ESZ) st16<NT>(out + r * n * ESZ + cb, (v4i){(int)r, (int)cb, 3, 4});
    }
  }
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int ESZ, bool NT>
void run_all(char *d, int64_t n) {
  const double bytes = (double)n * n * ESZ;
  const int tiles_n = (int)((n + 255) / 256);
  const int64_t ntiles = (int64_t)tiles_n * tiles_n;
  const unsigned grid = (unsigned)((ntiles + 7) & ~7LL);
  auto rep = [&](const char *name, float ms) {
    printf("{\"pattern\": \"%s\", \"esz\": %d, \"nt\": %d, \"n\": %lld, \"ms\": %.4f, \"GBps\": %.1f}\n",
           name, ESZ, (int)NT, (long long)n, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  rep("memset", time_it([&] { CK(hipMemsetAsync(d, 0, (size_t)bytes, 0)); }, 10));
  rep("rows1024", time_it([&] { rows_kernel<ESZ, NT><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsB0", time_it([&] { rows_buf_kernel<ESZ, 0><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsB1sc0", time_it([&] { rows_buf_kernel<ESZ, 1><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsB2nt", time_it([&] { rows_buf_kernel<ESZ, 2><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsB16sc1", time_it([&] { rows_buf_kernel<ESZ, 16><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsB17sc0sc1", time_it([&] { rows_buf_kernel<ESZ, 17><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsB18sc1nt", time_it([&] { rows_buf_kernel<ESZ, 18><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsB3sc0nt", time_it([&] { rows_buf_kernel<ESZ, 3><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("strideU8_256x1024", time_it([&] { stride_kernel<8, 256><<<1024, 256>>>(d, (int64_t)bytes); }, 10));
  rep("strideU4_256x2048", time_it([&] { stride_kernel<4, 256><<<2048, 256>>>(d, (int64_t)bytes); }, 10));
  rep("strideU8_64x4096", time_it([&] { stride_kernel<8, 64><<<4096, 64>>>(d, (int64_t)bytes); }, 10));
  rep("strideU1_256x8192", time_it([&] { stride_kernel<1, 256><<<8192, 256>>>(d, (int64_t)bytes); }, 10));
  rep("strideU16_1024x256", time_it([&] { stride_kernel<16, 1024><<<256, 1024>>>(d, (int64_t)bytes); }, 10));
  rep("rowsD1", time_it([&] { rows_delay_kernel<ESZ, NT, 1><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsD2", time_it([&] { rows_delay_kernel<ESZ, NT, 2><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsD4", time_it([&] { rows_delay_kernel<ESZ, NT, 4><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("rowsD8", time_it([&] { rows_delay_kernel<ESZ, NT, 8><<<(unsigned)n, 1024>>>(d, n); }, 10));
  rep("linear2048", time_it([&] { linear_kernel<NT><<<2048, 1024>>>(d, (int64_t)bytes); }, 10));
  rep("linear512", time_it([&] { linear_kernel<NT><<<512, 1024>>>(d, (int64_t)bytes); }, 10));
  rep("rowsP256", time_it([&] { rows_persist_kernel<ESZ, NT><<<256, 1024>>>(d, n); }, 10));
  rep("rowsP512", time_it([&] { rows_persist_kernel<ESZ, NT><<<512, 1024>>>(d, n); }, 10));
  rep("rowsP128", time_it([&] { rows_persist_kernel<ESZ, NT><<<128, 1024>>>(d, n); }, 10));
  rep("tile8x128", time_it([&] { tile_kernel<ESZ, 8, NT><<<grid, 512>>>(d, n, tiles_n, ntiles); }, 10));
  rep("tile2x512", time_it([&] { tile_kernel<ESZ, 2, NT><<<grid, 512>>>(d, n, tiles_n, ntiles); }, 10));
  rep("tile1x1k", time_it([&] { tile_kernel<ESZ, 1, NT><<<grid, 512>>>(d, n, tiles_n, ntiles); }, 10));
}

int main(int argc, char **argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 20000;
  char *d;
  CK(hipMalloc(&d, (size_t)n * n * 8));
  run_all<4, true>(d, n);
  run_all<4, false>(d, n);
  run_all<8, true>(d, n);
  run_all<8, false>(d, n);
  CK(hipFree(d));
  return 0;
}
