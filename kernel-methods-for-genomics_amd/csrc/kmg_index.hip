// kmg_index.hip — k-mer extraction and posting-index build on gfx950.
//
// Replaces the dense feature vectors of the reference:
//   get_phi_u  (kernels.py:12-25):  phi_u[b] = #{i < len(x)-k+1 : x[i:i+k] == b}
//   get_phi_km (kernels.py:161-175): phi_km[b] = #{i < 101-k+1 : ham(x[i:i+k], b) <= m}
// Instead of 4^k-wide float64 rows we keep, per k-mer key, the list of columns
// (sequences) holding it ("postings").  The Gram kernels then accumulate one row
// of K at a time in LDS (kmg_gram.hip).  All work here is integer: a histogram
// (global atomics), an exclusive scan and a scatter.
#include "kmg_internal.h"

namespace kmg {

// letter p of a k-mer code: most significant letter first (itertools.product order,
// kernels.py:37,206 — base-4 with A=0,C=1,G=2,T=3)
__device__ __forceinline__ uint32_t letter_at(uint32_t code, int p, int k) {
  return (code >> (2 * (k - 1 - p))) & 3u;
}
// the (k-1)-letter key obtained by deleting letter p
__device__ __forceinline__ uint32_t drop_letter(uint32_t code, int p, int k) {
  const uint64_t c = code;
  const int lo_bits = 2 * (k - 1 - p);
  const uint64_t hi = c >> (lo_bits + 2);
  const uint64_t lo = c & ((1ull << lo_bits) - 1ull);
  return (uint32_t)((hi << lo_bits) | lo);
}

__global__ __launch_bounds__(256) void extract_kernel(IndexGeom g, const uint8_t *__restrict__ codes,
                                                      const int32_t *__restrict__ lens, int64_t ldc,
                                                      uint32_t *__restrict__ kmers,
                                                      uint32_t *__restrict__ hist) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= g.n * g.pmax) return;
  const int64_t j = t / g.pmax;
  const int a = (int)(t - j * g.pmax);
  const int L = g.window > 0 ? g.window : lens[j];
  const int P = L - g.k + 1;  // number of windows (range(len(x)-k+1), kernels.py:21)
  uint32_t code = KMG_INVALID;
  if (a < P) {
    const uint8_t *s = codes + j * ldc + a;
    uint32_t c = 0, bad = 0;
    for (int q = 0; q < g.k; ++q) {
      const uint32_t v = s[q];
      bad |= v & ~3u;  // non-ACGT symbol: k-mer equals no beta (kernels.py:23-24)
      c = (c << 2) | (v & 3u);
    }
    if (!bad) code = c;
  }
  kmers[t] = code;
  if (code == KMG_INVALID) return;
  const int ch = (int)(j / g.chunk);
  if (g.copies == 1) {
    atomicAdd(&hist[(size_t)ch * g.nkeys + code], 1u);
  } else {
    for (int p = 0; p < g.copies; ++p) {
      const size_t bin = ((size_t)p * g.nchunks + ch) * g.nkeys + drop_letter(code, p, g.k);
      atomicAdd(&hist[bin], 1u);
    }
  }
}

__global__ __launch_bounds__(256) void scatter_kernel(IndexGeom g, const uint32_t *__restrict__ kmers,
                                                      uint32_t *__restrict__ cursor,
                                                      uint32_t *__restrict__ ent) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= g.n * g.pmax) return;
  const uint32_t code = kmers[t];
  if (code == KMG_INVALID) return;
  const int64_t j = t / g.pmax;
  const int ch = (int)(j / g.chunk);
  const uint32_t jj = (uint32_t)(j - (int64_t)ch * g.chunk);
  if (g.copies == 1) {
    const uint32_t pos = atomicAdd(&cursor[(size_t)ch * g.nkeys + code], 1u);
    ent[pos] = jj;
  } else {
    for (int p = 0; p < g.copies; ++p) {
      const size_t bin = ((size_t)p * g.nchunks + ch) * g.nkeys + drop_letter(code, p, g.k);
      const uint32_t pos = atomicAdd(&cursor[bin], 1u);
      ent[pos] = jj | (letter_at(code, p, g.k) << KMG_ENTRY_LETTER_SHIFT);
    }
  }
}

// ------------------------------------------------------------------ scan
// Three-phase exclusive scan over uint32 (counts < 2^32 checked by the host).
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// exclusive scan of one value per thread across the block; returns the block total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t &excl, uint32_t *tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if (lane == 63) tmp[wave] = inc;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < nw; ++w) {
    const uint32_t s = tmp[w];
    if (w < wave) base += s;
    total += s;
  }
  __syncthreads();
  excl = base + inc - v;
  return total;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_tiles_kernel(const uint32_t *__restrict__ in,
                                                                  int64_t nb,
                                                                  uint32_t *__restrict__ partials) {
  __shared__ uint32_t tmp[SCAN_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q)
    if (base + q < nb) s += in[base + q];
  uint32_t excl;
  const uint32_t total = block_excl_scan(s, excl, tmp);
  if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void scan_partials_kernel(uint32_t *__restrict__ partials,
                                                             int64_t np) {
  __shared__ uint32_t tmp[16];
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < np; b0 += blockDim.x) {
    const int64_t idx = b0 + threadIdx.x;
    const uint32_t v = idx < np ? partials[idx] : 0u;
    uint32_t excl;
    const uint32_t total = block_excl_scan(v, excl, tmp);
    if (idx < np) partials[idx] = carry + excl;
    carry += total;
  }
  if (threadIdx.x == 0) partials[np] = carry;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_finalize_kernel(
    const uint32_t *__restrict__ in, int64_t nb, const uint32_t *__restrict__ partials,
    uint32_t *__restrict__ off, uint32_t *__restrict__ cursor) {
  __shared__ uint32_t tmp[SCAN_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q) {
    v[q] = (base + q < nb) ? in[base + q] : 0u;
    s += v[q];
  }
  uint32_t excl;
  block_excl_scan(s, excl, tmp);
  uint32_t run = partials[blockIdx.x] + excl;
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q) {
    if (base + q < nb) {
      off[base + q] = run;
      cursor[base + q] = run;
    }
    run += v[q];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    const int64_t np = gridDim.x;
    off[nb] = partials[np];
  }
}

size_t scan_partials_words(int64_t nb) { return (size_t)((nb + SCAN_TILE - 1) / SCAN_TILE) + 1; }

hipError_t launch_extract(const IndexGeom &g, const uint8_t *codes, const int32_t *lens,
                          int64_t ldc, uint32_t *kmers, uint32_t *hist, hipStream_t s) {
  const int64_t items = g.n * g.pmax;
  if (items == 0) return hipSuccess;
  const int64_t blocks = (items + 255) / 256;
  hipLaunchKernelGGL(extract_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g, codes, lens, ldc,
                     kmers, hist);
  return hipGetLastError();
}

hipError_t launch_scatter(const IndexGeom &g, const uint32_t *kmers, uint32_t *cursor,
                          uint32_t *ent, hipStream_t s) {
  const int64_t items = g.n * g.pmax;
  if (items == 0) return hipSuccess;
  const int64_t blocks = (items + 255) / 256;
  hipLaunchKernelGGL(scatter_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g, kmers, cursor,
                     ent);
  return hipGetLastError();
}

hipError_t launch_scan(const uint32_t *hist, uint32_t *off, uint32_t *cursor, int64_t nb,
                       uint32_t *partials, hipStream_t s) {
  const int64_t tiles = (nb + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles == 0) return hipMemsetAsync(off, 0, sizeof(uint32_t), s);
  hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, s, hist, nb,
                     partials);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, partials, tiles);
  hipLaunchKernelGGL(scan_finalize_kernel, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, s, hist,
                     nb, partials, off, cursor);
  return hipGetLastError();
}

}  // namespace kmg
