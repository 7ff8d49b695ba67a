// kmg_dense.hip — dense count-vector formulation of the spectrum and mismatch Grams:
// K = F * F^T with F the int8 feature matrix, on the gfx950 int8 matrix cores.
//
// Reference hot loops replaced (afiliot/Kernel-Methods-For-Genomics kernels.py):
//   get_phi_u (kernels.py:12-25)        -> F[i][u] = #windows of x_i equal to u
//   get_phi_km (kernels.py:161-175)     -> F[i][b] = #windows a with ham(x_i[a], b) <= m
//   np.dot pair loops (kernels.py:41-45, 211-215) -> one symmetric int8 MFMA GEMM
//   normalize_K (kernels.py:398-415)    -> fused fp64 epilogue (diagonal from ||F_i||^2)
//
// This is the formulation for SMALL k (4^k feature columns, run.py's SP_k4..6 and
// MM_k4..6_m1): a row of F has 4^k int8 entries, every one of them <= 127 because a
// sequence has at most 127 windows (host check), so F*F^T accumulated in int32 is exact.
// Large k (sparse F, 4^k >> windows) goes through the posting-list kernels instead.
//
// Layout in HBM: F int8 [rows_alloc][dp], dp = 4^k rounded up to 128, rows_alloc >= n +
// 128 with the padding rows zero, so tile loads never need bounds checks.
#include "kmg_internal.h"

namespace kmg {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------ features
// One workgroup per sequence.  Byte counters packed four per LDS word (a count never
// exceeds 127, so adding 1 << 8*(b&3) never carries into the neighbour byte).
// Every valid window a with code u adds 1 to u ^ mask[t] for every neighbour mask t
// (mask 0 alone = spectrum; masks of Hamming weight <= m = mismatch).
__global__ __launch_bounds__(256) void dense_feat_kernel(
    const uint8_t *__restrict__ codes, const int32_t *__restrict__ lens, int64_t ldc, int k,
    int window, int dp, const uint32_t *__restrict__ masks, int nmask, int8_t *__restrict__ F,
    double *__restrict__ diagv, double *__restrict__ dsq) {
  extern __shared__ __align__(16) uint32_t hist[];  // dp / 4 words
  __shared__ int64_t red[4];
  const int64_t i = blockIdx.x;
  const int words = dp >> 2;
  for (int w = threadIdx.x; w < words; w += blockDim.x) hist[w] = 0;
  __syncthreads();
  const int L = window > 0 ? window : lens[i];
  const int P = L - k + 1;
  const uint8_t *rs = codes + i * ldc;
  if (P > 0) {
    const int items = P * nmask;
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
      const int a = it / nmask;
      const int t = it - a * nmask;
      uint32_t c = 0, bad = 0;
      for (int q = 0; q < k; ++q) {
        const uint32_t v = rs[a + q];
        bad |= v & ~3u;
        c = (c << 2) | (v & 3u);
      }
      if (bad) continue;
      const uint32_t b = c ^ masks[t];
      atomicAdd(&hist[b >> 2], 1u << ((b & 3) << 3));
    }
  }
  __syncthreads();
  // stream the row out (16 B per thread-iteration) and accumulate ||F_i||^2
  int64_t sq = 0;
  uint4 *dst = (uint4 *)(F + i * (int64_t)dp);
  for (int w = threadIdx.x; w < (words >> 2); w += blockDim.x) {
    const uint4 v = ((const uint4 *)hist)[w];
    const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int64_t e = (x[q] >> (8 * s)) & 0xFFu;
        sq += e * e;
      }
    }
    dst[w] = v;
  }
  // block reduction of sq (4 waves)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sq += __shfl_down(sq, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0 && diagv) {
    int64_t tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += red[w];
    const double d = (double)tot;
    diagv[i] = d;
    dsq[i] = sqrt(d);
  }
}

// ------------------------------------------------------------------ GEMM
// K[r][c] = sum_b F[r][b] F[c][b] over a 128 x 128 output tile per workgroup (4 waves,
// 2 x 2 of them, 64 x 64 each = 2 x 2 v_mfma_i32_32x32x32_i8 tiles).  The reduction
// runs over 128-byte stages of F staged in LDS (double buffered, XOR-swizzled 16-byte
// chunks so the fragment reads of 32 consecutive rows hit distinct banks).
//
// Both operands are rows of F, so A and B fragments are loaded by the same code:
// whatever order the instruction sums its 32 k-values in, A and B use the same lane/
// element -> k map, and the tile is the full dot product.  Output map (gfx950, every
// dtype): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5).
constexpr int DT_BM = 128;
constexpr int DT_BK = 128;                       // bytes of F per stage
constexpr int DT_STAGE = 2 * DT_BM * DT_BK;      // A + B bytes per stage

__device__ __forceinline__ int swz(int row, int c16) { return row * DT_BK + ((c16 ^ (row & 7)) << 4); }

template <int DT>
__device__ __forceinline__ void dense_store(const OutSpec &o, bool norm, int64_t row0, int64_t gr,
                                            int64_t gc, int v) {
  if constexpr (DT == KMG_I32) {
    __builtin_nontemporal_store(v, (int32_t *)o.out + (gr - row0) * o.ld + gc);
  } else {
    double r = (double)v;
    if (norm) r = (gr == gc) ? 1.0 : r / (o.dsq[gr] * o.dsq[gc]);
    if constexpr (DT == KMG_F64)
      __builtin_nontemporal_store(r, (double *)o.out + (gr - row0) * o.ld + gc);
    else
      __builtin_nontemporal_store((float)r, (float *)o.out + (gr - row0) * o.ld + gc);
  }
}

// Tile order: blocks are dispatched round-robin over the 8 XCDs, so block b is remapped
// to logical tile (b % 8) * per_xcd + b / 8 — each XCD walks a contiguous run of
// logical tiles — and logical tiles run down GROUP tile-rows before moving one
// tile-column right, so the workgroups resident on one XCD share a few F panels in its L2.
template <int DT>
__global__ __launch_bounds__(256, 2) void gram_dense_kernel(const int8_t *__restrict__ F, int dp,
                                                            int64_t n, int64_t row0, int64_t rows,
                                                            int tiles_m, int tiles_n, OutSpec o) {
  extern __shared__ __align__(16) uint8_t lds[];
  constexpr int GROUP = 8;
  const int total = tiles_m * tiles_n;
  const int per_xcd = (int)((gridDim.x + 7) >> 3);
  const int logical = (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3);
  if (logical >= total) return;
  const int band = logical / (GROUP * tiles_n);
  const int in_band = logical - band * GROUP * tiles_n;
  const int band_rows = min(GROUP, tiles_m - band * GROUP);
  const int tm = band * GROUP + in_band % band_rows;
  const int tn = in_band / band_rows;
  const int64_t rbase = row0 + (int64_t)tm * DT_BM;
  const int64_t cbase = (int64_t)tn * DT_BM;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // global -> register staging: 4 x 16 B of A and 4 x 16 B of B per thread per stage
  const int8_t *gA = F + rbase * (int64_t)dp;
  const int8_t *gB = F + cbase * (int64_t)dp;
  uint4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = tid + 256 * q;
      const int r = c >> 3, c16 = c & 7;
      ra[q] = *(const uint4 *)(gA + (int64_t)r * dp + k0 + c16 * 16);
      rb[q] = *(const uint4 *)(gB + (int64_t)r * dp + k0 + c16 * 16);
    }
  };
  auto lstore = [&](int buf) {
    uint8_t *sA = lds + buf * DT_STAGE;
    uint8_t *sB = sA + DT_BM * DT_BK;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = tid + 256 * q;
      const int r = c >> 3, c16 = c & 7;
      *(uint4 *)(sA + swz(r, c16)) = ra[q];
      *(uint4 *)(sB + swz(r, c16)) = rb[q];
    }
  };

  v16i acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (v16i){};

  const int nst = dp / DT_BK;
  gload(0);
  lstore(0);
  __syncthreads();
  const int fr = lane & 31, fh = lane >> 5;
  for (int st = 0; st < nst; ++st) {
    const int buf = st & 1;
    if (st + 1 < nst) gload((st + 1) * DT_BK);
    const uint8_t *sA = lds + buf * DT_STAGE;
    const uint8_t *sB = sA + DT_BM * DT_BK;
#pragma unroll
    for (int s = 0; s < DT_BK / 32; ++s) {
      const int c16 = 2 * s + fh;
      v4i a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = *(const v4i *)(sA + swz(wm * 64 + t * 32 + fr, c16));
        b[t] = *(const v4i *)(sB + swz(wn * 64 + t * 32 + fr, c16));
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[x], b[y], acc[x][y], 0, 0, 0);
    }
    if (st + 1 < nst) {
      lstore(buf ^ 1);
      __syncthreads();
    }
  }

  const bool norm = DT != KMG_I32 && o.normalize && o.diagv[0] != 1.0;
  const int64_t rend = row0 + rows;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int64_t gc = cbase + wn * 64 + y * 32 + fr;
      if (gc >= n) continue;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int64_t gr = rbase + wm * 64 + x * 32 + (g & 3) + 8 * (g >> 2) + 4 * fh;
        if (gr < rend) dense_store<DT>(o, norm, row0, gr, gc, acc[x][y][g]);
      }
    }
}

size_t dense_gram_lds_bytes() { return 2 * DT_STAGE; }

hipError_t launch_dense_features(const uint8_t *codes, const int32_t *lens, int64_t ldc, int64_t n,
                                 int k, int window, int dp, const uint32_t *masks, int nmask,
                                 int8_t *F, double *diagv, double *dsq, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if ((dp & 127) || dp > 65536) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dense_feat_kernel, dim3((unsigned)n), dim3(256), (size_t)dp, s, codes, lens,
                     ldc, k, window, dp, masks, nmask, F, diagv, dsq);
  return hipGetLastError();
}

// ------------------------------------------------------------------ gappy features
// Gappy (k, g) with the semantics get_gappy_K intends (kernels.py:420-455, report §3.7;
// the reference itself raises for every (k, g) but (1, 0)): F[i][b] = 1 if the (k-g)-mer b
// occurs as an order-preserving subsequence of k-g of the k positions of some window
// x[a : a+k], a < window - k + 1 (the reference's range(101 - k + 1)).  Presence, not
// count (``b in gap_set``).  combos[t] = the kept positions of combination t, 4 bits each
// (lowest nibble first, ascending).  One workgroup per sequence, byte flags in LDS.
__global__ __launch_bounds__(256) void gappy_feat_kernel(
    const uint8_t *__restrict__ codes, int64_t ldc, int k, int kk, int window, int dp,
    const uint32_t *__restrict__ combos, int ncomb, int8_t *__restrict__ F,
    double *__restrict__ diagv, double *__restrict__ dsq) {
  extern __shared__ __align__(16) uint32_t flags[];  // dp / 4 words
  __shared__ int64_t red[4];
  const int64_t i = blockIdx.x;
  const int words = dp >> 2;
  for (int w = threadIdx.x; w < words; w += blockDim.x) flags[w] = 0;
  __syncthreads();
  const int P = window - k + 1;
  const uint8_t *rs = codes + i * ldc;
  const int items = P > 0 ? P * ncomb : 0;
  for (int it = threadIdx.x; it < items; it += blockDim.x) {
    const int a = it / ncomb;
    const uint32_t cm = combos[it - a * ncomb];
    uint32_t c = 0, bad = 0;
    for (int q = 0; q < kk; ++q) {
      const uint32_t v = rs[a + ((cm >> (4 * q)) & 15u)];
      bad |= v & ~3u;
      c = (c << 2) | (v & 3u);
    }
    if (!bad) atomicOr(&flags[c >> 2], 1u << ((c & 3) << 3));
  }
  __syncthreads();
  int64_t sq = 0;
  uint4 *dst = (uint4 *)(F + i * (int64_t)dp);
  for (int w = threadIdx.x; w < (words >> 2); w += blockDim.x) {
    const uint4 v = ((const uint4 *)flags)[w];
    sq += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);  // bytes are 0 or 1
    dst[w] = v;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) sq += __shfl_down(sq, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) tot += red[w];
    const double d = (double)tot;
    diagv[i] = d;
    dsq[i] = sqrt(d);
  }
}

hipError_t launch_gappy_features(const uint8_t *codes, int64_t ldc, int64_t n, int k, int kk,
                                 int window, int dp, const uint32_t *combos, int ncomb, int8_t *F,
                                 double *diagv, double *dsq, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if ((dp & 127) || dp > 65536 || kk < 1 || kk > 8 || k > 15) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gappy_feat_kernel, dim3((unsigned)n), dim3(256), (size_t)dp, s, codes, ldc, k,
                     kk, window, dp, combos, ncomb, F, diagv, dsq);
  return hipGetLastError();
}

hipError_t launch_gram_dense(const int8_t *F, int dp, int64_t n, int64_t row0, int64_t row1,
                             const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || n <= 0) return hipSuccess;
  if (dp & (DT_BK - 1)) return hipErrorInvalidValue;
  const int tiles_m = (int)((rows + DT_BM - 1) / DT_BM);
  const int tiles_n = (int)((n + DT_BM - 1) / DT_BM);
  const int64_t total = (int64_t)tiles_m * tiles_n;
  if (total > 0x7FFFFFF0LL) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((total + 7) & ~7LL);
  const size_t lds = dense_gram_lds_bytes();
  switch (o.dtype) {
    case KMG_I32:
      hipLaunchKernelGGL(gram_dense_kernel<KMG_I32>, dim3(grid), dim3(256), lds, s, F, dp, n, row0,
                         rows, tiles_m, tiles_n, o);
      break;
    case KMG_F32:
      hipLaunchKernelGGL(gram_dense_kernel<KMG_F32>, dim3(grid), dim3(256), lds, s, F, dp, n, row0,
                         rows, tiles_m, tiles_n, o);
      break;
    default:
      hipLaunchKernelGGL(gram_dense_kernel<KMG_F64>, dim3(grid), dim3(256), lds, s, F, dp, n, row0,
                         rows, tiles_m, tiles_n, o);
      break;
  }
  return hipGetLastError();
}

}  // namespace kmg
