// kmg_features.hip — per-sequence feature vectors over caller-chosen k-mer columns (gfx950):
// the reference's feature maps as module-level functions, evaluated on the device.
//
//   get_phi_u(x, k, betas)      kernels.py:12-25   phi[j] = #{a < len(x)-k+1 : x[a:a+k] == b_j}
//   get_phi_km(x, k, m, betas)  kernels.py:161-175 phi[j] = #{a < 101-k+1 : ham(x[a:a+k], b_j) <= m}
//   gappy_k(x, 1, 0, betas)     kernels.py:420-433 phi[j] = [b_j occurs in x[0:101]]
//
// One workgroup per (sequence, 1024 columns): the sequence's windows are encoded once into
// LDS as a 2-bit code plus a "bad symbol" mask in the same 2-bit-per-position layout, then
// each lane scores four columns against every window (LDS broadcast reads):
//   ham(a, b) = popc(((w_a ^ b) | (w_a ^ b) >> 1) & 0x55.. | bad_a)
// so a non-ACGT symbol mismatches every letter (get_phi_km compares format()ed integers;
// for m = 0 a window holding one equals no beta, kernels.py:23-24).  Rows are streamed with
// one coalesced float64 store per lane and column.  Work is O(ncols x windows) per sequence
// (k = 8: 65536 x 94), microseconds per row: the call is bound by copying 8 B a column out.
#include "kmg_internal.h"

namespace kmg {

namespace {
constexpr int FT_THREADS = 256;
constexpr int FT_COLS = 4;                      // columns a lane
constexpr int FT_TILE = FT_THREADS * FT_COLS;   // columns a workgroup
}  // namespace

__global__ __launch_bounds__(FT_THREADS) void features_kernel(
    const uint8_t *__restrict__ codes, const int32_t *__restrict__ lens, int64_t ldc, int64_t row0,
    int k, int m, int window, int binary, const uint32_t *__restrict__ cols, int64_t ncols,
    double *__restrict__ out, int64_t ld) {
  __shared__ uint32_t wcode[KMG_FEAT_MAXW];
  __shared__ uint32_t wbad[KMG_FEAT_MAXW];
  const int64_t i = row0 + blockIdx.y;
  const uint8_t *x = codes + i * ldc;
  const int len = lens[i];
  // window starts a < P: every window of the row (window == 0), else the fixed range
  // range(window - k + 1) clipped to the windows that hold k symbols of the row
  int P = (window > 0 ? min(window, len) : len) - k + 1;
  P = max(0, min(P, KMG_FEAT_MAXW));
  for (int a = threadIdx.x; a < P; a += FT_THREADS) {
    uint32_t c = 0, b = 0;
    for (int p = 0; p < k; ++p) {
      const uint32_t s = x[a + p];
      c = (c << 2) | (s & 3u);
      b = (b << 2) | (s > 3u ? 1u : 0u);
    }
    wcode[a] = c;
    wbad[a] = b;
  }
  __syncthreads();
  const uint32_t M = k >= 16 ? 0x55555555u : (0x55555555u & ((1u << (2 * k)) - 1u));
  const int64_t j0 = (int64_t)blockIdx.x * FT_TILE + threadIdx.x;
  uint32_t cv[FT_COLS];
  int cnt[FT_COLS];
#pragma unroll
  for (int t = 0; t < FT_COLS; ++t) {
    const int64_t j = j0 + (int64_t)t * FT_THREADS;
    cv[t] = j < ncols ? cols[j] : KMG_INVALID;
    cnt[t] = 0;
  }
  for (int a = 0; a < P; ++a) {
    const uint32_t c = wcode[a], b = wbad[a];
#pragma unroll
    for (int t = 0; t < FT_COLS; ++t) {
      const uint32_t d = c ^ cv[t];
      cnt[t] += __popc(((d | (d >> 1)) & M) | b) <= (uint32_t)m ? 1 : 0;
    }
  }
  double *row = out + (int64_t)blockIdx.y * ld;
#pragma unroll
  for (int t = 0; t < FT_COLS; ++t) {
    const int64_t j = j0 + (int64_t)t * FT_THREADS;
    if (j < ncols) {
      const int v = cv[t] == KMG_INVALID ? 0 : (binary ? min(cnt[t], 1) : cnt[t]);
      row[j] = (double)v;
    }
  }
}

// Symbol columns (kmg_features_sym): a column is k symbol codes (16 bytes, bytes >= k unused),
// in the same code space as the rows, so any symbol compares by identity -- get_phi_u's string
// equality for betas holding letters outside A/C/G/T (a beta 'GTN' equals the window 'GTN',
// kernels.py:23-24), get_phi_km's integer comparison of format()ed values outside 1..4
// (kernels.py:174).  Window a of a row of length len: the symbols x[a .. a + ln), ln =
// max(0, min(k, len - a)); with `bcast` (get_phi_km on a row shorter than its window) the
// reference's numpy broadcasting of a short k-mer is reproduced: 1 symbol compares against
// every letter of the beta, 0 symbols (k = 1) mismatch nothing (an empty sum, <= m).  Other
// short windows raise in the reference and are refused by the host before the launch.
// mismatches(window, column) = number of differing bytes among the first k.
__global__ __launch_bounds__(FT_THREADS) void features_sym_kernel(
    const uint8_t *__restrict__ codes, const int32_t *__restrict__ lens, int64_t ldc, int64_t row0,
    int k, int m, int window, int bcast, const uint4 *__restrict__ cols, int64_t ncols,
    double *__restrict__ out, int64_t ld) {
  __shared__ uint4 wpat[KMG_FEAT_MAXW];
  __shared__ uint32_t wuse[KMG_FEAT_MAXW];  // 1: the window compares, 0: counts as a match
  const int64_t i = row0 + blockIdx.y;
  const uint8_t *x = codes + i * ldc;
  const int len = lens[i];
  int P;
  if (window > 0) P = bcast ? window - k + 1 : min(window, len) - k + 1;
  else P = len - k + 1;
  P = max(0, min(P, KMG_FEAT_MAXW));
  for (int a = threadIdx.x; a < P; a += FT_THREADS) {
    const int ln = max(0, min(k, len - a));
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (int q = 0; q < k; ++q) {
      const uint32_t sym = ln == k ? x[a + q] : ln == 1 ? x[a] : 0u;
      w[q >> 2] |= sym << (8 * (q & 3));
    }
    wpat[a] = make_uint4(w[0], w[1], w[2], w[3]);
    wuse[a] = ln > 0 ? 1u : 0u;
  }
  __syncthreads();
  const int nw = (k + 3) >> 2;
  uint32_t km[4];  // the bytes that count
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int nb = min(4, max(0, k - 4 * q));
    km[q] = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
  }
  const int64_t j0 = (int64_t)blockIdx.x * FT_TILE + threadIdx.x;
  uint4 cv[FT_COLS];
  int cnt[FT_COLS];
#pragma unroll
  for (int t = 0; t < FT_COLS; ++t) {
    const int64_t j = j0 + (int64_t)t * FT_THREADS;
    cv[t] = j < ncols ? cols[j] : make_uint4(0, 0, 0, 0);
    cnt[t] = 0;
  }
  for (int a = 0; a < P; ++a) {
    const uint4 wp = wpat[a];
    const uint32_t use = wuse[a];
    const uint32_t ww[4] = {wp.x, wp.y, wp.z, wp.w};
#pragma unroll
    for (int t = 0; t < FT_COLS; ++t) {
      const uint32_t cc[4] = {cv[t].x, cv[t].y, cv[t].z, cv[t].w};
      uint32_t mis = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q < nw) {
          const uint32_t d = (ww[q] ^ cc[q]) & km[q];
          // a byte is non-zero iff its top bit is set after adding 0x7F to its low 7 bits
          mis += __popc((((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u);
        }
      }
      cnt[t] += (use ? mis : 0u) <= (uint32_t)m ? 1 : 0;
    }
  }
  double *row = out + (int64_t)blockIdx.y * ld;
#pragma unroll
  for (int t = 0; t < FT_COLS; ++t) {
    const int64_t j = j0 + (int64_t)t * FT_THREADS;
    if (j < ncols) row[j] = (double)cnt[t];
  }
}

hipError_t launch_features_sym(const uint8_t *codes, const int32_t *lens, int64_t ldc, int64_t row0,
                               int64_t rows, int k, int m, int window, int bcast, const uint4 *cols,
                               int64_t ncols, double *out, int64_t ld, hipStream_t s) {
  if (rows <= 0 || ncols <= 0) return hipSuccess;
  if (k < 1 || k > 16 || rows > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((ncols + FT_TILE - 1) / FT_TILE), (unsigned)rows);
  hipLaunchKernelGGL(features_sym_kernel, grid, dim3(FT_THREADS), 0, s, codes, lens, ldc, row0, k,
                     m, window, bcast, cols, ncols, out, ld);
  return hipGetLastError();
}

hipError_t launch_features(const uint8_t *codes, const int32_t *lens, int64_t ldc, int64_t row0,
                           int64_t rows, int k, int m, int window, int binary,
                           const uint32_t *cols, int64_t ncols, double *out, int64_t ld,
                           hipStream_t s) {
  if (rows <= 0 || ncols <= 0) return hipSuccess;
  if (k < 1 || k > 16 || rows > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((ncols + FT_TILE - 1) / FT_TILE), (unsigned)rows);
  hipLaunchKernelGGL(features_kernel, grid, dim3(FT_THREADS), 0, s, codes, lens, ldc, row0, k, m,
                     window, binary, cols, ncols, out, ld);
  return hipGetLastError();
}

}  // namespace kmg
