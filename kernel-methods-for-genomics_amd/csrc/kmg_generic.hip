// kmg_generic.hip — generic per-pair kernels for the parameter ranges the specialised
// kernels do not cover (gfx950).  One lane per pair (i, j), the row i staged once in LDS
// for the 256 pairs of a block; O(L_x L_y) byte work per pair along the diagonals:
//
//   spectrum, any k > 16 (the posting-list / dense / Hamming kernels pack k-mers in 32
//     bits):  K(x, y) = #{(a, b) : x[a:a+k] == y[b:b+k], both all-ACGT}, the reference's
//     get_phi_u count over 4^k betas (kernels.py:12-47; a window holding another character
//     equals no beta).  Along each diagonal a run of equal ACGT symbols of length r holds
//     max(0, r - k + 1) equal windows.
//   mismatch (k, m), any k > 16:  K(x, y) = sum_{a,b} w[ham(x_a, y_b)] over the windows
//     a, b < 101 - k + 1 of the fixed window (kernels.py:161-175, 196-217; the closed form
//     of <Phi_x, Phi_y>, w from mismatch_weights), ham by a sliding count of mismatches
//     along each diagonal; the diagonal K(x, x) feeds the fused normalize_K.
//   WD with shifts, any S > 15:  get_WDShifts_d (kernels.py:115-135) term by term in the
//     reference's order (k, then i, then s), each slice comparison with Python's clipped-
//     slice semantics (equal iff same clipped length and same symbols).
// The reference itself needs 4^k betas in memory for spectrum / mismatch (k = 17: 17e9
// strings), so past k = 16 these values have no reference run to pin them; the kernels
// are checked against the oracle's direct restatements (tests/test_gpu_generic.py).
#include "kmg_internal.h"

namespace kmg {

namespace {

constexpr int GEN_THREADS = 256;
constexpr int GEN_MAXL = 4096;  // staged row bytes (LDS)

__device__ __forceinline__ void gen_store(const OutSpec &o, int64_t il, int64_t j, double v) {
  if (o.dtype == KMG_F64)
    ((double *)o.out)[il * o.ld + j] = v;
  else if (o.dtype == KMG_F32)
    ((float *)o.out)[il * o.ld + j] = (float)v;
  else
    ((int32_t *)o.out)[il * o.ld + j] = (int32_t)v;
}

// row i's symbols into LDS (every thread of the block), returns its length
__device__ __forceinline__ int stage_row(const SeqSpec &q, int64_t i, uint8_t *xs, int lim) {
  const int Lx = min(q.lens[i], lim);
  const uint8_t *src = q.codes + i * q.ldc;
  for (int t = threadIdx.x; t < Lx; t += blockDim.x) xs[t] = src[t];
  __syncthreads();
  return Lx;
}

// equal all-ACGT windows of length k along every diagonal of (x, y)
__device__ int64_t spectrum_pair(const uint8_t *x, int Lx, const uint8_t *y, int Ly, int k) {
  int64_t cnt = 0;
  for (int dlt = -(Ly - 1); dlt <= Lx - 1; ++dlt) {
    const int ox = max(dlt, 0), oy = max(-dlt, 0);
    const int len = min(Lx - ox, Ly - oy);
    int run = 0;
    for (int t = 0; t < len; ++t) {
      const uint32_t a = x[ox + t], b = y[oy + t];
      run = (a == b && a <= 3u) ? run + 1 : 0;
      cnt += run >= k ? 1 : 0;
    }
  }
  return cnt;
}

// sum over window pairs of w[ham]: windows start below P = W - k + 1 in both rows.  A
// window that reaches past its row's length or holds a non-ACGT symbol is invalid and
// weighs nothing, as in the packed k <= 16 kernels (pk_window); x and y are read only
// below their lengths, so padding bytes never enter.
__device__ __forceinline__ uint32_t sym_at(const uint8_t *x, int Lx, int p) {
  return p < Lx ? (uint32_t)x[p] : 0xFFu;  // 0xFF: past the row (invalid)
}

__device__ int64_t mismatch_pair(const uint8_t *x, int Lx, const uint8_t *y, int Ly, int W,
                                 int k, const int64_t *w, int maxd) {
  const int P = W - k + 1;
  int64_t tot = 0;
  for (int dlt = -(P - 1); dlt <= P - 1; ++dlt) {
    const int ox = max(dlt, 0), oy = max(-dlt, 0);
    // window starts t = 0 .. P - 1 - max(ox, oy) along this diagonal
    const int nwin = P - max(ox, oy);
    int h = 0, bad = 0;  // mismatches / invalid symbols (either row) inside the window
    auto step = [&](int t, int sgn) {
      const uint32_t a = sym_at(x, Lx, ox + t), b = sym_at(y, Ly, oy + t);
      h += sgn * (a != b ? 1 : 0);
      bad += sgn * ((a > 3u ? 1 : 0) + (b > 3u ? 1 : 0));
    };
    for (int t = 0; t < k; ++t) step(t, 1);
    for (int t = 0; t < nwin; ++t) {
      if (t > 0) {
        step(t + k - 1, 1);
        step(t - 1, -1);
      }
      tot += (bad == 0 && h <= maxd) ? w[h] : 0;
    }
  }
  return tot;
}

}  // namespace

// normalize_K (kernels.py:398-415) as the fused epilogues evaluate it
__device__ __forceinline__ double gen_norm(const OutSpec &o, int64_t r, int64_t c, int64_t raw) {
  if (!o.normalize || o.diagv[0] == 1.0) return (double)raw;
  return r == c ? 1.0 : (double)raw / (o.dsq[r] * o.dsq[c]);
}

__global__ __launch_bounds__(GEN_THREADS) void gram_sp_generic_kernel(SeqSpec q, int64_t row0,
                                                                      int64_t row1, int k,
                                                                      int mirror, OutSpec o) {
  __shared__ uint8_t xs[GEN_MAXL];
  const int64_t i = row0 + blockIdx.y;
  const int64_t jb = (mirror ? i : 0) + (int64_t)blockIdx.x * blockDim.x;
  if (i >= row1 || jb >= q.n) return;  // block-uniform
  const int Lx = stage_row(q, i, xs, GEN_MAXL);
  const int64_t j = jb + threadIdx.x;
  if (j >= q.n) return;
  const int Ly = q.lens[j];
  const int64_t v = (Lx < k || Ly < k) ? 0 : spectrum_pair(xs, Lx, q.codes + j * q.ldc, Ly, k);
  gen_store(o, i - row0, j, gen_norm(o, i, j, v));
  if (mirror && j != i && j >= row0 && j < row1) gen_store(o, j - row0, i, gen_norm(o, j, i, v));
}

// spectrum K(x, x) of every row (the fused normalize_K's diagonal)
__global__ __launch_bounds__(GEN_THREADS) void sp_generic_diag_kernel(SeqSpec q, int k,
                                                                      double *diagv, double *dsq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q.n) return;
  const uint8_t *x = q.codes + i * q.ldc;
  const int Lx = min(q.lens[i], GEN_MAXL);
  const double d = (Lx < k) ? 0.0 : (double)spectrum_pair(x, Lx, x, Lx, k);
  diagv[i] = d;
  dsq[i] = sqrt(d);
}

__global__ __launch_bounds__(GEN_THREADS) void mm_generic_diag_kernel(SeqSpec q, int W, int k,
                                                                      const int64_t *__restrict__ w,
                                                                      int maxd, double *diagv,
                                                                      double *dsq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q.n) return;
  const uint8_t *x = q.codes + i * q.ldc;
  const int Lx = min(q.lens[i], W);
  const double d = (double)mismatch_pair(x, Lx, x, Lx, W, k, w, maxd);
  diagv[i] = d;
  dsq[i] = sqrt(d);
}

__global__ __launch_bounds__(GEN_THREADS) void gram_mm_generic_kernel(SeqSpec q, int64_t row0,
                                                                      int64_t row1, int W, int k,
                                                                      const int64_t *__restrict__ w,
                                                                      int maxd, int mirror,
                                                                      OutSpec o) {
  __shared__ uint8_t xs[GEN_MAXL];
  const int64_t i = row0 + blockIdx.y;
  const int64_t jb = (mirror ? i : 0) + (int64_t)blockIdx.x * blockDim.x;
  if (i >= row1 || jb >= q.n) return;  // block-uniform
  const int Lx = stage_row(q, i, xs, W);
  const int64_t j = jb + threadIdx.x;
  if (j >= q.n) return;
  const int64_t raw =
      mismatch_pair(xs, Lx, q.codes + j * q.ldc, min(q.lens[j], W), W, k, w, maxd);
  gen_store(o, i - row0, j, gen_norm(o, i, j, raw));
  if (mirror && j != i && j >= row0 && j < row1) gen_store(o, j - row0, i, gen_norm(o, j, i, raw));
}

// Python slice equality x[a:a+k] == y[b:b+k]: both clipped to their row, equal iff the
// clipped lengths agree and the symbols do (two empty slices are equal)
__device__ __forceinline__ int slice_eq(const uint8_t *x, int Lx, int a, const uint8_t *y, int Ly,
                                        int b, int k) {
  const int la = max(0, min(k, Lx - a)), lb = max(0, min(k, Ly - b));
  if (la != lb) return 0;
  for (int t = 0; t < la; ++t)
    if (x[a + t] != y[b + t]) return 0;
  return 1;
}

// wd_diag: get_WD_K (the WD form, S = 0 with delta_0 = 1/2 so a match adds exactly 1.0):
// the diagonal is the closed form L - 1 + (1 - d) / 3 (kernels.py:96)
__global__ __launch_bounds__(GEN_THREADS) void gram_wds_generic_kernel(
    SeqSpec q, int64_t row0, int64_t row1, int d, int S, int span,
    const double *__restrict__ coef_a, const double *__restrict__ coef_b, int wd_diag, int mirror,
    OutSpec o) {
  __shared__ uint8_t xs[GEN_MAXL];
  const int64_t i = row0 + blockIdx.y;
  const int64_t jb = (mirror ? i : 0) + (int64_t)blockIdx.x * blockDim.x;
  if (i >= row1 || jb >= q.n) return;  // block-uniform
  const int Li = stage_row(q, i, xs, GEN_MAXL);
  const int64_t j = jb + threadIdx.x;
  if (j >= q.n) return;
  // x = the row of the smaller index (the reference fills j >= i, kernels.py:150-154)
  const bool rowx = i <= j;
  const uint8_t *yrow = q.codes + j * q.ldc;
  const uint8_t *x = rowx ? xs : yrow;
  const uint8_t *y = rowx ? yrow : xs;
  const int Lx = rowx ? Li : q.lens[j], Ly = rowx ? q.lens[j] : Li;
  const int L = span > 0 ? span : Lx;  // get_WDShifts_d's L = len(x)
  double ct = 0.0;
  if (wd_diag && i == j) {
    ct = __dadd_rn((double)(Li - 1), (double)(1 - d) / 3.0);
    gen_store(o, i - row0, j, ct);
    return;
  }
  for (int k = 1; k <= d; ++k) {
    double cst = 0.0;
    for (int ii = 1; ii < L - k + 1; ++ii)
      for (int s = 0; s <= S; ++s)
        if (s + ii < L) {
          const int m = slice_eq(x, Lx, ii + s, y, Ly, ii, k) + slice_eq(x, Lx, ii, y, Ly, ii + s, k);
          if (m) cst = __dadd_rn(cst, __dmul_rn(coef_b[s], (double)m));
        }
    ct = __dadd_rn(ct, __dmul_rn(coef_a[k - 1], cst));
  }
  gen_store(o, i - row0, j, ct);
  if (mirror && j != i && j >= row0 && j < row1) gen_store(o, j - row0, i, ct);
}

namespace {
dim3 gen_grid(const SeqSpec &q, int64_t row0, int64_t rows, int mirror) {
  const int64_t cols = mirror ? q.n - row0 : q.n;
  return dim3((unsigned)((cols + GEN_THREADS - 1) / GEN_THREADS), (unsigned)rows);
}
}  // namespace

hipError_t launch_gram_sp_generic(const SeqSpec &q, int64_t row0, int64_t row1, int k, int mirror,
                                  const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  if (rows > 65535 || q.maxlen > GEN_MAXL) return hipErrorNotSupported;
  hipLaunchKernelGGL(gram_sp_generic_kernel, gen_grid(q, row0, rows, mirror), dim3(GEN_THREADS), 0,
                     s, q, row0, row1, k, mirror, o);
  return hipGetLastError();
}

hipError_t launch_sp_generic_diag(const SeqSpec &q, int k, double *diagv, double *dsq,
                                  hipStream_t s) {
  if (q.n == 0) return hipSuccess;
  if (q.maxlen > GEN_MAXL) return hipErrorNotSupported;
  hipLaunchKernelGGL(sp_generic_diag_kernel, dim3((unsigned)((q.n + GEN_THREADS - 1) / GEN_THREADS)),
                     dim3(GEN_THREADS), 0, s, q, k, diagv, dsq);
  return hipGetLastError();
}

hipError_t launch_mm_generic_diag(const SeqSpec &q, int W, int k, const int64_t *w, int maxd,
                                  double *diagv, double *dsq, hipStream_t s) {
  if (q.n == 0) return hipSuccess;
  hipLaunchKernelGGL(mm_generic_diag_kernel, dim3((unsigned)((q.n + GEN_THREADS - 1) / GEN_THREADS)),
                     dim3(GEN_THREADS), 0, s, q, W, k, w, maxd, diagv, dsq);
  return hipGetLastError();
}

hipError_t launch_gram_mm_generic(const SeqSpec &q, int64_t row0, int64_t row1, int W, int k,
                                  const int64_t *w, int maxd, int mirror, const OutSpec &o,
                                  hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  if (rows > 65535 || W > GEN_MAXL) return hipErrorNotSupported;
  hipLaunchKernelGGL(gram_mm_generic_kernel, gen_grid(q, row0, rows, mirror), dim3(GEN_THREADS), 0,
                     s, q, row0, row1, W, k, w, maxd, mirror, o);
  return hipGetLastError();
}

hipError_t launch_gram_wds_generic(const SeqSpec &q, int64_t row0, int64_t row1, int d, int S,
                                   int span, const double *coef_a, const double *coef_b,
                                   int wd_diag, int mirror, const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  if (rows > 65535 || q.maxlen > GEN_MAXL) return hipErrorNotSupported;
  hipLaunchKernelGGL(gram_wds_generic_kernel, gen_grid(q, row0, rows, mirror), dim3(GEN_THREADS), 0,
                     s, q, row0, row1, d, S, span, coef_a, coef_b, wd_diag, mirror, o);
  return hipGetLastError();
}

}  // namespace kmg
