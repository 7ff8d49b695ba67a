// kmg_solve.hip — elementwise/reduction kernels of the dense learners on K.
//
// Reference consumers of the Gram (afiliot/Kernel-Methods-For-Genomics):
//   KRR.fit    KRR.py:33      a = inv(K_fit + lbda*n*I) . y
//   KLR.IRLS   KLR.py:30-42   m = K.alpha, W = s(m) s(-m), z = m + y / s(-y m)
//   KLR.WKRR   KLR.py:44-55   alpha = W_s inv(W_s K W_s + n*lbda*I) W_s z
//   KLR.fit    KLR.py:57-75   loop while ||alpha - alpha_prev||_2 > tol, <= maxiter times
// The factorisation itself (Cholesky, LU fallback) is rocSOLVER's (kmg_api.cpp); these
// kernels build the shifted / scaled matrix in one HBM pass and do the O(n) vector work
// between factorisations.  All HBM-bound (8 B read + 8 B write per matrix element).
#include "kmg_internal.h"

namespace kmg {

constexpr int SV_THREADS = 256;

// B[i][j] = (s_i * K[i][j]) * s_j  (s == nullptr: K[i][j]),  B[i][i] += shift.
// One workgroup per row slice; 2 doubles per lane per step, rows contiguous.
__global__ __launch_bounds__(SV_THREADS) void shift_scale_kernel(const double *__restrict__ K,
                                                                 int64_t ldk,
                                                                 const double *__restrict__ s,
                                                                 double shift, int64_t n,
                                                                 double *__restrict__ B,
                                                                 int64_t ldb) {
  const int64_t i = blockIdx.y;
  const double si = s ? s[i] : 1.0;
  const double *kr = K + i * ldk;
  double *br = B + i * ldb;
  for (int64_t j = (int64_t)blockIdx.x * SV_THREADS + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * SV_THREADS) {
    double v = kr[j];
    if (s) v = __dmul_rn(__dmul_rn(si, v), s[j]);
    if (j == i) v = __dadd_rn(v, shift);
    br[j] = v;
  }
}

__device__ __forceinline__ double sigmoid(double x) { return 1.0 / (1.0 + exp(-x)); }

// IRLS step (KLR.py:30-42) + the right-hand side of WKRR: s = sqrt(W), rhs = s * z
__global__ __launch_bounds__(SV_THREADS) void irls_kernel(const double *__restrict__ m,
                                                          const double *__restrict__ y, int64_t n,
                                                          double *__restrict__ s,
                                                          double *__restrict__ rhs) {
  const int64_t i = (int64_t)blockIdx.x * SV_THREADS + threadIdx.x;
  if (i >= n) return;
  const double mi = m[i], yi = y[i];
  const double W = __dmul_rn(sigmoid(mi), sigmoid(-mi));
  const double z = __dadd_rn(mi, yi / sigmoid(__dmul_rn(-yi, mi)));
  const double si = sqrt(W);
  s[i] = si;
  rhs[i] = __dmul_rn(si, z);
}

// alpha = s * x; out[0] = sum (alpha - prev)^2 (single workgroup, fixed order per n)
__global__ __launch_bounds__(1024) void scale_diff_kernel(const double *__restrict__ s,
                                                          const double *__restrict__ x,
                                                          const double *__restrict__ prev,
                                                          int64_t n, double *__restrict__ alpha,
                                                          double *__restrict__ out) {
  __shared__ double red[1024];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double a = __dmul_rn(s[i], x[i]);
    alpha[i] = a;
    const double d = __dadd_rn(a, -prev[i]);
    acc = __dadd_rn(acc, __dmul_rn(d, d));
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = __dadd_rn(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

hipError_t launch_shift_scale(const double *K, int64_t ldk, const double *s, double shift,
                              int64_t n, double *B, int64_t ldb, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t xb = (n + SV_THREADS - 1) / SV_THREADS;
  dim3 grid((unsigned)(xb < 8 ? xb : 8), (unsigned)n);
  shift_scale_kernel<<<grid, SV_THREADS, 0, st>>>(K, ldk, s, shift, n, B, ldb);
  return hipGetLastError();
}

hipError_t launch_irls(const double *m, const double *y, int64_t n, double *s, double *rhs,
                       hipStream_t st) {
  if (n <= 0) return hipSuccess;
  irls_kernel<<<(unsigned)((n + SV_THREADS - 1) / SV_THREADS), SV_THREADS, 0, st>>>(m, y, n, s,
                                                                                    rhs);
  return hipGetLastError();
}

hipError_t launch_scale_diff(const double *s, const double *x, const double *prev, int64_t n,
                             double *alpha, double *out, hipStream_t st) {
  scale_diff_kernel<<<1, 1024, 0, st>>>(s, x, prev, n, alpha, out);
  return hipGetLastError();
}

}  // namespace kmg
