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

// B[i][j] = (s_i * K[i][j]) * s_j  (s == nullptr: K[i][j]),  B[i][i] += shift (+ dvec[i]).
// One workgroup per row slice; 2 doubles per lane per step, rows contiguous.
__global__ __launch_bounds__(SV_THREADS) void shift_scale_kernel(const double *__restrict__ K,
                                                                 int64_t ldk,
                                                                 const double *__restrict__ s,
                                                                 double shift,
                                                                 const double *__restrict__ dvec,
                                                                 int64_t n,
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
    if (j == i) v = __dadd_rn(v, dvec ? __dadd_rn(shift, dvec[i]) : shift);
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
                              const double *dvec, int64_t n, double *B, int64_t ldb,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t xb = (n + SV_THREADS - 1) / SV_THREADS;
  dim3 grid((unsigned)(xb < 8 ? xb : 8), (unsigned)n);
  shift_scale_kernel<<<grid, SV_THREADS, 0, st>>>(K, ldk, s, shift, dvec, n, B, ldb);
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

// ------------------------------------------------------------------ C-SVM dual QP
// C_SVM.fit, solver 'CVX' (SVM.py:78-89): cvxopt.solvers.qp(P=K, q=-y, G=[diag(y); -diag(y)],
// h=[C; 0]), i.e. min 1/2 a'Ka - y'a subject to 0 <= y_i a_i <= C.  With x = y o a the box
// is 0 <= x <= C and Q = YKY.  Solved by a Mehrotra predictor-corrector primal-dual
// interior-point method (the method family of cvxopt.solvers.qp); every Newton system is
// (Q + diag(z1/x + z2/(C-x))) dx = rhs, factorised once per iteration by rocSOLVER.
// These single-workgroup kernels do the O(n) work between the GEMV and the factorisation
// (n <= a few 10^4: one workgroup of 1024 lanes is microseconds).
// Vector block layout (n doubles each): x z1 z2 rd D dxa dz1a dz2a v u rhs.
struct SvmVec {
  double *x, *z1, *z2, *rd, *D, *dxa, *dz1a, *dz2a, *v, *u, *rhs;
};

__device__ double block_sum(double a, double *red) {
  red[threadIdx.x] = a;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__device__ double block_min(double a, double *red) {
  red[threadIdx.x] = a;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = fmin(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__device__ double block_max(double a, double *red) { return -block_min(-a, red); }

// largest step t keeping x + t dx in [0, C] and z + t dz >= 0 (per lane; +inf if unbounded)
__device__ __forceinline__ double max_step(double x, double dx, double z1, double dz1, double z2,
                                           double dz2, double C) {
  double t = INFINITY;
  if (dx < 0) t = fmin(t, -x / dx);
  if (dx > 0) t = fmin(t, (C - x) / dx);
  if (dz1 < 0) t = fmin(t, -z1 / dz1);
  if (dz2 < 0) t = fmin(t, -z2 / dz2);
  return t;
}

// mode 0: v = y o x (the GEMV input).  mode 1 (after u = K v): residual rd = y o u - 1 - z1
// + z2, D = z1/x + z2/(C-x), predictor rhs = -rd - z1 + z2; sc = {mu, ||rd||_inf, obj}
__global__ __launch_bounds__(1024) void svm_resid_kernel(int mode, const double *__restrict__ y,
                                                         int64_t n, double C, SvmVec V,
                                                         double *__restrict__ sc) {
  __shared__ double red[1024];
  if (mode == 0) {
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) V.v[i] = y[i] * V.x[i];
    return;
  }
  double gap = 0.0, rinf = 0.0, obj = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = V.x[i], s2 = C - x, z1 = V.z1[i], z2 = V.z2[i];
    const double qx = y[i] * V.u[i];
    const double rd = qx - 1.0 - z1 + z2;
    V.rd[i] = rd;
    V.D[i] = z1 / x + z2 / s2;
    V.rhs[i] = -rd - z1 + z2;
    gap += x * z1 + s2 * z2;
    rinf = fmax(rinf, fabs(rd));
    obj += 0.5 * x * qx - x;
  }
  gap = block_sum(gap, red);
  rinf = block_max(rinf, red);
  obj = block_sum(obj, red);
  if (threadIdx.x == 0) {
    sc[0] = gap / (2.0 * (double)n);
    sc[1] = rinf;
    sc[2] = obj;
  }
}

// after the predictor solve (rhs = dx_aff): dz_aff, the affine step and mu_aff -> sc[3];
// then the corrector rhs for sigma = (mu_aff / mu)^3 (computed here from sc[0])
__global__ __launch_bounds__(1024) void svm_affine_kernel(int64_t n, double C, SvmVec V,
                                                          double *__restrict__ sc) {
  __shared__ double red[1024];
  double t = INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = V.x[i], s2 = C - x, z1 = V.z1[i], z2 = V.z2[i], dx = V.rhs[i];
    const double dz1 = (-x * z1 - z1 * dx) / x;
    const double dz2 = (-s2 * z2 + z2 * dx) / s2;
    V.dxa[i] = dx;
    V.dz1a[i] = dz1;
    V.dz2a[i] = dz2;
    t = fmin(t, max_step(x, dx, z1, dz1, z2, dz2, C));
  }
  t = fmin(1.0, block_min(t, red));
  double g = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = V.x[i], dx = V.dxa[i];
    g += (x + t * dx) * (V.z1[i] + t * V.dz1a[i]) + (C - x - t * dx) * (V.z2[i] + t * V.dz2a[i]);
  }
  g = block_sum(g, red);
  const double mu = sc[0], mu_aff = g / (2.0 * (double)n);
  const double ratio = mu > 0 ? mu_aff / mu : 0.0;
  const double smu = ratio * ratio * ratio * mu;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = V.x[i], s2 = C - x, z1 = V.z1[i], z2 = V.z2[i];
    const double t1 = smu - x * z1 - V.dxa[i] * V.dz1a[i];
    const double t2 = smu - s2 * z2 + V.dxa[i] * V.dz2a[i];
    V.rhs[i] = -V.rd[i] + t1 / x - t2 / s2;
    V.dz1a[i] = t1;  // keep t1, t2 for the step kernel
    V.dz2a[i] = t2;
  }
  if (threadIdx.x == 0) {
    sc[3] = mu_aff;
    sc[4] = smu;
  }
}

// after the corrector solve (rhs = dx): dz, common step 0.99 * max, update x, z1, z2
__global__ __launch_bounds__(1024) void svm_step_kernel(int64_t n, double C, SvmVec V,
                                                        double *__restrict__ sc) {
  __shared__ double red[1024];
  double t = INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double x = V.x[i], s2 = C - x, z1 = V.z1[i], z2 = V.z2[i], dx = V.rhs[i];
    const double dz1 = (V.dz1a[i] - z1 * dx) / x;
    const double dz2 = (V.dz2a[i] + z2 * dx) / s2;
    V.dz1a[i] = dz1;
    V.dz2a[i] = dz2;
    t = fmin(t, max_step(x, dx, z1, dz1, z2, dz2, C));
  }
  t = fmin(1.0, 0.99 * block_min(t, red));  // fraction to the boundary
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    V.x[i] += t * V.rhs[i];
    V.z1[i] += t * V.dz1a[i];
    V.z2[i] += t * V.dz2a[i];
  }
  if (threadIdx.x == 0) sc[5] = t;
}

__global__ void svm_init_kernel(int64_t n, double C, SvmVec V) {
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    V.x[i] = 0.5 * C;
    V.z1[i] = 1.0;
    V.z2[i] = 1.0;
  }
}

// flag[0] := 1 if K != K^T anywhere (bitwise compare of the upper triangle with the
// lower): 32 x 32 tiles staged through LDS so both reads are row-contiguous
__global__ __launch_bounds__(256) void asym_kernel(const double *__restrict__ K, int64_t ld,
                                                   int64_t n, int *__restrict__ flag) {
  __shared__ double t[32][33];
  const int64_t bi = blockIdx.y, bj = blockIdx.x;
  if (bj < bi) return;  // upper tile (bi, bj) against the transpose of (bj, bi)
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8) {
    const int64_t gi = bj * 32 + r, gj = bi * 32 + tx;
    if (gi < n && gj < n) t[r][tx] = K[gi * ld + gj];
  }
  __syncthreads();
  bool diff = false;
  for (int r = ty; r < 32; r += 8) {
    const int64_t gi = bi * 32 + r, gj = bj * 32 + tx;
    if (gi < n && gj < n)
      diff |= __double_as_longlong(K[gi * ld + gj]) != __double_as_longlong(t[tx][r]);
  }
  if (__any(diff) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

hipError_t launch_asymmetry(const double *K, int64_t ld, int64_t n, int *flag, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nt = (n + 31) / 32;
  if (nt > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(asym_kernel, dim3((unsigned)nt, (unsigned)nt), dim3(256), 0, st, K, ld, n, flag);
  return hipGetLastError();
}

// a = y o x (the reference's alpha: cvxopt's solution vector)
__global__ void svm_alpha_kernel(const double *__restrict__ y, int64_t n, const double *x,
                                 double *a) {
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) a[i] = y[i] * x[i];
}

hipError_t launch_svm(int phase, const double *y, int64_t n, double C, double *vec,
                      double *sc, double *alpha, hipStream_t st) {
  SvmVec V;
  double **f[] = {&V.x, &V.z1, &V.z2, &V.rd, &V.D, &V.dxa, &V.dz1a, &V.dz2a, &V.v, &V.u, &V.rhs};
  for (int q = 0; q < 11; ++q) *f[q] = vec + (size_t)q * n;
  switch (phase) {
    case 0: svm_init_kernel<<<1, 1024, 0, st>>>(n, C, V); break;
    case 1: svm_resid_kernel<<<1, 1024, 0, st>>>(0, y, n, C, V, sc); break;
    case 2: svm_resid_kernel<<<1, 1024, 0, st>>>(1, y, n, C, V, sc); break;
    case 3: svm_affine_kernel<<<1, 1024, 0, st>>>(n, C, V, sc); break;
    case 4: svm_step_kernel<<<1, 1024, 0, st>>>(n, C, V, sc); break;
    case 5: svm_alpha_kernel<<<1, 1024, 0, st>>>(y, n, V.x, alpha); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kmg
