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

// ------------------------------------------------------------------ blocked Cholesky
// The diagonal blocks (nb <= CHOL_NB) of the right-looking blocked Cholesky (kmg_api.cpp
// chol_factor).  chol_diag_kernel factorises one block with one 1024-thread workgroup, the
// block held in registers 2-D block-cyclic: thread t owns rows (t & 31) + 32 i and columns
// (t >> 5) + 32 j, so the shrinking trailing triangle stays spread over all threads.  A step
// publishes columns j, j+1 through LDS (double-buffered: one barrier a step) and every owner
// of a trailing element subtracts their rank-2 term; the columns are scaled by 1/sqrt of
// their pivots at the end.  The step loop is latency-bound (the chain of 128 pivots); a version blocked by
// 32-column panels with the pivot chain in one wave measured slower (314 vs 193 us a block
// with the inverse; profiles/r05be_*), since one wave hides none of the LDS and fp64 latency.
// A pivot <= 0 (or NaN) sets *info = j0 + j + 1 and leaves the block: the caller rebuilds and
// falls back to LU, and every later block returns at once.
constexpr int CHOL_NB = 128;
constexpr int CHOL_SWEEP_ROWS = 128;       // rows of b a tri_sweep workgroup updates
constexpr int CHOL_RT = 32;                // rows (and columns) of the thread grid
constexpr int CHOL_S = CHOL_NB / CHOL_RT;  // owned rows / columns a thread

// 1/d to within an ulp or so: v_rcp_f64 and two Newton steps (a division's fix-up
// sequence is ~3x the instructions, on every wave of the step loop)
__device__ __forceinline__ double chol_recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
  return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
}

__global__ __launch_bounds__(1024) void chol_diag_kernel(double *__restrict__ A, int64_t lda, int nb,
                                                         int j0, int *__restrict__ info) {
  __shared__ double cb[2][2][CHOL_NB];  // [step parity][column j / j+1]
  if (*info != 0) return;               // an earlier block failed
  const int r0 = (int)threadIdx.x & (CHOL_RT - 1), c0 = (int)threadIdx.x / CHOL_RT;
  // Slots (ri, ci) with ri < ci lie above the diagonal (r < 32 ri + 32 <= c): never held.
  // Slots with ri >= ci may still hold r < c or r >= nb: they are updated like the rest
  // (their values are never stored), so the step loop carries no per-element masks; the
  // column multipliers are zeroed instead where a column must not change, and slot columns
  // that are finished are skipped by a wave-uniform branch.  Each step retires two columns
  // j, j+1 behind one barrier: both are published as they stand after step j-1, and every
  // thread applies column j to the entries of column j+1 it needs itself.
  double a[CHOL_S][CHOL_S], pv[CHOL_S];
  for (int t = threadIdx.x; t < 4 * CHOL_NB; t += blockDim.x) (&cb[0][0][0])[t] = 0.0;
#pragma unroll
  for (int ri = 0; ri < CHOL_S; ++ri)
#pragma unroll
    for (int ci = 0; ci <= ri; ++ci) {
      const int r = r0 + CHOL_RT * ri, c = c0 + CHOL_RT * ci;
      a[ri][ci] = (r < nb && c < nb && r >= c) ? A[r + (int64_t)c * lda] : 0.0;
    }
#pragma unroll
  for (int ci = 0; ci < CHOL_S; ++ci) pv[ci] = 1.0;
  __syncthreads();
  for (int j = 0; j < nb; j += 2) {
    double *b0 = cb[(j >> 1) & 1][0], *b1 = cb[(j >> 1) & 1][1];
    const int j1 = j + 1;
    const bool two = j1 < nb;
    const int jq = j / CHOL_RT, jq1 = j1 / CHOL_RT;
    if (c0 == (j & (CHOL_RT - 1))) {
#pragma unroll
      for (int ci = 0; ci < CHOL_S; ++ci)
        if (ci == jq) {
#pragma unroll
          for (int ri = ci; ri < CHOL_S; ++ri) {
            const int r = r0 + CHOL_RT * ri;
            if (r >= j && r < nb) b0[r] = a[ri][ci];
          }
        }
    }
    if (two && c0 == (j1 & (CHOL_RT - 1))) {
#pragma unroll
      for (int ci = 0; ci < CHOL_S; ++ci)
        if (ci == jq1) {
#pragma unroll
          for (int ri = ci; ri < CHOL_S; ++ri) {
            const int r = r0 + CHOL_RT * ri;
            if (r >= j1 && r < nb) b1[r] = a[ri][ci];
          }
        }
    }
    __syncthreads();
    // every LDS read of the step at once (clamped, unconditional): one latency, not five
    const int jc1 = min(j1, nb - 1);
    const double d0 = b0[j], a10 = b0[jc1], a11 = b1[jc1];
    double rw0[CHOL_S], rw1[CHOL_S], cl0[CHOL_S], cl1[CHOL_S];
#pragma unroll
    for (int q = 0; q < CHOL_S; ++q) {
      const int r = min(r0 + CHOL_RT * q, nb - 1), c = min(c0 + CHOL_RT * q, nb - 1);
      rw0[q] = b0[r];
      rw1[q] = b1[r];
      cl0[q] = b0[c];
      cl1[q] = b1[c];
    }
    // (no branch between the reads and their use: a failed pivot is acted on after the
    // update, whose values are then discarded)
    const double rd0 = chol_recip(d0);
    const double l10 = two ? a10 * rd0 : 0.0;  // a_{j+1,j} / a_jj
    const double d1 = two ? __builtin_fma(-a10, l10, a11) : 1.0;
    const double rd1 = chol_recip(d1);
    // row factors: u0 = a_rj, u1 = a_r,j+1 after column j (rows below j only matter)
    double u0[CHOL_S], u1[CHOL_S];
#pragma unroll
    for (int ri = 0; ri < CHOL_S; ++ri) {
      u0[ri] = rw0[ri];
      u1[ri] = __builtin_fma(-rw0[ri], l10, rw1[ri]);
    }
    if (c0 == (j1 & (CHOL_RT - 1))) {  // column j+1 itself, after column j
#pragma unroll
      for (int ci = 0; ci < CHOL_S; ++ci)
        if (ci == jq1) {
#pragma unroll
          for (int ri = ci; ri < CHOL_S; ++ri) a[ri][ci] = u1[ri];
        }
    }
#pragma unroll
    for (int ci = 0; ci < CHOL_S; ++ci) {
      if (CHOL_RT * ci + CHOL_RT - 1 <= j1) continue;  // slot columns all <= j+1: finished
      const bool live = c0 + CHOL_RT * ci > j1;
      const double lc0 = live ? cl0[ci] * rd0 : 0.0;
      const double lc1 = live ? __builtin_fma(-cl0[ci], l10, cl1[ci]) * rd1 : 0.0;
#pragma unroll
      for (int ri = ci; ri < CHOL_S; ++ri)
        a[ri][ci] = __builtin_fma(-u1[ri], lc1, __builtin_fma(-u0[ri], lc0, a[ri][ci]));
    }
    if (!(d0 > 0.0) || !(d1 > 0.0)) {  // not positive definite (or NaN): the same in every thread
      if (threadIdx.x == 0) *info = j0 + (d0 > 0.0 ? j1 : j) + 1;
      return;
    }
#pragma unroll
    for (int ci = 0; ci < CHOL_S; ++ci) {
      if (ci == jq && c0 == (j & (CHOL_RT - 1))) pv[ci] = d0;
      if (two && ci == jq1 && c0 == (j1 & (CHOL_RT - 1))) pv[ci] = d1;
    }
    if (!two) break;
  }
  // L_rc = a_rc / sqrt(a_cc), L_cc = sqrt(a_cc)
#pragma unroll
  for (int ci = 0; ci < CHOL_S; ++ci) {
    const int c = c0 + CHOL_RT * ci;
    const double sd = __builtin_sqrt(pv[ci]), rs = 1.0 / sd;
#pragma unroll
    for (int ri = ci; ri < CHOL_S; ++ri) {
      const int r = r0 + CHOL_RT * ri;
      if (r < nb && c < nb && r >= c) A[r + (int64_t)c * lda] = r == c ? sd : a[ri][ci] * rs;
    }
  }
}

// LDS written by some lanes of the wave, read by others next (a wave's LDS ops run in order)
__device__ __forceinline__ void chol_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Y = L^-1 for one factorised diagonal block, one column of Y a workgroup: the block's
// columns are independent triangular solves L y = e_c, so the 128 pivot chains run side by
// side on 128 CUs instead of one after another.  The workgroup's 16 waves stage columns
// c.. of L in LDS (all loads in flight at once), then wave 0 alone runs the chain: lane l
// holds rows l and l + 64; step k takes y_k from its owner lane (readlane) and every row
// r > k subtracts L_rk y_k.  Writes Y and Y^T (128 x 128, ld CHOL_NB,
// zero above the diagonal and past nb).
__global__ __launch_bounds__(1024) void chol_inv_kernel(const double *__restrict__ L, int64_t lda, int nb,
                                                        const int *__restrict__ info, double *__restrict__ Y,
                                                        double *__restrict__ YT) {
  extern __shared__ __align__(16) double ls[];  // [CHOL_NB][CHOL_NB + 1], columns >= c only
  if (*info != 0) return;
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  constexpr int LD = CHOL_NB + 1;
  if (c >= nb) {  // zero column (block past nb)
    if (tid < 64) {
      Y[lane + c * CHOL_NB] = Y[lane + 64 + c * CHOL_NB] = 0.0;
      YT[c + lane * CHOL_NB] = YT[c + (lane + 64) * CHOL_NB] = 0.0;
    }
    return;
  }
  double *dinv = ls + CHOL_NB * LD;  // 1 / L_kk
  {  // stage columns c .. nb-1 with every load in flight at once (16 a thread)
    const int row = tid & (CHOL_NB - 1), k0 = c + (tid >> 7);
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = L[min(row, nb - 1) + (int64_t)min(k0 + 8 * u, nb - 1) * lda];
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (row < nb && k0 + 8 * u < nb) ls[row + (k0 + 8 * u) * LD] = v[u];
  }
  __syncthreads();
  if (tid >= 64) return;
  if (lane >= c && lane < nb) dinv[lane] = 1.0 / ls[lane + lane * LD];
  if (lane + 64 >= c && lane + 64 < nb) dinv[lane + 64] = 1.0 / ls[lane + 64 + (lane + 64) * LD];
  chol_wave_sync();
  double b0 = lane == c ? 1.0 : 0.0, b1 = lane + 64 == c ? 1.0 : 0.0;
  for (int k = c; k < nb; ++k) {
    const double yk = (k < 64 ? readlane_f64(b0, k) : readlane_f64(b1, k - 64)) * dinv[k];
    if (lane == (k & 63)) {
      if (k < 64)
        b0 = yk;
      else
        b1 = yk;
    }
    if (lane > k && lane < nb) b0 = __builtin_fma(-ls[lane + k * LD], yk, b0);
    if (lane + 64 > k && lane + 64 < nb) b1 = __builtin_fma(-ls[lane + 64 + k * LD], yk, b1);
  }
  const double y0 = (lane >= c && lane < nb) ? b0 : 0.0;
  const double y1 = (lane + 64 >= c && lane + 64 < nb) ? b1 : 0.0;
  Y[lane + c * CHOL_NB] = y0;
  Y[lane + 64 + c * CHOL_NB] = y1;
  YT[c + lane * CHOL_NB] = y0;
  YT[c + (lane + 64) * CHOL_NB] = y1;
}

size_t chol_diag_lds_bytes() { return sizeof(double) * (CHOL_NB * (CHOL_NB + 1) + CHOL_NB); }

hipError_t launch_chol_diag(double *A, int64_t lda, int nb, int j0, int *info, double *Y, double *YT,
                            hipStream_t st) {
  if (nb <= 0 || nb > CHOL_NB) return hipErrorInvalidValue;
  hipLaunchKernelGGL(chol_diag_kernel, dim3(1), dim3(1024), 0, st, A, lda, nb, j0, info);
  const size_t lds = chol_diag_lds_bytes();
  hipLaunchKernelGGL(chol_inv_kernel, dim3(CHOL_NB), dim3(1024), lds, st, (const double *)A, lda, nb,
                     (const int *)info, Y, YT);
  return hipGetLastError();
}

// One block step of the substitution sweeps of chol_solve, for the factor L (column-major,
// ld n) and the block's inverse M (Y for the forward sweep, Y^T for the backward one;
// nb x nb, ld CHOL_NB): x = M src[j0 : j0+jb] (every workgroup, from L2), workgroup 0 stores
// x at dst[j0 : j0+jb], and each workgroup subtracts the block's contribution from 128 rows
// of src: forward  src[r] -= sum_c L[r, j0+c] x_c for r >= j0 + jb (lanes down a column,
// coalesced; eight thread groups split c); backward src[r] -= sum_c L[j0+c, r] x_c for
// r < j0 (8 lanes a row, 16 contiguous c each).  Every load of a phase is issued before its
// first use: the kernel is latency-bound (~9 MB of L at n = 9000).  src[j0 : j0+jb] is only
// read here and dst is another vector: no workgroup waits on another.
__global__ __launch_bounds__(1024) void tri_sweep_kernel(const double *__restrict__ L, int64_t n,
                                                         const double *__restrict__ M, int64_t j0, int jb,
                                                         int back, double *__restrict__ src,
                                                         double *__restrict__ dst) {
  __shared__ double bs[CHOL_NB], xs[CHOL_NB], ps[8][CHOL_NB];
  const int tid = threadIdx.x;
  // this workgroup's share of L first: it does not depend on x, so its latency overlaps
  // the x = M b phase.  Forward: thread (row rl, octant cq) holds L[r, j0 + 16 cq ..];
  // backward: 8 lanes a row, lane (lane & 7) holds L[j0 + 16 (lane & 7) .., r].
  double v[16];
  const int rl = tid & (CHOL_SWEEP_ROWS - 1), cq = tid / CHOL_SWEEP_ROWS;
  const int lane = tid & 63, seg = (lane & 7) * 16;
  const int64_t rf = j0 + jb + (int64_t)blockIdx.x * CHOL_SWEEP_ROWS + rl;
  const int64_t rb = (int64_t)blockIdx.x * CHOL_SWEEP_ROWS + (tid >> 3);
  if (!back) {
    const double *col = L + min(rf, n - 1) + j0 * n;
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = col[(int64_t)min(cq * 16 + u, jb - 1) * n];
  } else {
    const double *row = L + j0 + (j0 > 0 ? min(rb, j0 - 1) : 0) * n;  // L[j0 + c, r]
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = row[min(seg + u, jb - 1)];
  }
  if (tid < CHOL_NB) bs[tid] = tid < jb ? src[j0 + tid] : 0.0;
  __syncthreads();
  {
    const int i = tid & (CHOL_NB - 1), q = tid >> 7;
    double m[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) m[u] = M[i + (q * 16 + u) * CHOL_NB];  // zero past jb
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += m[u] * bs[q * 16 + u];
    ps[q][i] = acc;
  }
  __syncthreads();
  if (tid < CHOL_NB) {
    double x = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) x += ps[q][tid];
    xs[tid] = x;  // zero past jb (M is)
    if (blockIdx.x == 0 && tid < jb) dst[j0 + tid] = x;
  }
  __syncthreads();
  if (!back) {
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += v[u] * xs[cq * 16 + u];  // xs[c >= jb] = 0
    ps[cq][rl] = acc;  // (ps reused: every read of it is behind the barrier above)
    __syncthreads();
    if (tid < CHOL_SWEEP_ROWS && rf < n) {
      double t = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) t += ps[q][tid];
      src[rf] -= t;
    }
  } else {
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < 16; ++u) acc += v[u] * xs[seg + u];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    acc += __shfl_xor(acc, 4);
    if (rb < j0 && (lane & 7) == 0) src[rb] -= acc;
  }
}

hipError_t launch_tri_sweep(const double *L, int64_t n, const double *M, int64_t j0, int jb, int back,
                            double *src, double *dst, hipStream_t st) {
  if (jb <= 0 || jb > CHOL_NB || j0 < 0 || j0 + jb > n) return hipErrorInvalidValue;
  const int64_t rows = back ? j0 : n - j0 - jb;
  const int64_t g = std::max<int64_t>(1, (rows + CHOL_SWEEP_ROWS - 1) / CHOL_SWEEP_ROWS);
  hipLaunchKernelGGL(tri_sweep_kernel, dim3((unsigned)g), dim3(1024), 0, st, L, n, M, j0, jb, back, src, dst);
  return hipGetLastError();
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
