// kmg_combine.hip — the kernel-combination consumers of the Gram matrices on gfx950.
//
// The reference combines several Grams on the host, with numpy temporaries of p*n*n:
//   NLCK.svm_step / get_K (NLCKernels.py:52, 97):  K = (sum_m u_m K_m) ** degree
//   NLCK.grad            (NLCKernels.py:61-66):   grad_m = -d * alpha^T (K_t o K_m) alpha,
//                                                 K_t = (sum_m u_m K_m) ** (d - 1)
//   ALIGNF.get_a / get_M (ALIGNF.py:43-58) on center_K(K_m) (kernels.py:387-395):
//                                                 a_m = <Kc_m, y y^T>_F, M_lm = <Kc_l, Kc_m>_F
// Each of these is one streaming pass over the p matrices (HBM-bound: 8 p n^2 bytes read),
// so each is one fused kernel here.  The p matrices are a device array of p row-major
// float64 pointers with a common leading dimension.  Reductions are two-stage (per-row
// partials, then a fixed-order sum), so results are run-to-run reproducible.
#include "kmg_internal.h"

namespace kmg {

constexpr int CMB_THREADS = 256;

// x ** d as numpy evaluates `float64_array ** int`: d = 1 -> x, d = 2 -> x * x (the
// np.square fast path); other d -> pow(x, d).
__device__ __forceinline__ double int_pow(double x, int d) {
  if (d == 1) return x;
  if (d == 2) return __dmul_rn(x, x);
  if (d == 0) return 1.0;
  return pow(x, (double)d);
}

// sum_m K_m[off] * u_m, accumulated slice after slice (np.sum over axis 0 of the
// p x n x n product array adds the slices in order)
__device__ __forceinline__ double weighted_sum(const double *const *K, const double *u, int p,
                                               int64_t off) {
  double s = __dmul_rn(K[0][off], u[0]);
  for (int m = 1; m < p; ++m) s = __dadd_rn(s, __dmul_rn(K[m][off], u[m]));
  return s;
}

__global__ __launch_bounds__(CMB_THREADS) void combine_kernel(const double *const *__restrict__ K,
                                                              const double *__restrict__ u, int p,
                                                              int degree, int64_t n, int64_t ld,
                                                              double *__restrict__ out,
                                                              int64_t ld_out) {
  const int64_t i = blockIdx.y;
  for (int64_t j = (int64_t)blockIdx.x * CMB_THREADS + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * CMB_THREADS)
    __builtin_nontemporal_store(int_pow(weighted_sum(K, u, p, i * ld + j), degree),
                                out + i * ld_out + j);
}

// per row i: part[i * p + m] = sum_j (K_t[i][j] * alpha_j) * K_m[i][j]
template <int PMAX>
__global__ __launch_bounds__(CMB_THREADS) void nlck_grad_rows_kernel(
    const double *const *__restrict__ K, const double *__restrict__ u, int p, int degree,
    const double *__restrict__ alpha, int64_t n, int64_t ld, double *__restrict__ part) {
  __shared__ double red[CMB_THREADS / 64][PMAX];
  const int64_t i = blockIdx.x;
  double acc[PMAX];
#pragma unroll
  for (int m = 0; m < PMAX; ++m) acc[m] = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += CMB_THREADS) {
    const int64_t off = i * ld + j;
    const double a = __dmul_rn(int_pow(weighted_sum(K, u, p, off), degree - 1), alpha[j]);
#pragma unroll
    for (int m = 0; m < PMAX; ++m)
      if (m < p) acc[m] = __dadd_rn(acc[m], __dmul_rn(a, K[m][off]));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int m = 0; m < PMAX; ++m) {
    double v = acc[m];
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0) red[wave][m] = v;
  }
  __syncthreads();
  if ((int)threadIdx.x < p) {
    double v = 0.0;
    for (int w = 0; w < CMB_THREADS / 64; ++w) v += red[w][threadIdx.x];
    part[i * p + threadIdx.x] = v;
  }
}

// out[m] = scale * sum_i w_i * part[i * stride + m] (w = nullptr: 1), one block, fixed order
__global__ __launch_bounds__(CMB_THREADS) void weighted_colsum_kernel(const double *__restrict__ part,
                                                                      const double *__restrict__ w,
                                                                      int64_t rows, int cols,
                                                                      double scale,
                                                                      double *__restrict__ out) {
  __shared__ double red[CMB_THREADS];
  for (int m = 0; m < cols; ++m) {
    double v = 0.0;
    for (int64_t i = threadIdx.x; i < rows; i += CMB_THREADS)
      v += (w ? w[i] : 1.0) * part[i * cols + m];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = CMB_THREADS / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[m] = scale * red[0];
    __syncthreads();
  }
}

// row means of every K_m: rmean[m * n + i]
__global__ __launch_bounds__(CMB_THREADS) void row_means_kernel(const double *const *__restrict__ K,
                                                                int64_t n, int64_t ld,
                                                                double *__restrict__ rmean) {
  __shared__ double red[CMB_THREADS / 64];
  const int64_t i = blockIdx.x;
  const int m = blockIdx.y;
  double v = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += CMB_THREADS) v += K[m][i * ld + j];
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < CMB_THREADS / 64; ++w) s += red[w];
    rmean[(int64_t)m * n + i] = s / (double)n;
  }
}

// column means: thread = one column of one matrix, sweeping the rows (coalesced per row)
__global__ __launch_bounds__(CMB_THREADS) void col_means_kernel(const double *const *__restrict__ K,
                                                                int64_t n, int64_t ld,
                                                                double *__restrict__ cmean) {
  const int m = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * CMB_THREADS + threadIdx.x;
  if (j >= n) return;
  double v = 0.0;
  for (int64_t i = 0; i < n; ++i) v += K[m][i * ld + j];
  cmean[(int64_t)m * n + j] = v / (double)n;
}

// total means: tmean[m] = mean of rmean[m][.]
__global__ __launch_bounds__(CMB_THREADS) void total_means_kernel(const double *__restrict__ rmean,
                                                                  int p, int64_t n,
                                                                  double *__restrict__ tmean) {
  __shared__ double red[CMB_THREADS];
  for (int m = 0; m < p; ++m) {
    double v = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += CMB_THREADS) v += rmean[(int64_t)m * n + i];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int s = CMB_THREADS / 2; s > 0; s >>= 1) {
      if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) tmean[m] = red[0] / (double)n;
    __syncthreads();
  }
}

// Per row i of the centred matrices Kc_m = K_m - r_m 1^T - 1 c_m^T + t_m (the value of
// center_K, kernels.py:387-395, without the O(n^3) product):
//   part[i][m]               = y_i * sum_j Kc_m[i][j] y_j           (-> a_m)
//   part[i][p + pair(l, m)]  = sum_j Kc_l[i][j] Kc_m[i][j], l <= m    (-> M_lm)
template <int PMAX>
__global__ __launch_bounds__(CMB_THREADS) void alignf_rows_kernel(
    const double *const *__restrict__ K, int p, const double *__restrict__ y, int64_t n,
    int64_t ld, const double *__restrict__ rmean, const double *__restrict__ cmean,
    const double *__restrict__ tmean, double *__restrict__ part) {
  constexpr int NPAIR = PMAX * (PMAX + 1) / 2;
  __shared__ double red[CMB_THREADS / 64][PMAX + NPAIR];
  const int64_t i = blockIdx.x;
  const int stride = p + p * (p + 1) / 2;
  double sa[PMAX], sm[NPAIR], ri[PMAX];
#pragma unroll
  for (int m = 0; m < PMAX; ++m) {
    sa[m] = 0.0;
    ri[m] = m < p ? rmean[(int64_t)m * n + i] - tmean[m] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < NPAIR; ++q) sm[q] = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += CMB_THREADS) {
    double kc[PMAX];
    const double yj = y[j];
#pragma unroll
    for (int m = 0; m < PMAX; ++m) {
      kc[m] = m < p ? (K[m][i * ld + j] - ri[m]) - cmean[(int64_t)m * n + j] : 0.0;
      sa[m] += kc[m] * yj;
    }
    int q = 0;
#pragma unroll
    for (int l = 0; l < PMAX; ++l)
#pragma unroll
      for (int m = l; m < PMAX; ++m) sm[q++] += kc[l] * kc[m];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < PMAX + NPAIR; ++q) {
    double v = q < PMAX ? sa[q] : sm[q - PMAX];
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == 0) red[wave][q] = v;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < stride; q += CMB_THREADS) {
    int src;  // compact (p) layout -> PMAX-sized accumulators
    if (q < p) {
      src = q;
    } else {
      int t = q - p, l = 0;
      while (t >= p - l) {
        t -= p - l;
        ++l;
      }
      src = PMAX + l * PMAX - l * (l - 1) / 2 + t;
    }
    double v = 0.0;
    for (int w = 0; w < CMB_THREADS / 64; ++w) v += red[w][src];
    part[i * stride + q] = q < p ? v * y[i] : v;
  }
}

// ------------------------------------------------------------------ launchers
hipError_t launch_combine(const double *const *K, const double *u, int p, int degree, int64_t n,
                          int64_t ld, double *out, int64_t ld_out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const unsigned gx = (unsigned)std::min<int64_t>((n + CMB_THREADS - 1) / CMB_THREADS, 16);
  hipLaunchKernelGGL(combine_kernel, dim3(gx, (unsigned)n), dim3(CMB_THREADS), 0, s, K, u, p,
                     degree, n, ld, out, ld_out);
  return hipGetLastError();
}

#define KMG_PMAX_DISPATCH(P_, KERNEL, ...)                                      \
  if ((P_) <= 4) {                                                              \
    hipLaunchKernelGGL((KERNEL<4>), __VA_ARGS__);                               \
  } else if ((P_) <= 8) {                                                       \
    hipLaunchKernelGGL((KERNEL<8>), __VA_ARGS__);                               \
  } else if ((P_) <= KMG_COMBINE_PMAX) {                                        \
    hipLaunchKernelGGL((KERNEL<KMG_COMBINE_PMAX>), __VA_ARGS__);                \
  } else {                                                                      \
    return hipErrorInvalidValue;                                                \
  }

hipError_t launch_nlck_grad(const double *const *K, const double *u, int p, int degree,
                            const double *alpha, int64_t n, int64_t ld, double *part,
                            double *grad, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  KMG_PMAX_DISPATCH(p, nlck_grad_rows_kernel, dim3((unsigned)n), dim3(CMB_THREADS), 0, s, K, u, p,
                    degree, alpha, n, ld, part)
  hipLaunchKernelGGL(weighted_colsum_kernel, dim3(1), dim3(CMB_THREADS), 0, s, part, alpha, n, p,
                     -(double)degree, grad);
  return hipGetLastError();
}

hipError_t launch_alignf(const double *const *K, int p, const double *y, int64_t n, int64_t ld,
                         double *rmean, double *cmean, double *tmean, double *part, double *out,
                         hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(row_means_kernel, dim3((unsigned)n, (unsigned)p), dim3(CMB_THREADS), 0, s, K,
                     n, ld, rmean);
  hipLaunchKernelGGL(col_means_kernel,
                     dim3((unsigned)((n + CMB_THREADS - 1) / CMB_THREADS), (unsigned)p),
                     dim3(CMB_THREADS), 0, s, K, n, ld, cmean);
  hipLaunchKernelGGL(total_means_kernel, dim3(1), dim3(CMB_THREADS), 0, s, rmean, p, n, tmean);
  KMG_PMAX_DISPATCH(p, alignf_rows_kernel, dim3((unsigned)n), dim3(CMB_THREADS), 0, s, K, p, y, n,
                    ld, rmean, cmean, tmean, part)
  hipLaunchKernelGGL(weighted_colsum_kernel, dim3(1), dim3(CMB_THREADS), 0, s, part,
                     (const double *)nullptr, n, p + p * (p + 1) / 2, 1.0, out);
  return hipGetLastError();
}

#undef KMG_PMAX_DISPATCH

}  // namespace kmg
