// kmg_gram.hip — spectrum and mismatch Gram kernels for gfx950.
//
// Reference hot loops replaced (afiliot/Kernel-Methods-For-Genomics kernels.py):
//   get_spectrum_K pair loop (kernels.py:41-45): K[i,j] = np.dot(phi_u[i], phi_u[j])
//   get_mismatch_K pair loop (kernels.py:211-215) + normalize_K (kernels.py:398-415)
//
// Formulation ("row accumulator over postings", Gustavson SpGEMM with a dense LDS
// accumulator): one workgroup owns (row i, column chunk c).  For every k-mer of
// sequence i it walks the posting list of that k-mer restricted to chunk c and adds
// into acc[column] in LDS.  When done, the LDS row is converted and streamed to HBM
// with 16-byte stores.  Integer work only until the (optional) float64 epilogue, so
// spectrum and raw mismatch counts are exact; the normalise epilogue reproduces
// normalize_K's fp64 expression K_ij / (sqrt(K_ii) * sqrt(K_jj)).
//
// Mismatch (m=1) uses the closed form K(x,y) = sum_{a,b} w[ham(x_a, y_b)],
// w = (1+3k, 4, 2, 0, ...)  (= <Phi_x, Phi_y> of kernels.py:161-175) and
// enumerates the Hamming<=2 neighbourhood through the "drop one letter" index
// (kmg_index.hip): list (p, key_p(z)) holds every occurrence that equals z outside
// position p, tagged with its letter at p.
#include "kmg_internal.h"

namespace kmg {

__device__ __forceinline__ uint32_t letter_at_g(uint32_t code, int p, int k) {
  return (code >> (2 * (k - 1 - p))) & 3u;
}
__device__ __forceinline__ uint32_t drop_letter_g(uint32_t code, int p, int k) {
  const uint64_t c = code;
  const int lo_bits = 2 * (k - 1 - p);
  return (uint32_t)(((c >> (lo_bits + 2)) << lo_bits) | (c & ((1ull << lo_bits) - 1ull)));
}

// ------------------------------------------------------------------ epilogue
template <int DT>
__device__ __forceinline__ void emit4(const OutSpec &o, int64_t il, int64_t ig, int64_t col,
                                      int cnt, int64_t v0, int64_t v1, int64_t v2, int64_t v3,
                                      bool norm) {
  const int64_t v[4] = {v0, v1, v2, v3};
  if constexpr (DT == KMG_I32) {
    int32_t *p = (int32_t *)o.out + il * o.ld + col;
    if (cnt == 4 && ((uintptr_t)p & 15) == 0) {
      *(int4 *)p = make_int4((int)v0, (int)v1, (int)v2, (int)v3);
    } else {
      for (int q = 0; q < cnt; ++q) p[q] = (int32_t)v[q];
    }
  } else {
    double r[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q < cnt) {
        if (norm) {
          // normalize_K: K[i,j] /= (d * diag[j]) with d = sqrt(K[i,i]); diagonal := 1
          r[q] = (ig == col + q) ? 1.0 : (double)v[q] / (o.dsq[ig] * o.dsq[col + q]);
        } else {
          r[q] = (double)v[q];
        }
      } else {
        r[q] = 0.0;
      }
    }
    if constexpr (DT == KMG_F64) {
      double *p = (double *)o.out + il * o.ld + col;
      if (cnt == 4 && ((uintptr_t)p & 15) == 0) {
        *(double2 *)p = make_double2(r[0], r[1]);
        *(double2 *)(p + 2) = make_double2(r[2], r[3]);
      } else {
        for (int q = 0; q < cnt; ++q) p[q] = r[q];
      }
    } else {
      float *p = (float *)o.out + il * o.ld + col;
      if (cnt == 4 && ((uintptr_t)p & 15) == 0) {
        *(float4 *)p = make_float4((float)r[0], (float)r[1], (float)r[2], (float)r[3]);
      } else {
        for (int q = 0; q < cnt; ++q) p[q] = (float)r[q];
      }
    }
  }
}

// ------------------------------------------------------------------ spectrum
// PACK16: two 16-bit counters per LDS word (valid when every K_ij <= 65535, i.e.
// P_i * P_j <= 65535; the host checks P_max <= 255).
template <bool PACK16, int DT>
__global__ __launch_bounds__(256) void gram_sp_kernel(IndexGeom g, const uint32_t *__restrict__ kmers,
                                                      const uint32_t *__restrict__ off,
                                                      const uint32_t *__restrict__ ent,
                                                      int64_t row0, OutSpec o) {
  extern __shared__ __align__(16) uint32_t acc[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int words = PACK16 ? (((cw + 7) >> 3) << 2) : (((cw + 3) >> 2) << 2);
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (words >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  __syncthreads();

  const uint32_t *__restrict__ o_c = off + (size_t)c * g.nkeys;
  const uint32_t *__restrict__ row = kmers + (size_t)i * g.pmax;
  for (int a = threadIdx.x; a < g.pmax; a += blockDim.x) {
    const uint32_t u = row[a];
    if (u == KMG_INVALID) continue;
    const uint32_t beg = o_c[u], end = o_c[u + 1];
    uint32_t e = beg;
    for (; e + 4 <= end; e += 4) {
      const uint32_t j0 = ent[e], j1 = ent[e + 1], j2 = ent[e + 2], j3 = ent[e + 3];
      if (PACK16) {
        atomicAdd(&acc[j0 >> 1], 1u << ((j0 & 1) << 4));
        atomicAdd(&acc[j1 >> 1], 1u << ((j1 & 1) << 4));
        atomicAdd(&acc[j2 >> 1], 1u << ((j2 & 1) << 4));
        atomicAdd(&acc[j3 >> 1], 1u << ((j3 & 1) << 4));
      } else {
        atomicAdd(&acc[j0], 1u);
        atomicAdd(&acc[j1], 1u);
        atomicAdd(&acc[j2], 1u);
        atomicAdd(&acc[j3], 1u);
      }
    }
    for (; e < end; ++e) {
      const uint32_t j0 = ent[e];
      if (PACK16)
        atomicAdd(&acc[j0 >> 1], 1u << ((j0 & 1) << 4));
      else
        atomicAdd(&acc[j0], 1u);
    }
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int q = threadIdx.x * 4; q < cw; q += blockDim.x * 4) {
    uint32_t v0, v1, v2, v3;
    if (PACK16) {
      const uint2 w = *(const uint2 *)&acc[q >> 1];
      v0 = w.x & 0xFFFFu; v1 = w.x >> 16; v2 = w.y & 0xFFFFu; v3 = w.y >> 16;
    } else {
      const uint4 w = *(const uint4 *)&acc[q];
      v0 = w.x; v1 = w.y; v2 = w.z; v3 = w.w;
    }
    emit4<DT>(o, il, i, col0 + q, min(4, cw - q), v0, v1, v2, v3, norm);
  }
}

// ------------------------------------------------------------------ mismatch m=1
struct MMSub {
  int8_t p, q, ci, pad;
};
__constant__ MMSub c_mmsub[16 + 3 * 120];

// G lanes cooperate on one posting list.
template <int G, int DT>
__global__ __launch_bounds__(256) void gram_mm1_kernel(IndexGeom g, int nsub,
                                                       const uint32_t *__restrict__ kmers,
                                                       const uint32_t *__restrict__ off,
                                                       const uint32_t *__restrict__ ent,
                                                       int64_t row0, int w0, int w1, int w2,
                                                       OutSpec o) {
  extern __shared__ __align__(16) uint32_t smem[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int words = ((cw + 3) >> 2) << 2;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rowk = smem + (((g.chunk + 3) >> 2) << 2);
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (words >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  for (int a = threadIdx.x; a < g.pmax; a += blockDim.x) rowk[a] = kmers[(size_t)i * g.pmax + a];
  __syncthreads();

  const int k = g.k;
  const int grp = threadIdx.x / G, gl = threadIdx.x % G, ngrp = blockDim.x / G;
  const int total = g.pmax * nsub;
  for (int L = grp; L < total; L += ngrp) {
    const int a = L / nsub;
    const int s = L - a * nsub;
    const uint32_t u = rowk[a];
    if (u == KMG_INVALID) continue;
    const MMSub sb = c_mmsub[s];
    const int p = sb.p;
    uint32_t z = u;
    int wa, wb;
    if (sb.q < 0) {
      // neighbours differing from u at most at p: ham 0 (counted once, on p==0) or 1
      wa = (p == 0) ? w0 : 0;
      wb = w1;
    } else {
      // neighbours differing exactly at {q, p}, q < p: substitute letter q, scan list p
      const int sh = 2 * (k - 1 - sb.q);
      const uint32_t lq = (u >> sh) & 3u;
      const uint32_t nl = (lq + 1u + (uint32_t)sb.ci) & 3u;
      z = (u & ~(3u << sh)) | (nl << sh);
      wa = 0;
      wb = w2;
    }
    const uint32_t up = letter_at_g(u, p, k);
    const size_t bin = ((size_t)p * g.nchunks + c) * g.nkeys + drop_letter_g(z, p, k);
    const uint32_t beg = off[bin], end = off[bin + 1];
    for (uint32_t e = beg + gl; e < end; e += G) {
      const uint32_t v = ent[e];
      const int w = ((v >> KMG_ENTRY_LETTER_SHIFT) == up) ? wa : wb;
      if (w) atomicAdd(&acc[v & KMG_ENTRY_SEQ_MASK], w);
    }
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int q = threadIdx.x * 4; q < cw; q += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[q];
    emit4<DT>(o, il, i, col0 + q, min(4, cw - q), w.x, w.y, w.z, w.w, norm);
  }
}

// ------------------------------------------------------------------ Hamming forms
__device__ __forceinline__ int ham2bit(uint32_t a, uint32_t b, uint32_t mask55) {
  const uint32_t x = a ^ b;
  return __popc((x | (x >> 1)) & mask55);
}

// one 256-thread block = row i x 64 columns; each wave owns 16 columns
template <int DT>
__global__ __launch_bounds__(256) void gram_ham_kernel(IndexGeom g, const uint32_t *__restrict__ kmers,
                                                       int64_t row0, const int64_t *__restrict__ wtab,
                                                       OutSpec o) {
  __shared__ int64_t w_s[33];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t il = blockIdx.y;
  const int64_t i = row0 + il;
  if (threadIdx.x <= g.k) w_s[threadIdx.x] = wtab[threadIdx.x];
  __syncthreads();
  const uint32_t mask55 = (g.k >= 16) ? 0x55555555u : (0x55555555u & ((1u << (2 * g.k)) - 1u));
  uint32_t xa[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int a = lane + 64 * q;
    xa[q] = (a < g.pmax) ? kmers[(size_t)i * g.pmax + a] : KMG_INVALID;
  }
  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int jj = 0; jj < 16; ++jj) {
    const int64_t j = (int64_t)blockIdx.x * 64 + wave * 16 + jj;
    if (j >= g.n) break;
    int64_t s = 0;
    const uint32_t *yc = kmers + (size_t)j * g.pmax;
    for (int b = 0; b < g.pmax; ++b) {
      const uint32_t yb = yc[b];
      if (yb == KMG_INVALID) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (xa[q] != KMG_INVALID) s += w_s[ham2bit(xa[q], yb, mask55)];
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
    if (lane == 0) emit4<DT>(o, il, i, j, 1, s, 0, 0, 0, norm);
  }
}

// raw self-kernel K_ii for every sequence (diagonal used by normalize_K)
__global__ __launch_bounds__(64) void diag_ham_kernel(IndexGeom g, const uint32_t *__restrict__ kmers,
                                                      const int64_t *__restrict__ wtab,
                                                      double *__restrict__ diagv,
                                                      double *__restrict__ dsq) {
  __shared__ int64_t w_s[33];
  const int lane = threadIdx.x;
  const int64_t i = blockIdx.x;
  if (lane <= g.k) w_s[lane] = wtab[lane];
  __syncthreads();
  const uint32_t mask55 = (g.k >= 16) ? 0x55555555u : (0x55555555u & ((1u << (2 * g.k)) - 1u));
  const uint32_t *xc = kmers + (size_t)i * g.pmax;
  int64_t s = 0;
  for (int a = lane; a < g.pmax; a += 64) {
    const uint32_t xa = xc[a];
    if (xa == KMG_INVALID) continue;
    for (int b = 0; b < g.pmax; ++b) {
      const uint32_t yb = xc[b];
      if (yb != KMG_INVALID) s += w_s[ham2bit(xa, yb, mask55)];
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if (lane == 0) {
    const double v = (double)s;
    diagv[i] = v;
    dsq[i] = __builtin_sqrt(v);  // np.sqrt(np.diag(K)) (kernels.py:408): IEEE sqrt
  }
}

// ------------------------------------------------------------------ launchers
#define KMG_DISPATCH_DT(DT, ...)                       \
  switch (DT) {                                        \
    case KMG_I32: { constexpr int D = KMG_I32; __VA_ARGS__; } break; \
    case KMG_F32: { constexpr int D = KMG_F32; __VA_ARGS__; } break; \
    default: { constexpr int D = KMG_F64; __VA_ARGS__; } break;      \
  }

hipError_t launch_gram_spectrum(const IndexGeom &g, const uint32_t *kmers, const uint32_t *off,
                                const uint32_t *ent, int64_t row0, int64_t row1,
                                const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  const bool pack = g.pmax <= 255;
  const int words = pack ? (((g.chunk + 7) >> 3) << 2) : (((g.chunk + 3) >> 2) << 2);
  const size_t lds = (size_t)words * 4;
  const dim3 grid((unsigned)(rows * g.nchunks));
  if (pack) {
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<true, D>), grid, dim3(256), lds, s,
                                                g, kmers, off, ent, row0, o));
  } else {
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<false, D>), grid, dim3(256), lds, s,
                                                g, kmers, off, ent, row0, o));
  }
  return hipGetLastError();
}

static int g_mm_nsub_k = -1;
static int g_mm_nsub = 0;

static hipError_t upload_mmsub(int k, hipStream_t s) {
  if (g_mm_nsub_k == k) return hipSuccess;
  MMSub tab[16 + 3 * 120];
  int n = 0;
  for (int p = 0; p < k; ++p) tab[n++] = MMSub{(int8_t)p, (int8_t)-1, 0, 0};
  for (int p = 1; p < k; ++p)
    for (int q = 0; q < p; ++q)
      for (int ci = 0; ci < 3; ++ci) tab[n++] = MMSub{(int8_t)p, (int8_t)q, (int8_t)ci, 0};
  hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_mmsub), tab, sizeof(MMSub) * n, 0,
                                        hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return e;
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  g_mm_nsub_k = k;
  g_mm_nsub = n;
  return hipSuccess;
}

static int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

hipError_t launch_gram_mismatch1(const IndexGeom &g, const uint32_t *kmers, const uint32_t *off,
                                 const uint32_t *ent, int64_t row0, int64_t row1, int w0, int w1,
                                 int w2, const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  hipError_t e = upload_mmsub(g.k, s);
  if (e != hipSuccess) return e;
  const size_t lds = (size_t)((((g.chunk + 3) >> 2) << 2) + g.pmax) * 4;
  const dim3 grid((unsigned)(rows * g.nchunks));
  // lanes per posting list ~ half the expected list length (chunk * P / 4^(k-1))
  const double avg = (double)g.chunk * g.pmax / (double)g.nkeys;
  int G = 1;
  while (G < 64 && G * 2 <= avg / 2) G *= 2;
  G = env_int("KMG_MM_G", G);
  const int nsub = g_mm_nsub;
#define KMG_MM_CASE(GG)                                                                          \
  case GG:                                                                                       \
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_mm1_kernel<GG, D>), grid, dim3(256), lds, \
                                                s, g, nsub, kmers, off, ent, row0, w0, w1, w2, o)); \
    break;
  switch (G) {
    KMG_MM_CASE(1)
    KMG_MM_CASE(2)
    KMG_MM_CASE(4)
    KMG_MM_CASE(8)
    KMG_MM_CASE(16)
    KMG_MM_CASE(32)
    default:
      KMG_MM_CASE(64)
  }
#undef KMG_MM_CASE
  return hipGetLastError();
}

hipError_t launch_gram_hamming(const IndexGeom &g, const uint32_t *kmers, int64_t row0,
                               int64_t row1, const int64_t *wtab, const OutSpec &o,
                               hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  const dim3 grid((unsigned)((g.n + 63) / 64), (unsigned)rows);
  KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_ham_kernel<D>), grid, dim3(256), 0, s, g,
                                              kmers, row0, wtab, o));
  return hipGetLastError();
}

hipError_t launch_diag_hamming(const IndexGeom &g, const uint32_t *kmers, const int64_t *wtab,
                               double *diagv, double *dsq, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  hipLaunchKernelGGL(diag_ham_kernel, dim3((unsigned)g.n), dim3(64), 0, s, g, kmers, wtab, diagv,
                     dsq);
  return hipGetLastError();
}

}  // namespace kmg
