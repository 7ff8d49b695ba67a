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
template <int DT, bool NT = false>
__device__ __forceinline__ void emit4(const OutSpec &o, int64_t il, int64_t ig, int64_t col,
                                      int cnt, int64_t v0, int64_t v1, int64_t v2, int64_t v3,
                                      bool norm) {
  const int64_t v[4] = {v0, v1, v2, v3};
  if constexpr (DT == KMG_I32) {
    int32_t *p = (int32_t *)o.out + il * o.ld + col;
    if (cnt == 4 && ((uintptr_t)p & 15) == 0) {
      typedef int v4i __attribute__((ext_vector_type(4)));
      const v4i x = {(int)v0, (int)v1, (int)v2, (int)v3};
      if constexpr (NT)
        __builtin_nontemporal_store(x, (v4i *)p);
      else
        *(v4i *)p = x;
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
        if constexpr (NT) {
          typedef double v2d __attribute__((ext_vector_type(2)));
          const v2d a = {r[0], r[1]}, b = {r[2], r[3]};
          __builtin_nontemporal_store(a, (v2d *)p);
          __builtin_nontemporal_store(b, (v2d *)(p + 2));
        } else {
          *(double2 *)p = make_double2(r[0], r[1]);
          *(double2 *)(p + 2) = make_double2(r[2], r[3]);
        }
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

// row k-mer code of window a of a staged row (KMG_INVALID if it holds a non-ACGT symbol)
__device__ __forceinline__ uint32_t window_code(const uint8_t *rs, int a, int k) {
  uint32_t c = 0, bad = 0;
  for (int q = 0; q < k; ++q) {
    const uint32_t v = rs[a + q];
    bad |= v & ~3u;
    c = (c << 2) | (v & 3u);
  }
  return bad ? KMG_INVALID : c;
}

// ------------------------------------------------------------------ spectrum
// PACK16: two 16-bit counters per LDS word (valid when every K_ij <= 65535, i.e.
// P_i * P_j <= 65535; the host checks P_max <= 255).
// G lanes walk one posting list (G * windows ~ the block): each lane issues U entry
// loads per round before its atomics, so a list of ~30 entries (k=8, N=20000) costs one
// memory round trip instead of four.
template <bool PACK16, int DT, bool NT, int G = 1>
__global__ __launch_bounds__(256) void gram_sp_kernel(IndexGeom g, const uint8_t *__restrict__ codes,
                                                      const int32_t *__restrict__ lens, int64_t ldc,
                                                      const uint32_t *__restrict__ off,
                                                      const uint16_t *__restrict__ ent,
                                                      int64_t row0, OutSpec o, int64_t nitems) {
  extern __shared__ __align__(16) uint32_t acc[];
  // nitems > gridDim.x: persistent blocks walk (row, chunk) items, so the row stores of
  // one item drain while the block already accumulates the next
  for (int64_t item = blockIdx.x; item < nitems; item += gridDim.x) {
  const int64_t il = item / g.nchunks;
  const int64_t i = row0 + il;
  const int c = (int)(item - il * g.nchunks);
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int words = PACK16 ? (((cw + 7) >> 3) << 2) : (((cw + 3) >> 2) << 2);
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (words >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  __syncthreads();

  const uint32_t *__restrict__ o_c = off + (size_t)c * g.nkeys;
  const int L = g.window > 0 ? g.window : lens[i];
  const uint8_t *rs = codes + i * ldc;
  auto add = [&](uint32_t j0) {
    if (PACK16)
      atomicAdd(&acc[j0 >> 1], 1u << ((j0 & 1) << 4));
    else
      atomicAdd(&acc[j0], 1u);
  };
  if constexpr (G == 1) {
    for (int a = threadIdx.x; a <= L - g.k; a += blockDim.x) {
      const uint32_t u = window_code(rs, a, g.k);
      if (u == KMG_INVALID) continue;
      const uint32_t beg = o_c[u], end = o_c[u + 1];
      uint32_t e = beg;
      for (; e + 8 <= end; e += 8) {
        uint32_t j[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) j[q] = ent[e + q];
#pragma unroll
        for (int q = 0; q < 8; ++q) add(j[q]);
      }
      for (; e < end; ++e) add(ent[e]);
    }
  } else {
    constexpr int U = 16;
    const int gl = threadIdx.x % G;
    for (int a = threadIdx.x / G; a <= L - g.k; a += blockDim.x / G) {
      const uint32_t u = window_code(rs, a, g.k);
      if (u == KMG_INVALID) continue;
      const uint32_t beg = o_c[u], end = o_c[u + 1];
      for (uint32_t e = beg + gl; e < end; e += U * G) {
        uint32_t j[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
          const uint32_t x = e + (uint32_t)(q * G);
          j[q] = x < end ? (uint32_t)ent[x] : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int q = 0; q < U; ++q)
          if (j[q] != 0xFFFFFFFFu) add(j[q]);
      }
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
    emit4<DT, NT>(o, il, i, col0 + q, min(4, cw - q), v0, v1, v2, v3, norm);
  }
  __syncthreads();  // the accumulator is re-zeroed by the next item
  }
}

// ------------------------------------------------------------------ mismatch m=1
// Sub-list s of a row k-mer u (nsub = k + 3*k*(k-1)/2 of them):
//   s <  k: list (p=s, key_p(u)): neighbours equal to u outside p -> ham 0 (counted
//           once, on p=0, weight w0) or ham 1 at p (weight w1)
//   s >= k: (p, q<p, ci): substitute letter q of u by the ci-th other letter, scan list
//           (p, key_p) keeping letters != u_p -> ham 2 exactly at {q,p} (weight w2)
// Every Hamming<=2 neighbour of u is visited exactly once with its weight.
constexpr int MM_THREADS = 512;

template <int G, int DT>
__global__ __launch_bounds__(MM_THREADS) void gram_mm1_kernel(IndexGeom g, int nsub,
                                                              const uint8_t *__restrict__ codes,
                                                              int64_t ldc,
                                                              const uint32_t *__restrict__ off,
                                                              const uint16_t *__restrict__ ent,
                                                              int64_t row0, int w0, int w1, int w2,
                                                              OutSpec o) {
  extern __shared__ __align__(16) uint32_t smem[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rowk = smem + accw;          // pmax row k-mers
  uint32_t *sub = rowk + g.pmax;         // nsub descriptors: p | q << 8 | ci << 16
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const int k = g.k;
  const uint8_t *rs = codes + i * ldc;
  for (int a = threadIdx.x; a < g.pmax; a += blockDim.x) rowk[a] = window_code(rs, a, k);
  for (int s = threadIdx.x; s < nsub; s += blockDim.x) {
    uint32_t d;
    if (s < k) {
      d = (uint32_t)s | (0xFFu << 8);
    } else {
      const int t = s - k, pi = t / 3, ci = t - 3 * pi;
      int p = 1;
      while ((p + 1) * p / 2 <= pi) ++p;  // pi = p(p-1)/2 + q
      const int q = pi - p * (p - 1) / 2;
      d = (uint32_t)p | ((uint32_t)q << 8) | ((uint32_t)ci << 16);
    }
    sub[s] = d;
  }
  __syncthreads();

  const int grp = threadIdx.x / G, gl = threadIdx.x % G, ngrp = blockDim.x / G;
  const int total = g.pmax * nsub;
  // list descriptor: bin, letter u_p, weights for (letter == u_p) / (letter != u_p)
  auto describe = [&](int L, uint32_t &bin, uint32_t &up, int &wa, int &wb) -> bool {
    const int a = L / nsub;
    const int s = L - a * nsub;
    const uint32_t u = rowk[a];
    if (u == KMG_INVALID) return false;
    const uint32_t d = sub[s];
    const int p = d & 0xFF, q = (d >> 8) & 0xFF;
    uint32_t z = u;
    if (q == 0xFF) {
      wa = (p == 0) ? w0 : 0;
      wb = w1;
    } else {
      const int sh = 2 * (k - 1 - q);
      const uint32_t lq = (u >> sh) & 3u;
      const uint32_t nl = (lq + 1u + (d >> 16)) & 3u;
      z = (u & ~(3u << sh)) | (nl << sh);
      wa = 0;
      wb = w2;
    }
    up = letter_at_g(u, p, k);
    bin = (uint32_t)(((int64_t)p * g.nchunks + c) * g.nkeys + drop_letter_g(z, p, k));
    return true;
  };

  int L = grp;
  uint32_t beg = 0, end = 0, up = 0;
  int wa = 0, wb = 0;
  if (L < total) {
    uint32_t bin;
    if (describe(L, bin, up, wa, wb)) {
      beg = off[bin];
      end = off[bin + 1];
    }
  }
  while (L < total) {
    // software pipeline: fetch the next list's bounds while this list's entries load
    const int Ln = L + ngrp;
    uint32_t nbeg = 0, nend = 0, nup = 0;
    int nwa = 0, nwb = 0;
    if (Ln < total) {
      uint32_t bin;
      if (describe(Ln, bin, nup, nwa, nwb)) {
        nbeg = off[bin];
        nend = off[bin + 1];
      }
    }
    const uint32_t e0 = beg + gl;
    uint32_t v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = (e0 + q * G < end) ? (uint32_t)ent[e0 + q * G] : 0xFFFFFFFFu;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (v[q] != 0xFFFFFFFFu) {
        const int w = ((v[q] >> 14) == up) ? wa : wb;
        if (w) atomicAdd(&acc[v[q] & 0x3FFFu], w);
      }
    }
    for (uint32_t e = e0 + 4 * G; e < end; e += G) {
      const uint32_t x = ent[e];
      const int w = ((x >> 14) == up) ? wa : wb;
      if (w) atomicAdd(&acc[x & 0x3FFFu], w);
    }
    L = Ln;
    beg = nbeg;
    end = nend;
    up = nup;
    wa = nwa;
    wb = nwb;
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int q = threadIdx.x * 4; q < cw; q += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[q];
    emit4<DT>(o, il, i, col0 + q, min(4, cw - q), w.x, w.y, w.z, w.w, norm);
  }
}

// ------------------------------------------------------------------ mismatch m=1, v2
// Same enumeration as gram_mm1_kernel, restructured for the per-list cost:
//  - K is a compile-time constant (k=4..12), so sub-list decoding is constant division;
//  - per row, the drop-one-letter base keys key_p(u_a) and letters u_p live in LDS, and a
//    type-2 list key is base XOR (letter delta << digit(q)) — no 64-bit shifting per list;
//  - each lane group owns a CONTIGUOUS range of lists (same occurrence, consecutive
//    sub-lists), decoded incrementally; the next list's bounds are prefetched while this
//    list's entries load (4 per lane, G lanes per list).
template <int K, int G>
__global__ __launch_bounds__(MM_THREADS) void gram_mm1v2_kernel(IndexGeom g,
                                                                const uint8_t *__restrict__ codes,
                                                                int64_t ldc,
                                                                const uint32_t *__restrict__ off,
                                                                const uint16_t *__restrict__ ent,
                                                                int64_t row0, int w0, int w1, int w2,
                                                                OutSpec o) {
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *basek = smem + accw;       // [P][K]: key_p(u_a) | u_p << 30
  uint32_t *rowu = basek + P * K;      // [P]: u_a
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const uint8_t *rs = codes + i * ldc;
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = window_code(rs, a, K);
    basek[t] = drop_letter_g(u, p, K) | (letter_at_g(u, p, K) << 30);
    if (p == 0) rowu[a] = u;
  }
  __syncthreads();

  const uint32_t chunk_keys = (uint32_t)c * g.nkeys;          // + p * nchunks * nkeys
  const uint32_t copy_stride = (uint32_t)g.nchunks * g.nkeys;
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int total = P * NSUB;
  const int per = (total + ngrp - 1) / ngrp;
  int L = grp * per;
  const int Lend = min(total, L + per);

  // decode (a, s) incrementally; s -> (p, q, ci) via the fixed enumeration
  int a = L / NSUB, s = L - a * NSUB;
  int p = 0, q = -1, ci = 0;
  auto set_sub = [&]() {
    if (s < K) {
      p = s; q = -1; ci = 0;
    } else {
      const int t = s - K, pi = t / 3;
      ci = t - 3 * pi;
      int pp = 1;
      while ((pp + 1) * pp / 2 <= pi) ++pp;
      p = pp;
      q = pi - pp * (pp - 1) / 2;
    }
  };
  auto describe = [&](uint32_t &bin, uint32_t &up, int &wa, int &wb) {
    const uint32_t bk = basek[a * K + p];
    up = bk >> 30;
    uint32_t key = bk & 0x3FFFFFFFu;
    if (q < 0) {
      wa = (p == 0) ? w0 : 0;
      wb = w1;
    } else {
      const uint32_t lq = (rowu[a] >> (2 * (K - 1 - q))) & 3u;
      const uint32_t nl = (lq + 1u + (uint32_t)ci) & 3u;
      key ^= (lq ^ nl) << (2 * (K - 2 - q));  // q < p: digit of q inside key_p
      wa = 0;
      wb = w2;
    }
    bin = (uint32_t)p * copy_stride + chunk_keys + key;
  };
  auto advance = [&]() {
    if (++s == NSUB) { s = 0; ++a; }
    set_sub();
  };
  set_sub();

  uint32_t beg = 0, end = 0, up = 0;
  int wa = 0, wb = 0;
  if (L < Lend) {
    uint32_t bin;
    describe(bin, up, wa, wb);
    beg = off[bin];
    end = off[bin + 1];
  }
  for (; L < Lend; ++L) {
    uint32_t nbeg = 0, nend = 0, nup = 0;
    int nwa = 0, nwb = 0;
    if (L + 1 < Lend) {
      advance();
      uint32_t bin;
      describe(bin, nup, nwa, nwb);
      nbeg = off[bin];
      nend = off[bin + 1];
    }
    const uint32_t e0 = beg + gl;
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (e0 + u * G < end) ? (uint32_t)ent[e0 + u * G] : 0xFFFFFFFFu;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (v[u] != 0xFFFFFFFFu) {
        const int w = ((v[u] >> 14) == up) ? wa : wb;
        if (w) atomicAdd(&acc[v[u] & 0x3FFFu], w);
      }
    }
    for (uint32_t e = e0 + 4 * G; e < end; e += G) {
      const uint32_t x = ent[e];
      const int w = ((x >> 14) == up) ? wa : wb;
      if (w) atomicAdd(&acc[x & 0x3FFFu], w);
    }
    beg = nbeg;
    end = nend;
    up = nup;
    wa = nwa;
    wb = nwb;
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int qq = threadIdx.x * 4; qq < cw; qq += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[qq];
    if (o.dtype == KMG_F64)
      emit4<KMG_F64>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else if (o.dtype == KMG_F32)
      emit4<KMG_F32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else
      emit4<KMG_I32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
  }
}

// ------------------------------------------------------------------ mismatch m=1, v3
// Rotated layout: copy p lists every occurrence z under rot_p(z) = key_p(z)*4 + z_p, so
// the drop-one-letter list (p, key) is the 4 adjacent bins key*4 .. key*4+3, one per
// letter at p.  A list is then 3 segments: letters below u_p (weight wb), letter u_p
// (weight wa, skipped unloaded when wa == 0) and letters above u_p (weight wb).
// Entries are plain 16-bit columns (chunks up to 65536 columns).
template <int K, int G>
__global__ __launch_bounds__(1024) void gram_mm1rot_kernel(IndexGeom g,
                                                           const uint8_t *__restrict__ codes,
                                                           int64_t ldc,
                                                           const uint32_t *__restrict__ off,
                                                           const uint16_t *__restrict__ ent,
                                                           int64_t row0, int w0, int w1, int w2,
                                                           OutSpec o) {
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rotk = smem + accw;   // [P][K]: rot_p(u_a)
  uint32_t *sub = rotk + P * K;   // [NSUB]: p | q << 8 | ci << 16 (q = 0xFF: type 1)
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const uint8_t *rs = codes + i * ldc;
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = window_code(rs, a, K);
    rotk[t] = (drop_letter_g(u, p, K) << 2) | letter_at_g(u, p, K);
  }
  for (int s = threadIdx.x; s < NSUB; s += blockDim.x) {
    uint32_t d;
    if (s < K) {
      d = (uint32_t)s | (0xFFu << 8);
    } else {
      const int t = s - K, pi = t / 3, ci = t - 3 * pi;
      int pp = 1;
      while ((pp + 1) * pp / 2 <= pi) ++pp;
      d = (uint32_t)pp | ((uint32_t)(pi - pp * (pp - 1) / 2) << 8) | ((uint32_t)ci << 16);
    }
    sub[s] = d;
  }
  __syncthreads();

  const uint32_t chunk_bins = (uint32_t)c * g.nkeys;
  const uint32_t copy_stride = (uint32_t)g.nchunks * g.nkeys;
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int total = P * NSUB;
  // groups of a wave take consecutive sub-lists of the same k-mer (strided over the
  // row's list space): their bins are close in memory (shared cache lines)
  int L = grp;
  const int Lend = total;
  // list -> base bin of its 4 letter sub-lists, u_p, weights
  auto describe = [&](int Lx, uint32_t &base, uint32_t &up, int &wa, int &wb) {
    const int a = Lx / NSUB, s = Lx - a * NSUB;
    const uint32_t d = sub[s];
    const int p = d & 0xFF, q = (d >> 8) & 0xFF;
    const uint32_t rk = rotk[a * K + p];
    up = rk & 3u;
    uint32_t key = rk >> 2;
    if (q == 0xFF) {
      wa = (p == 0) ? w0 : 0;
      wb = w1;
    } else {
      // letter q of u sits at key digit q (q < p); substitute the ci-th other letter
      const int sh = 2 * (K - 2 - q);
      const uint32_t lq = (key >> sh) & 3u;
      const uint32_t nl = (lq + 1u + (d >> 16)) & 3u;
      key ^= (lq ^ nl) << sh;
      wa = 0;
      wb = w2;
    }
    base = (uint32_t)p * copy_stride + chunk_bins + (key << 2);
  };

  // segment bounds of the current list: [b0,b1) wb, [b1,b2) wa, [b2,b3) wb
  uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
  int wa = 0, wb = 0;
  auto load_bounds = [&](uint32_t base, uint32_t up, uint32_t &x0, uint32_t &x1, uint32_t &x2,
                         uint32_t &x3) {
    const uint4 o4 = *(const uint4 *)(off + base);  // base % 4 == 0: 16-byte aligned
    const uint32_t o5 = off[base + 4];
    const uint32_t lo = up == 0 ? o4.x : up == 1 ? o4.y : up == 2 ? o4.z : o4.w;
    const uint32_t hi = up == 0 ? o4.y : up == 1 ? o4.z : up == 2 ? o4.w : o5;
    x0 = o4.x; x1 = lo; x2 = hi; x3 = o5;
  };
  if (L < Lend) {
    uint32_t base, up;
    describe(L, base, up, wa, wb);
    load_bounds(base, up, b0, b1, b2, b3);
  }
  for (; L < Lend; L += ngrp) {
    uint32_t n0 = 0, n1 = 0, n2 = 0, n3 = 0;
    int nwa = 0, nwb = 0;
    if (L + ngrp < Lend) {
      uint32_t base, up;
      describe(L + ngrp, base, up, nwa, nwb);
      load_bounds(base, up, n0, n1, n2, n3);
    }
    // virtual index t over [b0,b1) ++ ([b1,b2) if wa) ++ [b2,b3)
    const uint32_t lA = b1 - b0, lB = wa ? (b2 - b1) : 0u, lC = b3 - b2;
    const uint32_t tot = lA + lB + lC;
    for (uint32_t t0 = 0; t0 < tot; t0 += 4 * G) {
      uint32_t col[4];
      int wt[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t t = t0 + u * G + gl;
        uint32_t e;
        int w;
        if (t < lA) { e = b0 + t; w = wb; }
        else if (t < lA + lB) { e = b1 + (t - lA); w = wa; }
        else { e = b2 + (t - lA - lB); w = wb; }
        wt[u] = (t < tot) ? w : 0;
        col[u] = (t < tot) ? (uint32_t)ent[e] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (wt[u]) atomicAdd(&acc[col[u]], wt[u]);
    }
    b0 = n0; b1 = n1; b2 = n2; b3 = n3;
    wa = nwa;
    wb = nwb;
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int qq = threadIdx.x * 4; qq < cw; qq += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[qq];
    if (o.dtype == KMG_F64)
      emit4<KMG_F64>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else if (o.dtype == KMG_F32)
      emit4<KMG_F32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else
      emit4<KMG_I32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
  }
}

// ------------------------------------------------------------------ mismatch m=1, v4
// Rotated layout (as v3) with a 3-stage software pipeline per lane group, lists taken
// interleaved (groups of a wave work on consecutive sub-lists of one k-mer):
//   iteration t: (1) decode list t+2, issue its 5 bin offsets;
//                (2) wait for list t+1's offsets, issue up to U*G of its entries;
//                (3) wait for list t's entries, LDS atomics.
// Loads are unconditional (clamped address, masked weight) so hipcc can emit counted
// vmcnt waits instead of draining; a list longer than U*G entries finishes in a slow
// synchronous loop (rare: average list length ~ 3/4 * 4 * chunk * P / 4^k).
template <int K, int G, int U>
__global__ __launch_bounds__(1024) void gram_mm1p_kernel(IndexGeom g,
                                                         const uint8_t *__restrict__ codes,
                                                         int64_t ldc,
                                                         const uint32_t *__restrict__ off,
                                                         const uint16_t *__restrict__ ent,
                                                         int64_t row0, int w0, int w1, int w2,
                                                         OutSpec o) {
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rotk = smem + accw;   // [P][K]: rot_p(u_a)
  uint32_t *sub = rotk + P * K;   // [NSUB]: p | q << 8 | ci << 16 (q = 0xFF: type 1)
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const uint8_t *rs = codes + i * ldc;
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = window_code(rs, a, K);
    rotk[t] = (drop_letter_g(u, p, K) << 2) | letter_at_g(u, p, K);
  }
  for (int s = threadIdx.x; s < NSUB; s += blockDim.x) {
    uint32_t d;
    if (s < K) {
      d = (uint32_t)s | (0xFFu << 8);
    } else {
      const int t = s - K, pi = t / 3, ci = t - 3 * pi;
      int pp = 1;
      while ((pp + 1) * pp / 2 <= pi) ++pp;
      d = (uint32_t)pp | ((uint32_t)(pi - pp * (pp - 1) / 2) << 8) | ((uint32_t)ci << 16);
    }
    sub[s] = d;
  }
  __syncthreads();

  const uint32_t chunk_bins = (uint32_t)c * g.nkeys;
  const uint32_t copy_stride = (uint32_t)g.nchunks * g.nkeys;
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int total = P * NSUB;
  const uint32_t last_bin = (uint32_t)g.nbins() - 4u;  // clamp for out-of-range lists

  // decode list Lx: base bin (multiple of 4) of its 4 letter sub-lists, and meta =
  // u_p | wa << 8 | wb << 16 (weights <= 255, checked by the host)
  auto describe = [&](int Lx, uint32_t &base, uint32_t &meta) {
    if (Lx >= total) {
      base = last_bin;
      meta = 0;  // zero weights: contributes nothing
      return;
    }
    const int a = Lx / NSUB, s = Lx - a * NSUB;
    const uint32_t d = sub[s];
    const int p = d & 0xFF, q = (d >> 8) & 0xFF;
    const uint32_t rk = rotk[a * K + p];
    uint32_t key = rk >> 2;
    uint32_t wa, wb;
    if (q == 0xFF) {
      wa = (p == 0) ? (uint32_t)w0 : 0u;
      wb = (uint32_t)w1;
    } else {
      const int sh = 2 * (K - 2 - q);  // letter q of u sits at key digit q (q < p)
      const uint32_t lq = (key >> sh) & 3u;
      const uint32_t nl = (lq + 1u + (d >> 16)) & 3u;
      key ^= (lq ^ nl) << sh;
      wa = 0u;
      wb = (uint32_t)w2;
    }
    base = (uint32_t)p * copy_stride + chunk_bins + (key << 2);
    meta = (rk & 3u) | (wa << 8) | (wb << 16);
  };
  // segments of a list: [x0,x1) wb, [x1,x2) wa (dropped when wa == 0), [x2,x3) wb
  struct Seg {
    uint32_t b0, b1, b2, lA, lB, tot;
    int wa, wb;
  };
  auto segs = [&](const uint4 o4, uint32_t o5, uint32_t meta) {
    const uint32_t up = meta & 3u;
    Seg sg;
    const uint32_t lo = up == 0 ? o4.x : up == 1 ? o4.y : up == 2 ? o4.z : o4.w;
    const uint32_t hi = up == 0 ? o4.y : up == 1 ? o4.z : up == 2 ? o4.w : o5;
    sg.wa = (int)((meta >> 8) & 0xFFu);
    sg.wb = (int)(meta >> 16);
    sg.b0 = o4.x;
    sg.b1 = lo;
    sg.b2 = hi;
    sg.lA = lo - o4.x;
    sg.lB = sg.wa ? (hi - lo) : 0u;
    sg.tot = sg.lA + sg.lB + (o5 - hi);
    return sg;
  };
  auto ent_index = [&](const Seg &sg, uint32_t t, uint32_t &e, int &w) {
    if (t < sg.lA) { e = sg.b0 + t; w = sg.wb; }
    else if (t < sg.lA + sg.lB) { e = sg.b1 + (t - sg.lA); w = sg.wa; }
    else { e = sg.b2 + (t - sg.lA - sg.lB); w = sg.wb; }
    if (t >= sg.tot) { e = sg.b0; w = 0; }  // clamped, masked
  };

  int L = grp;
  // prologue: offsets of lists L and L+ngrp; entries of list L
  uint32_t baseA, metaA, baseB, metaB;
  describe(L, baseA, metaA);
  uint4 oA4 = *(const uint4 *)(off + baseA);
  uint32_t oA5 = off[baseA + 4];
  describe(L + ngrp, baseB, metaB);
  uint4 oB4 = *(const uint4 *)(off + baseB);
  uint32_t oB5 = off[baseB + 4];
  Seg cur = segs(oA4, oA5, metaA);
  uint32_t ecur[U];
  int wcur[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    uint32_t e;
    int w;
    ent_index(cur, (uint32_t)(u * G + gl), e, w);
    wcur[u] = w;
    ecur[u] = ent[e];
  }
  for (; L < total; L += ngrp) {
    // (1) offsets of list L + 2*ngrp
    uint32_t baseC, metaC;
    describe(L + 2 * ngrp, baseC, metaC);
    const uint4 oC4 = *(const uint4 *)(off + baseC);
    const uint32_t oC5 = off[baseC + 4];
    // (2) entries of list L + ngrp
    const Seg nxt = segs(oB4, oB5, metaB);
    uint32_t enxt[U];
    int wnxt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t e;
      int w;
      ent_index(nxt, (uint32_t)(u * G + gl), e, w);
      wnxt[u] = w;
      enxt[u] = ent[e];
    }
    // (3) atomics of list L
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (wcur[u]) atomicAdd(&acc[ecur[u]], wcur[u]);
    for (uint32_t t = (uint32_t)(U * G + gl); t < cur.tot; t += G) {  // rare long list
      uint32_t e;
      int w;
      ent_index(cur, t, e, w);
      if (w) atomicAdd(&acc[ent[e]], w);
    }
    cur = nxt;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ecur[u] = enxt[u];
      wcur[u] = wnxt[u];
    }
    oB4 = oC4;
    oB5 = oC5;
    metaB = metaC;
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int qq = threadIdx.x * 4; qq < cw; qq += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[qq];
    if (o.dtype == KMG_F64)
      emit4<KMG_F64>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else if (o.dtype == KMG_F32)
      emit4<KMG_F32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else
      emit4<KMG_I32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
  }
}

// ------------------------------------------------------------------ mismatch m=1, v5
// Rotated layout, branch-free: each lane group (G lanes, G = 1 or 2 by default) owns one
// list at a time and covers it with U unrolled entry slots per lane; every slot computes
// its entry index and weight with selects (masked slots add 0), entry and bin-offset
// reads are raw buffer loads (32-bit offsets, out-of-range reads return 0), and the
// next list's offsets load while this list's entries are in flight.
//   list (p, key): bins key*4 .. key*4+3 (letter at p); type 1 p=0 covers all 4 bins
//   (letter u_p -> w0, others -> w1); otherwise the letter-u_p bin is skipped.
template <int K, int G, int U>
__global__ __launch_bounds__(1024) void gram_mm1b_kernel(IndexGeom g,
                                                         const uint8_t *__restrict__ codes,
                                                         int64_t ldc,
                                                         const uint32_t *__restrict__ off,
                                                         const uint16_t *__restrict__ ent,
                                                         uint32_t n_ent, int64_t row0, int w0,
                                                         int w1, int w2, OutSpec o) {
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rotk = smem + accw;   // [P][K]: rot_p(u_a)
  uint32_t *sub = rotk + P * K;   // [NSUB]: p | q << 8 | ci << 16 (q = 0xFF: type 1)
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const uint8_t *rs = codes + i * ldc;
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = window_code(rs, a, K);
    rotk[t] = (drop_letter_g(u, p, K) << 2) | letter_at_g(u, p, K);
  }
  for (int s = threadIdx.x; s < NSUB; s += blockDim.x) {
    uint32_t d;
    if (s < K) {
      d = (uint32_t)s | (0xFFu << 8);
    } else {
      const int t = s - K, pi = t / 3, ci = t - 3 * pi;
      int pp = 1;
      while ((pp + 1) * pp / 2 <= pi) ++pp;
      d = (uint32_t)pp | ((uint32_t)(pi - pp * (pp - 1) / 2) << 8) | ((uint32_t)ci << 16);
    }
    sub[s] = d;
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t roff =
      __builtin_amdgcn_make_buffer_rsrc((void *)off, (short)0, (int)((g.nbins() + 1) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rent =
      __builtin_amdgcn_make_buffer_rsrc((void *)ent, (short)0, (int)(n_ent * 2u), 0x00020000);
  const uint32_t chunk_bins = (uint32_t)c * g.nkeys;
  const uint32_t copy_stride = (uint32_t)g.nchunks * g.nkeys;
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int total = P * NSUB;

  // branch-free list decode -> base bin (multiple of 4), letter u_p, weights
  auto describe = [&](int L, uint32_t &base, uint32_t &up, int &wa, int &wb) {
    const bool valid = L < total;
    const int Lc = valid ? L : total - 1;
    const int a = Lc / NSUB, s = Lc - a * NSUB;
    const uint32_t d = sub[s];
    const int p = d & 0xFF;
    const bool t1 = ((d >> 8) & 0xFF) == 0xFF;
    const int q = t1 ? 0 : (int)((d >> 8) & 0xFF);
    const uint32_t rk = rotk[a * K + p];
    const uint32_t key = rk >> 2;
    const int sh = 2 * (K - 2 - q);
    const uint32_t lq = (key >> sh) & 3u;
    const uint32_t nl = (lq + 1u + (d >> 16)) & 3u;
    const uint32_t key2 = key ^ ((lq ^ nl) << sh);
    base = (uint32_t)p * copy_stride + chunk_bins + ((t1 ? key : key2) << 2);
    up = rk & 3u;
    wa = (valid && t1 && p == 0) ? w0 : 0;
    wb = valid ? (t1 ? w1 : w2) : 0;
  };

  int L = grp;
  uint32_t base, up;
  int wa, wb;
  describe(L, base, up, wa, wb);
  uint4 o4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(roff, base * 4u, 0, 0));
  uint32_t o5 = __builtin_amdgcn_raw_buffer_load_b32(roff, base * 4u + 16u, 0, 0);
  for (; L < total; L += ngrp) {
    // segments of this list
    const uint32_t lo = up == 0 ? o4.x : up == 1 ? o4.y : up == 2 ? o4.z : o4.w;
    const uint32_t hi = up == 0 ? o4.y : up == 1 ? o4.z : up == 2 ? o4.w : o5;
    const bool full = wa != 0;
    const uint32_t b0 = o4.x;
    const uint32_t lR1 = full ? (o5 - o4.x) : (lo - o4.x);
    const uint32_t b2p = hi;
    const uint32_t tot = full ? (o5 - o4.x) : (lo - o4.x) + (o5 - hi);
    const uint32_t lenB = full ? (hi - lo) : 0u;
    const int cwa = wa, cwb = wb;
    // issue this list's entries
    uint32_t col[U];
    int wt[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t t = (uint32_t)(u * G + gl);
      const uint32_t e = t < lR1 ? b0 + t : b2p + (t - lR1);
      col[u] = __builtin_amdgcn_raw_buffer_load_b16(rent, e * 2u, 0, 0);
      wt[u] = t < tot ? ((e - lo) < lenB ? cwa : cwb) : 0;
    }
    // next list's offsets in flight with them
    describe(L + ngrp, base, up, wa, wb);
    o4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(roff, base * 4u, 0, 0));
    o5 = __builtin_amdgcn_raw_buffer_load_b32(roff, base * 4u + 16u, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) atomicAdd(&acc[col[u]], wt[u]);
    for (uint32_t t = (uint32_t)(U * G + gl); t < tot; t += G) {  // rare long list
      const uint32_t e = t < lR1 ? b0 + t : b2p + (t - lR1);
      const uint32_t cc = __builtin_amdgcn_raw_buffer_load_b16(rent, e * 2u, 0, 0);
      atomicAdd(&acc[cc], (e - lo) < lenB ? cwa : cwb);
    }
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int qq = threadIdx.x * 4; qq < cw; qq += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[qq];
    if (o.dtype == KMG_F64)
      emit4<KMG_F64>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else if (o.dtype == KMG_F32)
      emit4<KMG_F32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else
      emit4<KMG_I32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
  }
}

// ------------------------------------------------------------------ mismatch m=1, v6
// Rotated layout; the texture-address unit, not the VALU, bounds a 2-byte gather (one
// wave-wide load with 64 scattered lines costs ~38 TA cycles), so every lane group (G
// lanes) reads its list's whole 4-bin range [b0, b4) with aligned V-entry vector loads
// (V=4: 8 B, V=8: 16 B per lane; U loads per lane), and each entry is masked by range
// and weighted by whether it lies in the letter-u_p bin [lo, hi):
//   type 1, p=0: u_p bin -> w0, other letters -> w1;  type 1, p>0: u_p bin -> 0, others w1;
//   type 2: u_p bin -> 0, others -> w2.
template <int K, int G, int V, int U>
__global__ __launch_bounds__(1024) void gram_mm1v_kernel(IndexGeom g,
                                                         const uint8_t *__restrict__ codes,
                                                         int64_t ldc,
                                                         const uint32_t *__restrict__ off,
                                                         const uint16_t *__restrict__ ent,
                                                         uint32_t n_ent, int64_t row0, int w0,
                                                         int w1, int w2, OutSpec o) {
  static_assert(V == 4 || V == 8, "vector width");
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];
  const int64_t il = blockIdx.x / g.nchunks;
  const int64_t i = row0 + il;
  const int c = blockIdx.x - (int)il * g.nchunks;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rotk = smem + accw;   // [P][K]: rot_p(u_a)
  uint32_t *sub = rotk + P * K;   // [NSUB]: p | q << 8 | ci << 16 (q = 0xFF: type 1)
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const uint8_t *rs = codes + i * ldc;
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = window_code(rs, a, K);
    rotk[t] = (drop_letter_g(u, p, K) << 2) | letter_at_g(u, p, K);
  }
  for (int s = threadIdx.x; s < NSUB; s += blockDim.x) {
    uint32_t d;
    if (s < K) {
      d = (uint32_t)s | (0xFFu << 8);
    } else {
      const int t = s - K, pi = t / 3, ci = t - 3 * pi;
      int pp = 1;
      while ((pp + 1) * pp / 2 <= pi) ++pp;
      d = (uint32_t)pp | ((uint32_t)(pi - pp * (pp - 1) / 2) << 8) | ((uint32_t)ci << 16);
    }
    sub[s] = d;
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t roff =
      __builtin_amdgcn_make_buffer_rsrc((void *)off, (short)0, (int)((g.nbins() + 1) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rent =
      __builtin_amdgcn_make_buffer_rsrc((void *)ent, (short)0, (int)(n_ent * 2u), 0x00020000);
  const uint32_t chunk_bins = (uint32_t)c * g.nkeys;
  const uint32_t copy_stride = (uint32_t)g.nchunks * g.nkeys;
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int total = P * NSUB;

  auto describe = [&](int L, uint32_t &base, uint32_t &up, int &wa, int &wb) {
    const bool valid = L < total;
    const int Lc = valid ? L : total - 1;
    const int a = Lc / NSUB, s = Lc - a * NSUB;
    const uint32_t d = sub[s];
    const int p = d & 0xFF;
    const bool t1 = ((d >> 8) & 0xFF) == 0xFF;
    const int q = t1 ? 0 : (int)((d >> 8) & 0xFF);
    const uint32_t rk = rotk[a * K + p];
    const uint32_t key = rk >> 2;
    const int sh = 2 * (K - 2 - q);
    const uint32_t lq = (key >> sh) & 3u;
    const uint32_t nl = (lq + 1u + (d >> 16)) & 3u;
    const uint32_t key2 = key ^ ((lq ^ nl) << sh);
    base = (uint32_t)p * copy_stride + chunk_bins + ((t1 ? key : key2) << 2);
    up = rk & 3u;
    wa = (valid && t1 && p == 0) ? w0 : 0;
    wb = valid ? (t1 ? w1 : w2) : 0;
  };

  int L = grp;
  uint32_t base, up;
  int wa, wb;
  describe(L, base, up, wa, wb);
  uint4 o4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(roff, base * 4u, 0, 0));
  uint32_t o5 = __builtin_amdgcn_raw_buffer_load_b32(roff, base * 4u + 16u, 0, 0);
  for (; L < total; L += ngrp) {
    const uint32_t lo = up == 0 ? o4.x : up == 1 ? o4.y : up == 2 ? o4.z : o4.w;
    const uint32_t hi = up == 0 ? o4.y : up == 1 ? o4.z : up == 2 ? o4.w : o5;
    const uint32_t b0 = o4.x, b4 = o5;
    const uint32_t a0 = b0 & ~(uint32_t)(V - 1);  // aligned window start
    const int cwa = wa, cwb = wb;
    // this list's entries: U aligned vectors of V entries per lane
    uint32_t vec[U][V / 2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t e0 = a0 + (uint32_t)((u * G + gl) * V);
      if constexpr (V == 8) {
        const uint4 x = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rent, e0 * 2u, 0, 0));
        vec[u][0] = x.x; vec[u][1] = x.y; vec[u][2] = x.z; vec[u][3] = x.w;
      } else {
        const uint2 x = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rent, e0 * 2u, 0, 0));
        vec[u][0] = x.x; vec[u][1] = x.y;
      }
    }
    const uint32_t span = (uint32_t)(U * G * V);
    // next list's offsets in flight with them
    describe(L + ngrp, base, up, wa, wb);
    o4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(roff, base * 4u, 0, 0));
    o5 = __builtin_amdgcn_raw_buffer_load_b32(roff, base * 4u + 16u, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t e0 = a0 + (uint32_t)((u * G + gl) * V);
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const uint32_t e = e0 + v;
        const uint32_t col = (vec[u][v >> 1] >> ((v & 1) * 16)) & 0xFFFFu;
        const int w = (e - b0 < b4 - b0) ? ((e - lo < hi - lo) ? cwa : cwb) : 0;
        atomicAdd(&acc[col], w);
      }
    }
    // rare: list longer than one window
    for (uint32_t e = a0 + span + (uint32_t)gl; e < b4; e += G) {
      const uint32_t cc = __builtin_amdgcn_raw_buffer_load_b16(rent, e * 2u, 0, 0);
      atomicAdd(&acc[cc], (e - lo < hi - lo) ? cwa : cwb);
    }
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int qq = threadIdx.x * 4; qq < cw; qq += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[qq];
    if (o.dtype == KMG_F64)
      emit4<KMG_F64>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else if (o.dtype == KMG_F32)
      emit4<KMG_F32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else
      emit4<KMG_I32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
  }
}

// ------------------------------------------------------------------ mismatch m=1, v7
// Slot layout (kmg_index.hip slot_pack_kernel): every 4-bin group (p, chunk, key) of the
// rotated index is also stored as ONE 128-byte line: uint16 e1, e2, e3, tot (ends of the
// letter-0/1/2 bins relative to the group start, and the group total; tot = 0xFFFF: the
// group is too large for 16-bit counts and lives in the CSR only) followed by the first
// KMG_SLOT_INLINE entries.  v6 pays an offsets line plus one or two entry lines per list
// and is bound by those L2-miss lines (Infinity-Cache traffic); here a list is one line.
// Entries past the inline ones come from the CSR (off/ent) in a slow path (rare at the
// chunk the host picks: mean group size <= 40).
//   G lanes per list, each loads 128/G bytes (CH = 8/G uint4); D lists in flight per
//   lane group (a ring unrolled at compile time); the grid is chunk-major so only one
//   chunk's slot table is live at a time (config 5: N = 200000 is 10 chunks).
template <int K, int G, int D>
__global__ __launch_bounds__(1024) void gram_mm1s_kernel(IndexGeom g,
                                                         const uint8_t *__restrict__ codes,
                                                         int64_t ldc,
                                                         const uint4 *__restrict__ slots,
                                                         const uint32_t *__restrict__ off,
                                                         const uint16_t *__restrict__ ent,
                                                         int64_t row0, int64_t rows, int w0,
                                                         int w1, int w2, OutSpec o) {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8, "lanes per list");
  constexpr int CH = 8 / G;
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];
  const int c = (int)(blockIdx.x / rows);
  const int64_t il = (int64_t)blockIdx.x - (int64_t)c * rows;
  const int64_t i = row0 + il;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rotk = smem + accw;   // [P][K]: rot_p(u_a)
  uint32_t *sub = rotk + P * K;   // [NSUB]: p | q << 8 | ci << 16 (q = 0xFF: type 1)
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const uint8_t *rs = codes + i * ldc;
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = window_code(rs, a, K);
    rotk[t] = (drop_letter_g(u, p, K) << 2) | letter_at_g(u, p, K);
  }
  for (int s = threadIdx.x; s < NSUB; s += blockDim.x) {
    uint32_t d;
    if (s < K) {
      d = (uint32_t)s | (0xFFu << 8);
    } else {
      const int t = s - K, pi = t / 3, ci = t - 3 * pi;
      int pp = 1;
      while ((pp + 1) * pp / 2 <= pi) ++pp;
      d = (uint32_t)pp | ((uint32_t)(pi - pp * (pp - 1) / 2) << 8) | ((uint32_t)ci << 16);
    }
    sub[s] = d;
  }
  __syncthreads();

  const uint32_t chunk_groups = (uint32_t)c * (g.nkeys >> 2);
  const uint32_t copy_groups = (uint32_t)g.nchunks * (g.nkeys >> 2);
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int lane = threadIdx.x & 63;
  const int total = P * NSUB;

  // list -> group index and meta = u_p | wa << 8 | wb << 16 (weights <= 255, host check)
  auto describe = [&](int L, uint32_t &gidx, uint32_t &meta) {
    const bool valid = L < total;
    const int Lc = valid ? L : total - 1;
    const int a = Lc / NSUB, s = Lc - a * NSUB;
    const uint32_t d = sub[s];
    const int p = d & 0xFF;
    const bool t1 = ((d >> 8) & 0xFF) == 0xFF;
    const int q = t1 ? 0 : (int)((d >> 8) & 0xFF);
    const uint32_t rk = rotk[a * K + p];
    const uint32_t key = rk >> 2;
    const int sh = 2 * (K - 2 - q);  // letter q of u sits at key digit q (q < p)
    const uint32_t lq = (key >> sh) & 3u;
    const uint32_t nl = (lq + 1u + (d >> 16)) & 3u;
    const uint32_t key2 = key ^ ((lq ^ nl) << sh);
    gidx = (uint32_t)p * copy_groups + chunk_groups + (t1 ? key : key2);
    const uint32_t wa = (valid && t1 && p == 0) ? (uint32_t)w0 : 0u;
    const uint32_t wb = valid ? (uint32_t)(t1 ? w1 : w2) : 0u;
    meta = (rk & 3u) | (wa << 8) | (wb << 16);
  };
  auto load = [&](uint32_t gidx, uint4(&b)[CH]) {
    const uint4 *sp = slots + (size_t)gidx * 8 + gl * CH;
#pragma unroll
    for (int j = 0; j < CH; ++j) b[j] = sp[j];
  };
  // slow path: entries [t0, tot) of group gidx from the CSR, letter bins from off[]
  auto csr_tail = [&](uint32_t gidx, uint32_t t0, uint32_t meta) {
    const uint32_t *ob = off + (size_t)gidx * 4;
    const uint32_t o0 = ob[0], o4 = ob[4];
    const uint32_t up = meta & 3u;
    const uint32_t lo = ob[up], hi = ob[up + 1];
    const int wa = (int)((meta >> 8) & 0xFFu), wb = (int)(meta >> 16);
    for (uint32_t e = o0 + t0 + (uint32_t)gl; e < o4; e += G) {
      const int w = (e - lo < hi - lo) ? wa : wb;
      if (w) atomicAdd(&acc[ent[e]], w);
    }
  };
  auto process = [&](const uint4(&b)[CH], uint32_t gidx, uint32_t meta) {
    // group header = the line's first 8 bytes (lane gl == 0, chunk 0)
    uint32_t h0 = b[0].x, h1 = b[0].y;
    if constexpr (G > 1) {
      const int src = lane & ~(G - 1);
      h0 = (uint32_t)__shfl((int)h0, src, 64);
      h1 = (uint32_t)__shfl((int)h1, src, 64);
    }
    const uint32_t e1 = h0 & 0xFFFFu, e2 = h0 >> 16, e3 = h1 & 0xFFFFu, tot = h1 >> 16;
    const uint32_t up = meta & 3u;
    const int wa = (int)((meta >> 8) & 0xFFu), wb = (int)(meta >> 16);
    const uint32_t lo = up == 0 ? 0u : up == 1 ? e1 : up == 2 ? e2 : e3;
    const uint32_t hi = up == 0 ? e1 : up == 1 ? e2 : up == 2 ? e3 : tot;
    const bool big = tot == 0xFFFFu;
    const uint32_t lim = big ? 0u : min(tot, (uint32_t)KMG_SLOT_INLINE);
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const uint32_t wd[4] = {b[j].x, b[j].y, b[j].z, b[j].w};
      const int tb = (gl * CH + j) * 8 - 4;  // entry index of the chunk's first halfword
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const int t = tb + v;  // t < 0: header halfwords
        const uint32_t col = (wd[v >> 1] >> ((v & 1) * 16)) & 0xFFFFu;
        const int w = (t >= 0 && (uint32_t)t < lim) ? (((uint32_t)t - lo < hi - lo) ? wa : wb) : 0;
        if (w) atomicAdd(&acc[col], w);
      }
    }
    if (big || tot > (uint32_t)KMG_SLOT_INLINE)
      csr_tail(gidx, big ? 0u : (uint32_t)KMG_SLOT_INLINE, meta);
  };

  uint4 buf[D][CH];
  uint32_t gid[D], met[D];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    describe(grp + r * ngrp, gid[r], met[r]);
    load(gid[r], buf[r]);
  }
  for (int L = grp; L < total; L += D * ngrp) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
      if (L + r * ngrp < total) process(buf[r], gid[r], met[r]);
      describe(L + (r + D) * ngrp, gid[r], met[r]);
      load(gid[r], buf[r]);
    }
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int qq = threadIdx.x * 4; qq < cw; qq += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[qq];
    if (o.dtype == KMG_F64)
      emit4<KMG_F64, true>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else if (o.dtype == KMG_F32)
      emit4<KMG_F32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else
      emit4<KMG_I32, true>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
  }
}

// LDS byte address of the 16-bit column in halfword H of w (acc at LDS offset 0): one
// SDWA shift instead of extract + shift-add.
template <int H>
__device__ __forceinline__ uint32_t col_addr_sdwa(uint32_t w) {
  uint32_t r;
  if constexpr (H == 0)
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
        "src1_sel:WORD_0"
        : "=v"(r)
        : "v"(w));
  else
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD "
        "src1_sel:WORD_1"
        : "=v"(r)
        : "v"(w));
  return r;
}

// ------------------------------------------------------------------ mismatch m=1, v8
// Same slot layout and list enumeration as v7 (gram_mm1s_kernel), two lanes per list,
// with the per-slot work cut down (v7 is VALU-issue-bound, profiles/r01s5_mm_pmc.txt):
//   * the two lanes of a list take the line's 16-byte pieces interleaved (lane gl takes
//     pieces gl, gl+2, gl+4, gl+6), so step j covers halfwords [16j, 16j+16) of every list
//     in the wave and a step is skipped when no list of the wave has entries there
//     (lists average ~28 entries of 60: the last step is almost never needed);
//   * SENT: positions past a group's entries hold sentinel columns (slot_pack_kernel)
//     that land in a 1024-dword scratch tail of the accumulator, so a slot costs
//     extract + weight select + ds_add with no validity test and no exec-mask juggling.
//     Only the four header halfwords of piece 0 are predicated.
template <int K, int D, int MODE>
__global__ __launch_bounds__(1024) void gram_mm1t_kernel(IndexGeom g,
                                                         const uint8_t *__restrict__ codes,
                                                         int64_t ldc,
                                                         const uint4 *__restrict__ slots,
                                                         const uint32_t *__restrict__ off,
                                                         const uint16_t *__restrict__ ent,
                                                         int64_t row0, int64_t rows, int w0,
                                                         int w1, int w2, OutSpec o, int tri,
                                                         int porder) {
  constexpr int G = 2, CH = 4;
  constexpr bool SENT = MODE == 1;  // sentinel slots
  constexpr bool DUMMY = MODE == 2;  // inactive lanes add into a per-lane dummy dword
  constexpr bool HALF = MODE == 3;   // ring loads the first 64 B (header + 28 entries);
                                     // the second 64 B only for groups of > 28 entries
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];  // acc first: LDS offset 0 (col_addr_sdwa)
  const int c = (int)(blockIdx.x / rows);
  const int64_t il = (int64_t)blockIdx.x - (int64_t)c * rows;
  const int64_t i = row0 + il;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int accl = SENT ? accw + 1024 : DUMMY ? accw + 64 : accw;  // + scratch tail
  // tri (full K, tested slots only): columns j >= i of row i; a chunk wholly left of the
  // diagonal is skipped, the lower triangle is mirrored afterwards (mirror_lower_kernel)
  const int64_t jlo = (tri && !SENT) ? max((int64_t)0, i - col0) : 0;
  if (jlo >= cw) return;
  const uint32_t thr4 = (uint32_t)jlo * 4u;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rotk = smem + accl;   // [P][K]: rot_p(u_a)
  uint32_t *sub = rotk + P * K;   // [NSUB]: p | q << 8 | ci << 16 (q = 0xFF: type 1)
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accl >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  const uint8_t *rs = codes + i * ldc;
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = window_code(rs, a, K);
    rotk[t] = (drop_letter_g(u, p, K) << 2) | letter_at_g(u, p, K);
  }
  for (int s = threadIdx.x; s < NSUB; s += blockDim.x) {
    uint32_t d;
    if (porder) {
      // copy-major: copy p owns 1 + 3p sub-lists (type 1, then (q < p, ci)); lists are
      // walked sub-list-major, so the lists in flight on an XCD read one copy's slot
      // table (2.1 MB at k = 9) and stay in its 4 MB L2
      int pp = 0;
      while ((pp + 1) + 3 * (pp + 1) * pp / 2 <= s) ++pp;
      const int r = s - (pp + 3 * pp * (pp - 1) / 2);
      d = r == 0 ? ((uint32_t)pp | (0xFFu << 8))
                 : ((uint32_t)pp | ((uint32_t)((r - 1) / 3) << 8) | ((uint32_t)((r - 1) % 3) << 16));
    } else if (s < K) {
      d = (uint32_t)s | (0xFFu << 8);
    } else {
      const int t = s - K, pi = t / 3, ci = t - 3 * pi;
      int pp = 1;
      while ((pp + 1) * pp / 2 <= pi) ++pp;
      d = (uint32_t)pp | ((uint32_t)(pi - pp * (pp - 1) / 2) << 8) | ((uint32_t)ci << 16);
    }
    sub[s] = d;
  }
  __syncthreads();

  const uint32_t chunk_groups = (uint32_t)c * (g.nkeys >> 2);
  const uint32_t copy_groups = (uint32_t)g.nchunks * (g.nkeys >> 2);
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int lane = threadIdx.x & 63;
  const int total = P * NSUB;
  const uint32_t dummy4 = (uint32_t)(accw + lane) * 4u;

  auto describe = [&](int L, uint32_t &gidx, uint32_t &meta) {
    const bool valid = L < total;
    const int Lc = valid ? L : total - 1;
    int a, s;
    if (porder) {
      s = Lc / P;
      a = Lc - s * P;
    } else {
      a = Lc / NSUB;
      s = Lc - a * NSUB;
    }
    const uint32_t d = sub[s];
    const int p = d & 0xFF;
    const bool t1 = ((d >> 8) & 0xFF) == 0xFF;
    const int q = t1 ? 0 : (int)((d >> 8) & 0xFF);
    const uint32_t rk = rotk[a * K + p];
    const uint32_t key = rk >> 2;
    const int sh = 2 * (K - 2 - q);
    const uint32_t lq = (key >> sh) & 3u;
    const uint32_t nl = (lq + 1u + (d >> 16)) & 3u;
    const uint32_t key2 = key ^ ((lq ^ nl) << sh);
    gidx = (uint32_t)p * copy_groups + chunk_groups + (t1 ? key : key2);
    const uint32_t wa = (valid && t1 && p == 0) ? (uint32_t)w0 : 0u;
    const uint32_t wb = valid ? (uint32_t)(t1 ? w1 : w2) : 0u;
    meta = (rk & 3u) | (wa << 8) | (wb << 16);
  };
  auto load = [&](uint32_t gidx, uint4(&b)[CH]) {
    const uint4 *sp = slots + (size_t)gidx * 8 + gl;
#pragma unroll
    for (int j = 0; j < (HALF ? 2 : CH); ++j) b[j] = sp[2 * j];
  };
  auto csr_tail = [&](uint32_t gidx, uint32_t t0, uint32_t meta) {
    const uint32_t *ob = off + (size_t)gidx * 4;
    const uint32_t o0 = ob[0], o4 = ob[4];
    const uint32_t up = meta & 3u;
    const uint32_t lo = ob[up], hi = ob[up + 1];
    const int wa = (int)((meta >> 8) & 0xFFu), wb = (int)(meta >> 16);
    for (uint32_t e = o0 + t0 + (uint32_t)gl; e < o4; e += G) {
      const int w = (e - lo < hi - lo) ? wa : wb;
      if (w) atomicAdd(&acc[ent[e]], w);
    }
  };
  auto process = [&](const uint4(&bin)[CH], uint32_t gidx, uint32_t meta) {
    uint4 b[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) b[j] = bin[j];
    // header = halfwords 0..3 of piece 0, held by lane gl == 0
    const int src = lane & ~(G - 1);
    const uint32_t h0 = (uint32_t)__shfl((int)b[0].x, src, 64);
    const uint32_t h1 = (uint32_t)__shfl((int)b[0].y, src, 64);
    const uint32_t e1 = h0 & 0xFFFFu, e2 = h0 >> 16, e3 = h1 & 0xFFFFu, tot = h1 >> 16;
    const uint32_t up = meta & 3u;
    const int wa = (int)((meta >> 8) & 0xFFu), wb = (int)(meta >> 16);
    const uint32_t lo = up == 0 ? 0u : up == 1 ? e1 : up == 2 ? e2 : e3;
    const uint32_t hi = up == 0 ? e1 : up == 1 ? e2 : up == 2 ? e3 : tot;
    const bool big = tot == 0xFFFFu;
    const uint32_t lim = (big || wb == 0) ? 0u : min(tot, (uint32_t)KMG_SLOT_INLINE);
    const uint32_t span = hi - lo;
    // entry index of halfword v of this lane's piece in step j: 16j + 8gl + v - 4
    const uint32_t lo_l = lo + 4u - 8u * (uint32_t)gl;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      if (j > 0 && !__any((int)lim > 16 * j - 4)) break;
      if constexpr (HALF) {
        if (j == 2) {  // second half of the line, loaded only by lists that reach it
          const uint4 *sp = slots + (size_t)gidx * 8 + gl;
          const uint4 z = make_uint4(0, 0, 0, 0);
          const bool need = (int)lim > 28;
          b[2] = need ? sp[4] : z;
          b[3] = need ? sp[6] : z;
        }
      }
      const uint32_t wd[4] = {b[j].x, b[j].y, b[j].z, b[j].w};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        const uint32_t col = (wd[v >> 1] >> ((v & 1) * 16)) & 0xFFFFu;
        const uint32_t rel = (uint32_t)(16 * j + v) - lo_l;  // = t - lo
        if constexpr (SENT) {
          const int w = rel < span ? wa : wb;
          if (j == 0 && v < 4) {
            if (gl != 0 && w) atomicAdd(&acc[col], w);
          } else {
            atomicAdd(&acc[col], w);
          }
        } else {
          // active: a valid inline entry outside the query letter's bin (weight wb); the
          // in-bin entries (weight wa: Hamming 0, copy 0 only) are added below
          const int t = 16 * j + 8 * gl + v - 4;
          const uint32_t ad = (v & 1) ? col_addr_sdwa<1>(wd[v >> 1]) : col_addr_sdwa<0>(wd[v >> 1]);
          const bool act = t >= 0 && (uint32_t)t < lim && rel >= span && ad >= thr4;
          if constexpr (DUMMY) {  // no exec-mask change: independent slots interleave
            __hip_atomic_fetch_add(
                (__attribute__((address_space(3))) int32_t *)(uintptr_t)(act ? ad : dummy4), wb,
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } else if (act) {
            __hip_atomic_fetch_add((__attribute__((address_space(3))) int32_t *)(uintptr_t)ad, wb,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
        }
      }
    }
    if constexpr (!SENT) {
      if (wa && !big) {  // in-bin inline entries [lo, min(hi, lim)) with weight wa, from the CSR
        const uint32_t o0 = off[(size_t)gidx * 4];
        const uint32_t e1x = o0 + min(hi, lim);
        for (uint32_t e = o0 + lo + (uint32_t)gl; e < e1x; e += G) atomicAdd(&acc[ent[e]], wa);
      }
    }
    if (big || tot > (uint32_t)KMG_SLOT_INLINE)
      csr_tail(gidx, big ? 0u : (uint32_t)KMG_SLOT_INLINE, meta);
  };

  uint4 buf[D][CH];
  uint32_t gid[D], met[D];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    describe(grp + r * ngrp, gid[r], met[r]);
    load(gid[r], buf[r]);
  }
  for (int L = grp; L < total; L += D * ngrp) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
      if (L + r * ngrp < total) process(buf[r], gid[r], met[r]);
      describe(L + (r + D) * ngrp, gid[r], met[r]);
      load(gid[r], buf[r]);
    }
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int qq = (int)(jlo & ~(int64_t)3) + threadIdx.x * 4; qq < cw; qq += blockDim.x * 4) {
    const int4 w = *(const int4 *)&acc[qq];
    if (o.dtype == KMG_F64)
      emit4<KMG_F64, true>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else if (o.dtype == KMG_F32)
      emit4<KMG_F32>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
    else
      emit4<KMG_I32, true>(o, il, i, col0 + qq, min(4, cw - qq), w.x, w.y, w.z, w.w, norm);
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
__global__ __launch_bounds__(64) void diag_ham_kernel(IndexGeom g, const uint8_t *__restrict__ codes,
                                                      const int32_t *__restrict__ lens, int64_t ldc,
                                                      const int64_t *__restrict__ wtab,
                                                      double *__restrict__ diagv,
                                                      double *__restrict__ dsq) {
  __shared__ int64_t w_s[33];
  __shared__ uint32_t xk[4096];
  const int lane = threadIdx.x;
  const int64_t i = blockIdx.x;
  if (lane <= g.k) w_s[lane] = wtab[lane];
  const int L = g.window > 0 ? g.window : lens[i];
  const int P = min(L - g.k + 1, 4096);
  const uint8_t *rs = codes + i * ldc;
  for (int a = lane; a < P; a += 64) xk[a] = window_code(rs, a, g.k);
  __syncthreads();
  const uint32_t mask55 = (g.k >= 16) ? 0x55555555u : (0x55555555u & ((1u << (2 * g.k)) - 1u));
  int64_t s = 0;
  for (int a = lane; a < P; a += 64) {
    const uint32_t xa = xk[a];
    if (xa == KMG_INVALID) continue;
    for (int b = 0; b < P; ++b) {
      const uint32_t yb = xk[b];
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

// raw self-kernel K_ii when the weights vanish beyond Hamming distance M2 = min(2m, k)
// <= 4 (m <= 2: every run.py / BASELINE mismatch kernel): one wave per sequence, four per
// block, k-mers staged in LDS; per lane only the histogram of distances 0..M2 is kept
// (int32) and weighted once at the end.  Same integer sum as diag_ham_kernel.
template <int M2>
__global__ __launch_bounds__(256) void diag_ham_small_kernel(IndexGeom g, const uint8_t *__restrict__ codes,
                                                             const int32_t *__restrict__ lens,
                                                             int64_t ldc,
                                                             const int64_t *__restrict__ wtab,
                                                             double *__restrict__ diagv,
                                                             double *__restrict__ dsq) {
  extern __shared__ __align__(16) uint32_t xk_all[];  // [4][pmax]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + wave;
  const bool valid = i < g.n;
  uint32_t *xk = xk_all + wave * g.pmax;
  int P = 0;
  if (valid) {
    const int L = g.window > 0 ? g.window : lens[i];
    P = max(0, min(L - g.k + 1, g.pmax));
    const uint8_t *rs = codes + i * ldc;
    for (int a = lane; a < P; a += 64) xk[a] = window_code(rs, a, g.k);
  }
  __syncthreads();
  if (!valid) return;
  const uint32_t mask55 = (g.k >= 16) ? 0x55555555u : (0x55555555u & ((1u << (2 * g.k)) - 1u));
  int cnt[M2 + 1];
#pragma unroll
  for (int d = 0; d <= M2; ++d) cnt[d] = 0;
  for (int a = lane; a < P; a += 64) {
    const uint32_t xa = xk[a];
    if (xa == KMG_INVALID) continue;
    for (int b = 0; b < P; ++b) {
      const uint32_t yb = xk[b];  // same address in every lane: LDS broadcast
      const int h = (yb == KMG_INVALID) ? 64 : ham2bit(xa, yb, mask55);
#pragma unroll
      for (int d = 0; d <= M2; ++d) cnt[d] += (h == d) ? 1 : 0;
    }
  }
  int64_t s = 0;
#pragma unroll
  for (int d = 0; d <= M2; ++d) s += (int64_t)cnt[d] * wtab[d];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
  if (lane == 0) {
    const double v = (double)s;
    diagv[i] = v;
    dsq[i] = __builtin_sqrt(v);  // np.sqrt(np.diag(K)) (kernels.py:408): IEEE sqrt
  }
}

// ------------------------------------------------------------------ launchers
static int env_int(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

#define KMG_DISPATCH_DT(DT, ...)                       \
  switch (DT) {                                        \
    case KMG_I32: { constexpr int D = KMG_I32; __VA_ARGS__; } break; \
    case KMG_F32: { constexpr int D = KMG_F32; __VA_ARGS__; } break; \
    default: { constexpr int D = KMG_F64; __VA_ARGS__; } break;      \
  }

hipError_t launch_gram_spectrum(const IndexGeom &g, const uint8_t *codes, const int32_t *lens,
                                int64_t ldc, const uint32_t *off, const uint16_t *ent,
                                int64_t row0, int64_t row1, const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  const bool pack = g.pmax <= 255;
  const int words = pack ? (((g.chunk + 7) >> 3) << 2) : (((g.chunk + 3) >> 2) << 2);
  const size_t lds = (size_t)words * 4;
  const int64_t nitems = rows * g.nchunks;
  // KMG_SP_PERSIST = p > 0: p waves of resident blocks (LDS-limited blocks per CU x 256
  // CUs) loop over the items instead of one block per item
  const int persist = env_int("KMG_SP_PERSIST", 0);
  int64_t nblk = nitems;
  if (persist > 0) {
    const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(8, (160 * 1024) / (int64_t)std::max<size_t>(lds, 1)));
    nblk = std::min<int64_t>(nitems, 256 * per_cu * persist);
  }
  const dim3 grid((unsigned)nblk);
  const bool nt = env_int("KMG_SP_NT", 1) != 0;
  // lanes per posting list (KMG_SP_G; 1, 2 or 4): at k=8, N=20000 the kernel is bound by
  // its row stores, and G = 1 measured 291.6 us against 298.9 (G = 2) and 303.5 (G = 4)
  const int G = env_int("KMG_SP_G", 1);
  if (pack && nt && G == 2) {
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<true, D, true, 2>), grid, dim3(256),
                                                lds, s, g, codes, lens, ldc, off, ent, row0, o, nitems));
  } else if (pack && nt && G == 4) {
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<true, D, true, 4>), grid, dim3(256),
                                                lds, s, g, codes, lens, ldc, off, ent, row0, o, nitems));
  } else if (pack && nt) {
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<true, D, true>), grid, dim3(256),
                                                lds, s, g, codes, lens, ldc, off, ent, row0, o, nitems));
  } else if (pack) {
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<true, D, false>), grid, dim3(256),
                                                lds, s, g, codes, lens, ldc, off, ent, row0, o, nitems));
  } else {
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<false, D, false>), grid, dim3(256),
                                                lds, s, g, codes, lens, ldc, off, ent, row0, o, nitems));
  }
  return hipGetLastError();
}

hipError_t launch_gram_mismatch1(const IndexGeom &g, const uint8_t *codes, int64_t ldc,
                                 const uint32_t *off, const uint16_t *ent, int64_t row0,
                                 int64_t row1, int w0, int w1, int w2, const OutSpec &o,
                                 hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  const int nsub = g.k + 3 * g.k * (g.k - 1) / 2;
  const size_t lds = (size_t)((((g.chunk + 3) >> 2) << 2) + g.pmax + nsub) * 4;
  const dim3 grid((unsigned)(rows * g.nchunks));
  // lanes per posting list: 4 unrolled loads per lane cover ~ the expected list length
  const double avg = (double)g.chunk * g.pmax / (double)g.nkeys;
  int G = 1;
  while (G < 64 && G * 4 < avg) G *= 2;
  G = env_int("KMG_MM_G", G);
  if (g.k >= 4 && g.k <= 12 && env_int("KMG_MM_VARIANT", 2) == 2) {
    const size_t lds2 = (size_t)((((g.chunk + 3) >> 2) << 2) + g.pmax * (g.k + 1)) * 4;
    const int G2 = G < 2 ? 2 : (G > 16 ? 16 : G);
    bool launched = false;
#define KMG_MM2(KK, GG)                                                                        \
  if (g.k == KK && G2 == GG) {                                                                 \
    hipLaunchKernelGGL((gram_mm1v2_kernel<KK, GG>), grid, dim3(MM_THREADS), lds2, s, g, codes, \
                       ldc, off, ent, row0, w0, w1, w2, o);                                    \
    launched = true;                                                                           \
  }
#define KMG_MM2K(KK) KMG_MM2(KK, 2) KMG_MM2(KK, 4) KMG_MM2(KK, 8) KMG_MM2(KK, 16)
    KMG_MM2K(4) KMG_MM2K(5) KMG_MM2K(6) KMG_MM2K(7) KMG_MM2K(8) KMG_MM2K(9) KMG_MM2K(10)
    KMG_MM2K(11) KMG_MM2K(12)
#undef KMG_MM2K
#undef KMG_MM2
    return launched ? hipGetLastError() : hipErrorInvalidConfiguration;
  }
#define KMG_MM_CASE(GG)                                                                    \
  case GG:                                                                                 \
    KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_mm1_kernel<GG, D>), grid,           \
                                                dim3(MM_THREADS), lds, s, g, nsub, codes, \
                                                ldc, off, ent, row0, w0, w1, w2, o));     \
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

hipError_t launch_gram_mismatch1_rot(const IndexGeom &g, const uint8_t *codes, int64_t ldc,
                                     const uint32_t *off, const uint16_t *ent, uint32_t n_ent,
                                     int64_t row0, int64_t row1, int w0, int w1, int w2,
                                     const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (g.k < 4 || g.k > 12) return hipErrorNotSupported;
  const int nsub = g.k + 3 * g.k * (g.k - 1) / 2;
  const size_t lds = (size_t)((((g.chunk + 3) >> 2) << 2) + g.pmax * g.k + nsub) * 4;
  const dim3 grid((unsigned)(rows * g.nchunks));
  const double avg = (double)g.chunk * g.pmax / ((double)g.nkeys / 4.0);  // per 4-bin list
  int G = 2;
  while (G < 16 && G * 4 < avg) G *= 2;
  G = env_int("KMG_MM_G", G);
  G = G < 2 ? 2 : (G > 16 ? 16 : G);
  const int threads = env_int("KMG_MM_THREADS", 1024) >= 1024 ? 1024 : 512;
  int variant = env_int("KMG_MM_VARIANT", 6);
  if (variant == 7) variant = 6;  // slot layout is k >= 8 only: v6 below that
  if (variant == 6) {
    const int G6 = env_int("KMG_MM_G", 4);
    const int V6 = env_int("KMG_MM_V", 4);
    const int U6 = env_int("KMG_MM_U", 2);
    bool launched = false;
#define KMG_MM6(KK, GG, VV, UU)                                                                    \
  if (g.k == KK && G6 == GG && V6 == VV && U6 == UU) {                                             \
    hipLaunchKernelGGL((gram_mm1v_kernel<KK, GG, VV, UU>), grid, dim3(threads), lds, s, g, codes,  \
                       ldc, off, ent, n_ent, row0, w0, w1, w2, o);                                 \
    launched = true;                                                                               \
  }
#define KMG_MM6K(KK)                                                                               \
  KMG_MM6(KK, 4, 4, 2) KMG_MM6(KK, 2, 4, 4) KMG_MM6(KK, 2, 8, 2) KMG_MM6(KK, 1, 8, 4)              \
  KMG_MM6(KK, 4, 8, 1) KMG_MM6(KK, 8, 4, 1) KMG_MM6(KK, 4, 4, 1) KMG_MM6(KK, 2, 8, 1)
    KMG_MM6K(4) KMG_MM6K(5) KMG_MM6K(6) KMG_MM6K(7) KMG_MM6K(8) KMG_MM6K(9) KMG_MM6K(10)
    KMG_MM6K(11) KMG_MM6K(12)
#undef KMG_MM6K
#undef KMG_MM6
    return launched ? hipGetLastError() : hipErrorInvalidConfiguration;
  }
  if (variant == 5) {
    const int G5 = env_int("KMG_MM_G", 1);
    const int U5 = env_int("KMG_MM_U", 24);
    bool launched = false;
#define KMG_MM5(KK, GG, UU)                                                                     \
  if (g.k == KK && G5 == GG && U5 == UU) {                                                      \
    hipLaunchKernelGGL((gram_mm1b_kernel<KK, GG, UU>), grid, dim3(threads), lds, s, g, codes,   \
                       ldc, off, ent, n_ent, row0, w0, w1, w2, o);                              \
    launched = true;                                                                            \
  }
#define KMG_MM5K(KK)                                                                            \
  KMG_MM5(KK, 1, 16) KMG_MM5(KK, 1, 24) KMG_MM5(KK, 1, 32) KMG_MM5(KK, 2, 8) KMG_MM5(KK, 2, 12)   \
  KMG_MM5(KK, 2, 16) KMG_MM5(KK, 4, 8)
    KMG_MM5K(4) KMG_MM5K(5) KMG_MM5K(6) KMG_MM5K(7) KMG_MM5K(8) KMG_MM5K(9) KMG_MM5K(10)
    KMG_MM5K(11) KMG_MM5K(12)
#undef KMG_MM5K
#undef KMG_MM5
    return launched ? hipGetLastError() : hipErrorInvalidConfiguration;
  }
  if (variant == 4) {
    const int U = env_int("KMG_MM_U", 8) >= 8 ? 8 : 4;
    bool launched = false;
#define KMG_MM4(KK, GG, UU)                                                                     \
  if (g.k == KK && G == GG && U == UU) {                                                        \
    hipLaunchKernelGGL((gram_mm1p_kernel<KK, GG, UU>), grid, dim3(threads), lds, s, g, codes,   \
                       ldc, off, ent, row0, w0, w1, w2, o);                                     \
    launched = true;                                                                            \
  }
#define KMG_MM4K(KK)                                                                            \
  KMG_MM4(KK, 2, 4) KMG_MM4(KK, 4, 4) KMG_MM4(KK, 8, 4) KMG_MM4(KK, 16, 4) KMG_MM4(KK, 2, 8)    \
  KMG_MM4(KK, 4, 8) KMG_MM4(KK, 8, 8) KMG_MM4(KK, 16, 8)
    KMG_MM4K(4) KMG_MM4K(5) KMG_MM4K(6) KMG_MM4K(7) KMG_MM4K(8) KMG_MM4K(9) KMG_MM4K(10)
    KMG_MM4K(11) KMG_MM4K(12)
#undef KMG_MM4K
#undef KMG_MM4
    return launched ? hipGetLastError() : hipErrorInvalidConfiguration;
  }
  bool launched = false;
#define KMG_MM3(KK, GG)                                                                         \
  if (g.k == KK && G == GG) {                                                                   \
    hipLaunchKernelGGL((gram_mm1rot_kernel<KK, GG>), grid, dim3(threads), lds, s, g, codes,     \
                       ldc, off, ent, row0, w0, w1, w2, o);                                     \
    launched = true;                                                                            \
  }
#define KMG_MM3K(KK) KMG_MM3(KK, 2) KMG_MM3(KK, 4) KMG_MM3(KK, 8) KMG_MM3(KK, 16)
  KMG_MM3K(4) KMG_MM3K(5) KMG_MM3K(6) KMG_MM3K(7) KMG_MM3K(8) KMG_MM3K(9) KMG_MM3K(10)
  KMG_MM3K(11) KMG_MM3K(12)
#undef KMG_MM3K
#undef KMG_MM3
  return launched ? hipGetLastError() : hipErrorInvalidConfiguration;
}

hipError_t launch_gram_mismatch1_slots(const IndexGeom &g, const uint8_t *codes, int64_t ldc,
                                       const uint4 *slots, const uint32_t *off,
                                       const uint16_t *ent, int64_t row0, int64_t row1, int w0,
                                       int w1, int w2, const OutSpec &o, int tri, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (g.k < 8 || g.k > 12 || !g.rot) return hipErrorNotSupported;
  if (w0 > 255 || w1 > 255 || w2 > 255) return hipErrorNotSupported;
  if (rows * g.nchunks > 0x7FFFFFFFLL) return hipErrorInvalidValue;
  const int nsub = g.k + 3 * g.k * (g.k - 1) / 2;
  const size_t lds = (size_t)((((g.chunk + 3) >> 2) << 2) + g.pmax * g.k + nsub) * 4;
  const dim3 grid((unsigned)(rows * g.nchunks));
  const int threads = env_int("KMG_MM_THREADS", 1024) >= 1024 ? 1024 : 512;
  const int G7 = env_int("KMG_MM_G", 2);
  const int D7 = env_int("KMG_MM_D", 2);
  // 0: v7, 1: v8 tested, 2: v8 sentinel slots, 3: v8 per-lane dummy, 4: v8 half lines
  const int V8 = env_int("KMG_MM_SLOTV", 1);
  bool launched = false;
  // v8 is built for two lanes per list and a 2- or 3-deep ring; other (G, D) choices
  // select the v7 instances below
  if (V8 >= 1 && V8 <= 4 && G7 == 2 && (D7 == 2 || D7 == 3)) {
    const size_t lds8 = lds + (V8 == 2 ? 1024 * 4 : V8 == 3 ? 64 * 4 : 0);
    const int porder = env_int("KMG_MM_PORDER", 1);
#define KMG_MM8(KK, DD, SS)                                                                      \
  if (g.k == KK && D7 == DD && V8 - 1 == SS) {                                                   \
    hipLaunchKernelGGL((gram_mm1t_kernel<KK, DD, SS>), grid, dim3(threads), lds8, s, g, codes,   \
                       ldc, slots, off, ent, row0, rows, w0, w1, w2, o, tri, porder);            \
    launched = true;                                                                             \
  }
#define KMG_MM8K(KK)                                                                             \
  KMG_MM8(KK, 2, 0) KMG_MM8(KK, 2, 1) KMG_MM8(KK, 2, 2) KMG_MM8(KK, 3, 0) KMG_MM8(KK, 3, 1)        \
  KMG_MM8(KK, 3, 2) KMG_MM8(KK, 2, 3) KMG_MM8(KK, 3, 3)
    KMG_MM8K(8) KMG_MM8K(9) KMG_MM8K(10) KMG_MM8K(11) KMG_MM8K(12)
#undef KMG_MM8K
#undef KMG_MM8
    return launched ? hipGetLastError() : hipErrorInvalidConfiguration;
  }
#define KMG_MM7(KK, GG, DD)                                                                      \
  if (g.k == KK && G7 == GG && D7 == DD) {                                                       \
    hipLaunchKernelGGL((gram_mm1s_kernel<KK, GG, DD>), grid, dim3(threads), lds, s, g, codes,    \
                       ldc, slots, off, ent, row0, rows, w0, w1, w2, o);                         \
    launched = true;                                                                             \
  }
#define KMG_MM7K(KK)                                                                             \
  KMG_MM7(KK, 2, 2) KMG_MM7(KK, 2, 3) KMG_MM7(KK, 2, 4) KMG_MM7(KK, 1, 2) KMG_MM7(KK, 1, 3)      \
  KMG_MM7(KK, 4, 2) KMG_MM7(KK, 8, 2) KMG_MM7(KK, 4, 3)
  KMG_MM7K(8) KMG_MM7K(9) KMG_MM7K(10) KMG_MM7K(11) KMG_MM7K(12)
#undef KMG_MM7K
#undef KMG_MM7
  return launched ? hipGetLastError() : hipErrorInvalidConfiguration;
}

// ------------------------------------------------------------------ mirror
// K[j][i] = K[i][j] for j > i on a full row-major n x n K (the reference fills j > i and
// mirrors, kernels.py:409-413): one 64 x 64 tile per workgroup, staged through LDS so both
// the upper-tile read and the lower-tile write are row-contiguous.
template <typename T>
__global__ __launch_bounds__(256) void mirror_lower_kernel(T *__restrict__ K, int64_t ld, int64_t n,
                                                           int64_t ntile) {
  // 16-byte row segments: V elements per lane, 64 / V lanes per tile row
  constexpr int V = 16 / (int)sizeof(T), LPR = 64 / V, RPP = 256 / LPR;
  __shared__ T tile[64][64 + 1];
  const int64_t b = blockIdx.x;  // -> (bi >= bj) over the lower tile triangle
  int64_t bi = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while (bi * (bi + 1) / 2 > b) --bi;
  while ((bi + 1) * (bi + 2) / 2 <= b) ++bi;
  const int64_t bj = b - bi * (bi + 1) / 2;
  if (bi >= ntile) return;
  const int64_t r0 = bj * 64, c0 = bi * 64;  // source: upper tile (rows of bj, cols of bi)
  const int cx = (threadIdx.x % LPR) * V, ry = threadIdx.x / LPR;
  const bool vec = ((ld * (int64_t)sizeof(T)) & 15) == 0 && (((uintptr_t)K) & 15) == 0;
  for (int r = ry; r < 64; r += RPP) {
    const int64_t gr = r0 + r, gc = c0 + cx;
    if (gr >= n) break;
    const T *src = K + gr * ld + gc;
    if (vec && gc + V <= n) {
      const uint4 w = *(const uint4 *)src;
      T v[V];
      __builtin_memcpy(v, &w, 16);
#pragma unroll
      for (int q = 0; q < V; ++q) tile[r][cx + q] = v[q];
    } else {
      for (int q = 0; q < V; ++q)
        if (gc + q < n) tile[r][cx + q] = src[q];
    }
  }
  __syncthreads();
  for (int r = ry; r < 64; r += RPP) {  // destination row c0 + r, columns r0 + cx ..
    const int64_t gr = c0 + r, gc = r0 + cx;
    if (gr >= n) break;
    T *dst = K + gr * ld + gc;
    T v[V];
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = tile[cx + q][r];
    if (vec && gc + V <= gr && gc + V <= n) {  // whole segment strictly below the diagonal
      uint4 w;
      __builtin_memcpy(&w, v, 16);
      __builtin_nontemporal_store(w.x, (uint32_t *)dst);
      __builtin_nontemporal_store(w.y, (uint32_t *)dst + 1);
      __builtin_nontemporal_store(w.z, (uint32_t *)dst + 2);
      __builtin_nontemporal_store(w.w, (uint32_t *)dst + 3);
    } else {
      for (int q = 0; q < V; ++q)
        if (gc + q < gr && gc + q < n) dst[q] = v[q];
    }
  }
}

hipError_t launch_mirror_lower(void *K, int64_t ld, int64_t n, int32_t dtype, hipStream_t s) {
  if (n <= 1) return hipSuccess;
  const int64_t nt = (n + 63) / 64;
  const int64_t blocks = nt * (nt + 1) / 2;
  if (blocks > 0x7FFFFFFFLL) return hipErrorInvalidValue;
  if (dtype == KMG_F64)
    hipLaunchKernelGGL(mirror_lower_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (double *)K, ld, n, nt);
  else
    hipLaunchKernelGGL(mirror_lower_kernel<uint32_t>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (uint32_t *)K, ld, n, nt);
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

hipError_t launch_diag_hamming(const IndexGeom &g, const uint8_t *codes, const int32_t *lens,
                               int64_t ldc, const int64_t *wtab, int max_dist, double *diagv,
                               double *dsq, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  if (max_dist <= 4 && g.pmax <= 4096 && env_int("KMG_DIAG_SMALL", 1)) {
    const dim3 grid((unsigned)((g.n + 3) / 4));
    const size_t lds = (size_t)4 * g.pmax * sizeof(uint32_t);
#define KMG_DIAG(M2_)                                                                          \
  case M2_:                                                                                    \
    hipLaunchKernelGGL((diag_ham_small_kernel<M2_>), grid, dim3(256), lds, s, g, codes, lens,   \
                       ldc, wtab, diagv, dsq);                                                 \
    break;
    switch (max_dist < 0 ? 0 : max_dist) {
      KMG_DIAG(0)
      KMG_DIAG(1)
      KMG_DIAG(2)
      KMG_DIAG(3)
      default:
        KMG_DIAG(4)
    }
#undef KMG_DIAG
    return hipGetLastError();
  }
  hipLaunchKernelGGL(diag_ham_kernel, dim3((unsigned)g.n), dim3(64), 0, s, g, codes, lens, ldc,
                     wtab, diagv, dsq);
  return hipGetLastError();
}

}  // namespace kmg
