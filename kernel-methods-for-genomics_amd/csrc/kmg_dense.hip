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
// Layout in HBM: F int8 [rows_alloc][dp], dp = 4^k rounded up to 128, rows_alloc >= n
// rounded up to 256, + 256, with the padding rows zero, so tile loads never need bounds
// checks.
#include "kmg_internal.h"

#include <type_traits>

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
// K[r][c] = sum_b F[r][b] F[c][b] over a 256 x 256 output tile per workgroup: 8 waves in a
// 2 x 4 grid, each 128 x 64 = 4 x 2 v_mfma_i32_32x32x32_i8 tiles (128 accumulator
// registers).  The reduction runs over BK-byte stages of F, double buffered in LDS and
// filled by LDS-DMA (global_load_lds_dwordx4, no staging registers or ds_write; the next
// stage's DMA is in flight while this stage multiplies; MM k=7 N=20000 3.17 -> 2.77 ms,
// k=6 0.89 -> 0.79, SP k=5 0.36 -> 0.34 with HALF; profiles/r02bk_dense_glds_ab.jsonl).
// The 16-byte chunk c of row r sits at slot c ^ swz_x(r), so the fragment reads of 16
// consecutive rows hit 16 distinct bank quads; the DMA writes lane-linearly, so each lane
// fetches the chunk its slot holds.
//
// Both operands are rows of F, so A and B fragments are loaded by the same code:
// whatever order the instruction sums its 32 k-values in, A and B use the same lane/
// element -> k map, and the tile is the full dot product.  Output map (gfx950, every
// dtype): col = lane & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5).
//
// SYM (full square K): only tiles tm <= tn are computed (half the MFMA work and half the
// F panel traffic); an off-diagonal tile is written twice, directly and transposed (K is
// symmetric and the fused normalisation K_ij / (d_i * d_j) is too, bit for bit).
// Epilogue: each wave stages one 32 x 32 sub-tile at a time in LDS and writes rows (and,
// for SYM, columns) of it with 16-byte non-temporal stores.
//
// HALF (dp <= 1024): the 256 x 256 tile is split over two 4-wave workgroups, each 256 x 128
// (2 x 2 waves of the same 128 x 64), BK = 64 only (48 KB of LDS per workgroup).  The 8-wave
// form keeps one workgroup per CU (128 accumulators + staging = 2 waves per SIMD), so a CU's
// k loop and its epilogue stores run one after the other; with two 4-wave workgroups per
// CU one can store while the other multiplies (the store phase is as long as the k loop:
// 512 KB of a SYM off-diagonal tile at a CU's 1/256 share of HBM ~ 17 us, the tile's int8
// MFMA work ~ 7 us at peak).
constexpr int DT_BM = 256;
constexpr int DT_EPI = 8 * 1024;                  // LDS bytes per wave for the epilogue (32 x 32 x 8 B)
// BK = bytes of F per stage: 64 (32 KB of A + B per stage) or 128 (64 KB, half the
// barriers per k; dp >= 1024)
// (a 3- / 4-stage ring of 64-byte stages measured no faster: the k loop is not bound by the
// DMA latency, profiles/r05aa_dense.jsonl)
template <int BK, bool HALF = false>
constexpr int dt_lds() {
  constexpr int nw = HALF ? 4 : 8, stage = (DT_BM + (HALF ? DT_BM / 2 : DT_BM)) * BK;
  return nw * DT_EPI > 2 * stage ? nw * DT_EPI : 2 * stage;
}

// 16-byte chunk c16 of row `row` in a stage: XOR-swizzled so the fragment reads of 16
// consecutive rows at one chunk cover all 64 banks (BK = 64: 4 rows per 256 B, BK = 128: 2)
template <int BK>
__device__ __forceinline__ int swz(int row, int c16) {
  if constexpr (BK == 64)
    return row * BK + ((c16 ^ ((row >> 2) & 3)) << 4);
  else
    return row * BK + ((c16 ^ ((row >> 1) & 7)) << 4);
}

// the XOR that swz<BK> applies to row `row`'s chunk index
template <int BK>
__device__ __forceinline__ int swz_x(int row) {
  return BK == 64 ? (row >> 2) & 3 : (row >> 1) & 7;
}

typedef __attribute__((address_space(3))) void lds_void;

template <typename T>
__device__ __forceinline__ void store16(T *p, const T (&v)[16 / sizeof(T)]) {
  typedef int v4i_t __attribute__((ext_vector_type(4)));
  v4i_t x;
  __builtin_memcpy(&x, v, 16);
  __builtin_nontemporal_store(x, (v4i_t *)p);
}

template <int DT, bool SYM, int DT_BK, bool HALF>
__global__ __launch_bounds__(HALF ? 256 : 512) __attribute__((amdgpu_waves_per_eu(HALF ? 2 : 1, 2))) void gram_dense_kernel(const int8_t *__restrict__ F, int dp,
                                                            int64_t n, int64_t row0, int64_t rows,
                                                            int tiles_m, int tiles_n, int64_t ntiles,
                                                            const uint32_t *__restrict__ order,
                                                            OutSpec o) {
  using T = typename std::conditional<DT == KMG_F64, double,
                                      typename std::conditional<DT == KMG_F32, float, int32_t>::type>::type;
  extern __shared__ __align__(16) uint8_t lds[];
  const int64_t per_xcd = ((int64_t)gridDim.x + 7) >> 3;
  const int64_t wlogical = (int64_t)(blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (wlogical >= (HALF ? 2 * ntiles : ntiles)) return;
  const int64_t logical = HALF ? wlogical >> 1 : wlogical;  // both halves of a tile: one XCD
  int tm, tn;
  if (order) {  // host-built super-block order (dense_tile_order, kmg_api.cpp)
    const uint32_t t = order[logical];
    tm = (int)(t & 0xFFFFu);
    tn = (int)(t >> 16);
  } else if constexpr (SYM) {  // row-band-major over tm <= tn: band tm holds tiles_n - tm tiles
    const double Tn = (double)tiles_n;
    int64_t t = (int64_t)((2.0 * Tn + 1.0 - sqrt((2.0 * Tn + 1.0) * (2.0 * Tn + 1.0) - 8.0 * (double)logical)) * 0.5);
    auto cum = [&](int64_t b) { return b * tiles_n - b * (b - 1) / 2; };
    while (t > 0 && cum(t) > logical) --t;
    while (cum(t + 1) <= logical) ++t;
    tm = (int)t;
    tn = (int)(tm + (logical - cum(t)));
  } else {
    tm = (int)(logical / tiles_n);
    tn = (int)(logical - (int64_t)tm * tiles_n);
  }
  const int64_t rbase = row0 + (int64_t)tm * DT_BM;
  constexpr int BN = HALF ? DT_BM / 2 : DT_BM;  // columns of this workgroup's part
  const int64_t cbase = (int64_t)tn * DT_BM + (HALF ? (wlogical & 1) * BN : 0);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = HALF ? wave >> 1 : wave >> 2, wn = HALF ? wave & 1 : wave & 3;

  constexpr int NT = HALF ? 256 : 512;
  constexpr int CPR = DT_BK / 16;          // 16-byte chunks per row and stage
  constexpr int DT_STAGE = (DT_BM + BN) * DT_BK;

  v16i acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (v16i){};

  const int fr = lane & 31, fh = lane >> 5;
  // one k-stage: DT_BK / 32 steps of 8 MFMAs; the fragments of step s + 1 are read from LDS
  // while step s multiplies (two fragment sets: without them every 4 MFMAs waited for the
  // reads issued just before, and the MFMA pipes stood ~70 % idle)
  auto mfma_stage = [&](const uint8_t *sA) {
    const uint8_t *sB = sA + DT_BM * DT_BK;
    constexpr int NSTEP = DT_BK / 32;
    v4i a[2][4], b[2][2];
    auto frag = [&](int s, int set) {
      const int c16 = 2 * s + fh;
#pragma unroll
      for (int x = 0; x < 4; ++x) a[set][x] = *(const v4i *)(sA + swz<DT_BK>(wm * 128 + x * 32 + fr, c16));
#pragma unroll
      for (int y = 0; y < 2; ++y) b[set][y] = *(const v4i *)(sB + swz<DT_BK>(wn * 64 + y * 32 + fr, c16));
    };
    frag(0, 0);
#pragma unroll
    for (int s = 0; s < NSTEP; ++s) {
      if (s + 1 < NSTEP) frag(s + 1, (s + 1) & 1);
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[s & 1][x], b[s & 1][y], acc[x][y], 0, 0, 0);
    }
    // schedule: step 0's 6 reads, then each step's 8 MFMAs with the next step's 6 reads
    // interleaved one by one (masks: 0x100 LDS read, 0x008 MFMA)
    __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
    for (int s = 0; s + 1 < NSTEP; ++s) {
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
  };
  {
    // LDS-DMA staging (global_load_lds_dwordx4): one wave-instruction fills 1 KB of the
    // stage linearly (RPI rows), so the swizzle moves to the source: LDS slot s of row r
    // holds chunk s ^ swz_x(r), the chunk swz<BK> put there.
    constexpr int RPI = 1024 / DT_BK, NW = NT / 64;
    constexpr int NIA = DT_BM / RPI / NW, NIB = BN / RPI / NW;
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int lrow = lane / CPR, slot = lane % CPR;
    const int8_t *srcA[NIA], *srcB[NIB];
#pragma unroll
    for (int q = 0; q < NIA; ++q) {
      const int row = (wv * NIA + q) * RPI + lrow;
      srcA[q] = F + (rbase + row) * (int64_t)dp + ((slot ^ swz_x<DT_BK>(row)) << 4);
    }
#pragma unroll
    for (int q = 0; q < NIB; ++q) {
      const int row = (wv * NIB + q) * RPI + lrow;
      srcB[q] = F + (cbase + row) * (int64_t)dp + ((slot ^ swz_x<DT_BK>(row)) << 4);
    }
    auto issue = [&](uint8_t *dst, int k0) {
#pragma unroll
      for (int q = 0; q < NIA; ++q)
        __builtin_amdgcn_global_load_lds((const void *)(srcA[q] + k0),
                                         (lds_void *)(dst + (wv * NIA + q) * 1024), 16, 0, 0);
#pragma unroll
      for (int q = 0; q < NIB; ++q)
        __builtin_amdgcn_global_load_lds((const void *)(srcB[q] + k0),
                                         (lds_void *)(dst + DT_BM * DT_BK + (wv * NIB + q) * 1024),
                                         16, 0, 0);
    };
    const int nst = dp / DT_BK;
    issue(lds, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's DMA has landed
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      const int buf = st & 1;
      const bool more = st + 1 < nst;
      if (more) issue(lds + (buf ^ 1) * DT_STAGE, (st + 1) * DT_BK);  // read in stage st-1
      mfma_stage(lds + buf * DT_STAGE);
      if (more) {
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
      }
    }
  }
  __syncthreads();  // staging buffers are reused by the epilogue

  const bool norm = DT != KMG_I32 && o.normalize && o.diagv[0] != 1.0;
  const int64_t rend = row0 + rows;

  // 32 x 32 sub-tile, row r's column c at r * 32 + ecol(r, c): the XOR keeps every 16-B
  // group of V columns together (row reads stay ds_read_b128) and spreads the column
  // reads of the mirror over all banks (4-way conflicts with a padded pitch instead)
  constexpr int PITCH = 32;
  constexpr int V = 16 / (int)sizeof(T);                                       // per 16 B
  auto ecol = [](int r, int c) {
    return sizeof(T) == 8 ? c ^ (2 * ((r >> 1) & 15)) : c ^ (4 * ((r >> 2) & 7));
  };
  T *tile = (T *)(lds + wave * DT_EPI);
  const bool mirror = SYM && tm != tn;
  const bool vec_ok = ((o.ld * (int64_t)sizeof(T)) & 15) == 0 && (((uintptr_t)o.out) & 15) == 0;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int64_t gr0 = rbase + wm * 128 + x * 32, gc0 = cbase + wn * 64 + y * 32;
      if (gr0 >= rend || gc0 >= n) continue;  // wave-uniform
      // the raw counts into the LDS sub-tile (exact in T: counts < 2^24)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = (g & 3) + 8 * (g >> 2) + 4 * fh;
        tile[r * PITCH + ecol(r, fr)] = (T)acc[x][y][g];
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's tile is in LDS
      __builtin_amdgcn_wave_barrier();
      // rows of the sub-tile: 32 rows x (32 / V) chunks of 16 B; normalize_K here, V
      // columns of one row a lane, the division unconditional (no branch around it: the
      // per-element branches of the bounded form were ~2x the epilogue's VALU), one
      // iteration at a time (16 divisions in flight spilled)
      constexpr int CPR = 32 / V;
      const int c4l = (lane % CPR) * V;  // the lane's columns: the same in every iteration
      double dcv[V];
#pragma unroll
      for (int q = 0; q < V; ++q) dcv[q] = norm ? o.dsq[min(gc0 + c4l + q, n - 1)] : 1.0;
#pragma unroll 2
      for (int it = 0; it < (32 * CPR) / 64; ++it) {
        const int ch = lane + 64 * it;
        const int r = ch / CPR, c4 = c4l;
        const int64_t gr = gr0 + r, gc = gc0 + c4;
        if (gr >= rend) continue;
        T v[V];
#pragma unroll
        for (int q = 0; q < V; ++q) v[q] = tile[r * PITCH + ecol(r, c4) + q];
        if constexpr (DT != KMG_I32) {
          if (norm) {
            const double dr = o.dsq[gr];
#pragma unroll
            for (int q = 0; q < V; ++q) {
              const double qv = (double)v[q] / (dr * dcv[q]);
              v[q] = (T)((gr == gc + q) ? 1.0 : qv);
            }
            if (mirror) {  // the mirror below reads the normalised values
#pragma unroll
              for (int q = 0; q < V; ++q) tile[r * PITCH + ecol(r, c4) + q] = v[q];
            }
          }
        }
        T *dst = (T *)o.out + (gr - row0) * o.ld + gc;
        if (vec_ok && gc + V <= n) {
          store16(dst, v);
        } else {
#pragma unroll
          for (int q = 0; q < V; ++q)
            if (gc + q < n) dst[q] = v[q];
        }
      }
      if (mirror) {  // K[gc][gr] = K[gr][gc]: output row c of the sub-tile is column c
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the normalised rows are in LDS
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < (32 * CPR) / 64; ++it) {
          const int ch = lane + 64 * it;
          const int c = ch / CPR, r4 = (ch - c * CPR) * V;
          const int64_t orow = gc0 + c, ocol = gr0 + r4;
          if (orow >= n) continue;
          T v[V];
#pragma unroll
          for (int q = 0; q < V; ++q) v[q] = tile[(r4 + q) * PITCH + ecol(r4 + q, c)];
          T *dst = (T *)o.out + orow * o.ld + ocol;
          if (vec_ok && ocol + V <= rend) {
            store16(dst, v);
          } else {
#pragma unroll
            for (int q = 0; q < V; ++q)
              if (ocol + q < rend) dst[q] = v[q];
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();  // the next sub-tile overwrites this wave's region
    }
  }
}

hipError_t launch_dense_features(const uint8_t *codes, const int32_t *lens, int64_t ldc, int64_t n,
                                 int k, int window, int dp, const uint32_t *masks, int nmask,
                                 int8_t *F, double *diagv, double *dsq, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if ((dp & 127) || dp > 65536) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dense_feat_kernel, dim3((unsigned)n), dim3(256), (size_t)dp, s, codes, lens,
                     ldc, k, window, dp, masks, nmask, F, diagv, dsq);
  return hipGetLastError();
}

// ------------------------------------------------------------------ fp32 GEMM form
// BASELINE configs[3]'s literal formulation ("count-vector fp32 GEMM"): the int8 count
// rows widened to fp32 for rocblas_sgemm (KMG_ALGO=3), and the fp32 K written out in the
// call's dtype with the fused normalize_K formula.  Every count product and partial sum
// is an integer below 2^24 (spectrum k=8 at L=101: K <= 94^2), so the fp32 K is exact.
__global__ __launch_bounds__(256) void i8_to_f32_kernel(const int8_t *__restrict__ F, int64_t n,
                                                        float *__restrict__ G) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t * 4 >= n) return;
  const uint32_t v = ((const uint32_t *)F)[t];
  ((float4 *)G)[t] = make_float4((float)(int8_t)(v & 0xFF), (float)(int8_t)((v >> 8) & 0xFF),
                                 (float)(int8_t)((v >> 16) & 0xFF), (float)(int8_t)(v >> 24));
}

__global__ __launch_bounds__(256) void f32_gram_out_kernel(const float *__restrict__ K32,
                                                           int64_t n, int64_t row0, OutSpec o) {
  const int64_t il = blockIdx.y;
  const int64_t i = row0 + il;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const double raw = (double)K32[i * n + j];
  double v = raw;
  if (o.normalize && o.diagv[0] != 1.0) v = (i == j) ? 1.0 : raw / (o.dsq[i] * o.dsq[j]);
  if (o.dtype == KMG_F64)
    ((double *)o.out)[il * o.ld + j] = v;
  else if (o.dtype == KMG_F32)
    ((float *)o.out)[il * o.ld + j] = (float)v;
  else
    ((int32_t *)o.out)[il * o.ld + j] = (int32_t)raw;
}

hipError_t launch_i8_to_f32(const int8_t *F, int64_t elems, float *G, hipStream_t s) {
  if (elems <= 0) return hipSuccess;
  if (elems & 3) return hipErrorInvalidValue;
  const int64_t t = elems / 4;
  hipLaunchKernelGGL(i8_to_f32_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, s, F, elems,
                     G);
  return hipGetLastError();
}

hipError_t launch_f32_gram_out(const float *K32, int64_t n, int64_t row0, int64_t row1,
                               const OutSpec &o, hipStream_t s) {
  for (int64_t r = row0; r < row1; r += 65535) {  // grid.y <= 65535 rows a launch
    const int64_t rows = std::min<int64_t>(65535, row1 - r);
    if (n == 0) break;
    OutSpec os = o;
    os.out = (char *)o.out + (size_t)(r - row0) * o.ld * (o.dtype == KMG_F64 ? 8 : 4);
    hipLaunchKernelGGL(f32_gram_out_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)rows),
                       dim3(256), 0, s, K32, n, r, os);
  }
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
                             const uint32_t *order, const OutSpec &o, hipStream_t s, int bk,
                             bool half) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || n <= 0) return hipSuccess;
  if (bk != 128 || (dp & 127) || half) bk = 64;
  if (dp & 63) return hipErrorInvalidValue;
  const bool sym = row0 == 0 && rows == n;
  const int tiles_m = (int)((rows + DT_BM - 1) / DT_BM);
  const int tiles_n = (int)((n + DT_BM - 1) / DT_BM);
  const int64_t total = sym ? (int64_t)tiles_n * (tiles_n + 1) / 2 : (int64_t)tiles_m * tiles_n;
  if (total > 0x7FFFFFF0LL) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)(((half ? 2 * total : total) + 7) & ~7LL);
#define KMG_DENSE_GO(DTV, SY, BKV, HV)                                                          \
  hipLaunchKernelGGL((gram_dense_kernel<DTV, SY, BKV, HV>), dim3(grid), dim3(HV ? 256 : 512),      \
                     (dt_lds<BKV, HV>()), s, F, dp, n, row0, rows, tiles_m, tiles_n, total, order, o)
#define KMG_DENSE(DTV, SY)                                                      \
  do {                                                                          \
    if (half) KMG_DENSE_GO(DTV, SY, 64, true);                                  \
    else if (bk == 128) KMG_DENSE_GO(DTV, SY, 128, false);                      \
    else KMG_DENSE_GO(DTV, SY, 64, false);                                      \
  } while (0)
  switch (o.dtype) {
    case KMG_I32:
      if (sym) KMG_DENSE(KMG_I32, true); else KMG_DENSE(KMG_I32, false);
      break;
    case KMG_F32:
      if (sym) KMG_DENSE(KMG_F32, true); else KMG_DENSE(KMG_F32, false);
      break;
    default:
      if (sym) KMG_DENSE(KMG_F64, true); else KMG_DENSE(KMG_F64, false);
      break;
  }
#undef KMG_DENSE
#undef KMG_DENSE_GO
  return hipGetLastError();
}

}  // namespace kmg
