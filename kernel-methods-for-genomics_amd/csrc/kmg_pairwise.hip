// kmg_pairwise.hip — per-pair Gram kernels (float64) for gfx950.
//
// Reference functions restated on the device, with the reference's floating-point
// operation order kept exactly (the library is built with -ffp-contract=off and the
// explicit __dmul_rn/__dadd_rn below so no FMA contraction changes a rounding):
//   get_WD_K / get_WD_d / beta            kernels.py:53-101
//   get_WDShifts_K / get_WDShifts_d / delta kernels.py:106-155
//   get_string_K / K_k / B_k              kernels.py:308-382
//   get_gappy_K (k=1, g=0)                kernels.py:420-455
// plus the dense host-matrix helpers normalize_K (kernels.py:398-415) and
// center_K (kernels.py:387-395).
#include "kmg_internal.h"
#include <type_traits>

#include <cmath>

namespace kmg {

struct Coef {
  double a[KMG_MAX_COEF];
  double b[KMG_MAX_COEF];
};

// exact per-byte equality flags of two 4-symbol words -> 4 bits (bit q = byte q equal)
__device__ __forceinline__ uint32_t eq4(uint32_t x, uint32_t y) {
  const uint32_t v = x ^ y;
  uint32_t t = (v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  t = ~(t | v | 0x7F7F7F7Fu);  // high bit of each zero byte
  return ((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u);
}

template <int NW>
__device__ __forceinline__ void range_mask(uint64_t (&m)[NW], int lo, int hi_excl) {
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int b0 = w * 64;
    const int a = max(lo - b0, 0), b = min(hi_excl - b0, 64);
    if (b <= a) {
      m[w] = 0;
    } else {
      const uint64_t hi = (b >= 64) ? ~0ull : ((1ull << b) - 1ull);
      const uint64_t lom = (a >= 64) ? ~0ull : ((1ull << a) - 1ull);
      m[w] = hi & ~lom;
    }
  }
}

// r = m >> sh (bit l of r = bit l+sh of m), 0 <= sh < 64*NW
template <int NW>
__device__ __forceinline__ void shr_bits(const uint64_t (&m)[NW], int sh, uint64_t (&r)[NW]) {
  const int ws = sh >> 6, bs = sh & 63;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    uint64_t lo = 0, hi = 0;
#pragma unroll
    for (int u = 0; u < NW; ++u) {
      if (u == w + ws) lo = m[u];
      if (u == w + ws + 1) hi = m[u];
    }
    r[w] = bs ? ((lo >> bs) | (hi << (64 - bs))) : lo;
  }
}

// symbol rows staged in LDS as words of 4 bytes, padded with 0xFF
template <int NW>
struct SeqTile {
  static constexpr int WORDS = 16 * NW + 8;  // + room for shifted reads
};

template <int NW>
__device__ __forceinline__ void stage_seq(uint32_t *dst, const SeqSpec &q, int64_t j) {
  // one wave loads one sequence: lane l writes word l, l+64, ...
  const int lane = threadIdx.x & 63;
  const int L = (j < q.n) ? q.lens[j] : 0;
  const uint8_t *src = q.codes + (j < q.n ? j : 0) * q.ldc;
  for (int w = lane; w < SeqTile<NW>::WORDS; w += 64) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int pos = 4 * w + b;
      const uint32_t c = (pos < L) ? src[pos] : 0xFFu;
      v |= c << (8 * b);
    }
    dst[w] = v;
  }
}

// match mask M[l] = [x_{l+sx} == y_{l+sy}] for l with l+sx < Lx and l+sy < Ly
template <int NW>
__device__ __forceinline__ void match_mask(const uint32_t *xs, int Lx, int sx, const uint32_t *ys,
                                           int Ly, int sy, uint64_t (&M)[NW]) {
#pragma unroll
  for (int w = 0; w < NW; ++w) M[w] = 0;
  const int qx = sx >> 2, rx = sx & 3, qy = sy >> 2, ry = sy & 3;
#pragma unroll
  for (int w = 0; w < 16 * NW; ++w) {
    const uint32_t xw = __builtin_amdgcn_alignbyte(xs[w + qx + 1], xs[w + qx], rx);
    const uint32_t yw = __builtin_amdgcn_alignbyte(ys[w + qy + 1], ys[w + qy], ry);
    M[w >> 4] |= (uint64_t)eq4(xw, yw) << (4 * (w & 15));
  }
  uint64_t lim[NW];
  range_mask<NW>(lim, 0, min(Lx - sx, Ly - sy));
#pragma unroll
  for (int w = 0; w < NW; ++w) M[w] &= lim[w];
}

template <int NW>
__device__ __forceinline__ int popc_and(const uint64_t (&a)[NW], const uint64_t (&b)[NW]) {
  int c = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) c += __popcll(a[w] & b[w]);
  return c;
}

__device__ __forceinline__ void store_f(const OutSpec &o, int64_t il, int64_t j, double v) {
  if (o.dtype == KMG_F64)
    ((double *)o.out)[il * o.ld + j] = v;
  else if (o.dtype == KMG_F32)
    ((float *)o.out)[il * o.ld + j] = (float)v;
  else
    ((int32_t *)o.out)[il * o.ld + j] = (int32_t)v;
}

// ------------------------------------------------------------------ WD
// K[i,j] (i<j) = sum_{k=1..d} beta_k * #{l in [1, L-k] : x[l:l+k] == y[l:l+k]},
// L = len(x_i) of the smaller index (kernels.py:64-81, 94-100); diagonal =
// L-1+(1-d)/3 (kernels.py:96).  Tile: 16 rows x 64 columns, 256 threads.
template <int NW>
__global__ __launch_bounds__(256) void gram_wd_kernel(SeqSpec q, int64_t row0, int64_t row1, int d,
                                                      int span, Coef cf, OutSpec o) {
  constexpr int WS = SeqTile<NW>::WORDS;
  __shared__ uint32_t srow[16][WS];
  __shared__ uint32_t scol[64][WS];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t rbase = row0 + (int64_t)blockIdx.y * 16;
  const int64_t cbase = (int64_t)blockIdx.x * 64;
  for (int r = wave; r < 16; r += 4) stage_seq<NW>(srow[r], q, rbase + r);
  for (int c = wave; c < 64; c += 4) stage_seq<NW>(scol[c], q, cbase + c);
  __syncthreads();
  const int64_t j = cbase + lane;
  if (j >= q.n) return;
  for (int r = wave; r < 16; r += 4) {
    const int64_t i = rbase + r;
    if (i >= row1) break;
    double val;
    if (i == j) {
      const int L = q.lens[i];
      val = __dadd_rn((double)(L - 1), (double)(1 - d) / 3.0);
    } else {
      const bool rowx = i < j;
      const uint32_t *xs = rowx ? srow[r] : scol[lane];
      const uint32_t *ys = rowx ? scol[lane] : srow[r];
      const int Lx = q.lens[rowx ? i : j], Ly = q.lens[rowx ? j : i];
      uint64_t M[NW], A[NW], Ms[NW], V[NW];
      const int Lr = span > 0 ? span : Lx;  // summation length L (get_WD_d's argument)
      match_mask<NW>(xs, Lx, 0, ys, Ly, 0, M);
#pragma unroll
      for (int w = 0; w < NW; ++w) { A[w] = M[w]; Ms[w] = M[w]; }
      val = 0.0;  // c_t = 0 (int); 0 + x is exact
      for (int k = 1; k <= d; ++k) {
        if (k > 1) {
          // Ms = M >> (k-1); A_k = A_{k-1} & Ms
#pragma unroll
          for (int w = 0; w < NW; ++w) {
            const uint64_t nxt = (w + 1 < NW) ? Ms[w + 1] : 0ull;
            Ms[w] = (Ms[w] >> 1) | (nxt << 63);
            A[w] &= Ms[w];
          }
        }
        range_mask<NW>(V, 1, Lr - k + 1);
        const int c = popc_and<NW>(A, V);
        val = __dadd_rn(val, __dmul_rn(cf.a[k - 1], (double)c));
      }
    }
    store_f(o, i - row0, j, val);
  }
}

// WD on the packed records, as bit planes.  Staging turns a record's 2-bit codes (symbol q
// of code word w at bits [30-2q, 31-2q]) into two planes of one bit per position —
// position l at bit 31 - l%32 of word l/32, plane 1 the high code bits, plane 0 the low —
// so the match mask of a pair is M_w = keep_w & ~((x1 ^ y1) | (x0 ^ y0)), one bit a
// position and position l+1 one bit below l.  keep_w holds the positions [1, min(Lx, Ly,
// L)) (kernels.py:78: l >= 1; a slice clipped by either end never equals a full one, and
// the range is symmetric in i, j).  Then A_1 = M, A_k = A_{k-1} & (A_{k-1} << 1) (one
// funnel shift a word) and c_k = popc(A_k) = #{l in [1, L-k] : x[l:l+k] == y[l:l+k]}
// (kernels.py:64-81); val accumulates beta_k * c_k in k order.  The k loop ends when no
// lane of the wave has a run left: a skipped beta_k * 0 adds +0.0 (no rounding change).
// Half the words of the 2-bit form per pair (4 against 7 at L = 101): 1.8x fewer VALU
// operations in the mask and k loop.  A pair holding a non-ACGT symbol (mask bit below
// len) is compared byte by byte from the codes (rare; exact for any alphabet).  Tile: 64
// columns (one per lane, planes in VGPRs) x 64 rows (16 per wave, planes read
// wave-uniform from LDS, four rows a pass so a lane runs four independent chains).  MIRROR (full square K): only tiles J >= I run; an off-diagonal
// tile also writes its transpose from an LDS copy, 64 coalesced 512-B rows.
__device__ __forceinline__ uint32_t wd_keep(int lim, int w) {
  const int nv = min(max(lim - 32 * w, 0), 32);
  return nv == 0 ? 0u : (0xFFFFFFFFu << (32 - nv));
}

__device__ __forceinline__ bool wd_has_other(const uint32_t *rec, int cw, int len) {
  bool bad = false;
  for (int w = 0; 32 * w < len; ++w) {
    const int nv = min(len - 32 * w, 32);
    const uint32_t below = nv >= 32 ? 0xFFFFFFFFu : ((1u << nv) - 1u);
    bad |= (rec[cw + w] & below) != 0u;
  }
  return bad;
}

// the even bits of x (bit 2i -> bit i): 16 bits in symbol order, first symbol highest
__device__ __forceinline__ uint32_t even_bits(uint32_t x) {
  x &= 0x55555555u;
  x = (x | (x >> 1)) & 0x33333333u;
  x = (x | (x >> 2)) & 0x0F0F0F0Fu;
  x = (x | (x >> 4)) & 0x00FF00FFu;
  return (x | (x >> 8)) & 0x0000FFFFu;
}

// planes of a record: dst[p] (high code bits) and dst[NP + p] (low) for p < NP
template <int NP>
__device__ __forceinline__ void wd_planes(const uint32_t *rec, int cw, uint32_t *dst) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const uint32_t w0 = 2 * p < cw ? rec[2 * p] : 0u, w1 = 2 * p + 1 < cw ? rec[2 * p + 1] : 0u;
    dst[p] = (even_bits(w0 >> 1) << 16) | even_bits(w1 >> 1);
    dst[NP + p] = (even_bits(w0) << 16) | even_bits(w1);
  }
}

template <int NP>
__device__ __forceinline__ void wd_mask_bytes(const SeqSpec &q, int64_t a, int64_t b, int lim,
                                              uint32_t (&M)[NP]) {
  const uint8_t *xa = q.codes + a * q.ldc, *yb = q.codes + b * q.ldc;
#pragma unroll
  for (int w = 0; w < NP; ++w) {
    uint32_t m = 0;
    for (int t = 0; t < 32; ++t) {
      const int pos = 32 * w + t;
      if (pos >= 1 && pos < lim && xa[pos] == yb[pos]) m |= 1u << (31 - t);
    }
    M[w] = m;
  }
}

template <int NP, bool MIRROR>
__global__ __launch_bounds__(256) void gram_wdp_kernel(SeqSpec q, Packed pk, int64_t row0,
                                                       int64_t row1, int d, int span, Coef cf,
                                                       OutSpec o) {
  constexpr int RB = 64;
  constexpr int SW = (2 * NP) | 1;  // odd word stride: the column reads are bank-conflict free
  __shared__ double tile[MIRROR ? RB : 1][MIRROR ? 65 : 1];
  __shared__ uint32_t srow[RB][SW], scol[64][SW];
  __shared__ int slen[RB];  // row length, -1 - length if the row holds a non-ACGT symbol
  if (MIRROR && blockIdx.x < blockIdx.y) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t rbase = row0 + (int64_t)blockIdx.y * RB;
  const int64_t cbase = (int64_t)blockIdx.x * 64;
  int Ly = 0;
  bool cbad = false;
  if (wave < 2) {  // wave 0 stages the rows, wave 1 the columns
    const int64_t t = (wave == 0 ? rbase : cbase) + lane;
    const int64_t lim = wave == 0 ? row1 : q.n;
    uint32_t(*dst)[SW] = wave == 0 ? srow : scol;
    int len = 0;
    bool bad = false;
    if (t < lim) {
      const uint32_t *rec = pk.w + t * pk.ldp;
      wd_planes<NP>(rec, pk.cw, dst[lane]);
      len = q.lens[t];
      bad = wd_has_other(rec, pk.cw, len);
    } else {
#pragma unroll
      for (int w = 0; w < 2 * NP; ++w) dst[lane][w] = 0u;
    }
    if (wave == 0) slen[lane] = bad ? -1 - len : len;
  }
  __syncthreads();
  const int64_t j = cbase + lane;
  const bool jin = j < q.n;
  const int64_t jj = jin ? j : 0;
  Ly = q.lens[jj];
  cbad = wd_has_other(pk.w + jj * pk.ldp, pk.cw, Ly);
  uint32_t y1[NP], y0[NP], ky[NP];
  const int Lyc = span > 0 ? min(Ly, span) : Ly;
#pragma unroll
  for (int w = 0; w < NP; ++w) {
    y1[w] = scol[lane][w];
    y0[w] = scol[lane][NP + w];
    ky[w] = wd_keep(Lyc, w);
  }
  ky[0] &= 0x7FFFFFFFu;  // l >= 1
  const bool diag_tile = MIRROR && blockIdx.x == blockIdx.y;
  // match mask of (row r, this lane's column): A[w] (A_1 of the k recursion)
  auto row_mask = [&](int r, int64_t i, uint32_t (&A)[NP]) {
    const int sl = __builtin_amdgcn_readfirstlane(slen[r]);
    const bool rbad = sl < 0;
    const int Lx = rbad ? -1 - sl : sl;
    if (rbad || cbad) {
      const int lim = span > 0 ? min(min(Lx, Ly), span) : min(Lx, Ly);
      wd_mask_bytes<NP>(q, i, jj, lim, A);
    } else {
#pragma unroll
      for (int w = 0; w < NP; ++w) {
        const uint32_t kx = wd_keep(Lx, w);
        const uint32_t v = (srow[r][w] ^ y1[w]) | (srow[r][NP + w] ^ y0[w]);
        A[w] = (kx & ky[w]) & ~v;
      }
    }
    return Lx;
  };
  {
    // RP rows (r, r + 4, ...) per pass: RP independent shift / popcount / fp64 chains a lane
    // (one row a pass: N=9000 d=4/5/10 0.221/0.234/0.270 -> 0.190/0.204/0.239 ms;
    // profiles/r02bp_wd_rows_per_pass_ab.jsonl)
    constexpr int RP = 4;
    for (int r = wave; r < RB; r += 4 * RP) {
      if (rbase + r >= row1) break;
      uint32_t A[RP][NP];
      int Lx[RP];
      double val[RP];
#pragma unroll
      for (int u = 0; u < RP; ++u) {
        const int64_t i = rbase + r + 4 * u;
        val[u] = 0.0;
        Lx[u] = 0;
        if (i < row1) {
          Lx[u] = row_mask(r + 4 * u, i, A[u]);
        } else {
#pragma unroll
          for (int w = 0; w < NP; ++w) A[u][w] = 0u;
        }
      }
      for (int k = 1; k <= d; ++k) {
        int c[RP], any = 0;
#pragma unroll
        for (int u = 0; u < RP; ++u) {
          c[u] = 0;
#pragma unroll
          for (int w = 0; w < NP; ++w) c[u] += __popc(A[u][w]);
          any |= c[u];
        }
        if (!__any(any != 0)) break;
        // a zero count adds +0.0: no rounding change
#pragma unroll
        for (int u = 0; u < RP; ++u) val[u] = __dadd_rn(val[u], __dmul_rn(cf.a[k - 1], (double)c[u]));
#pragma unroll
        for (int u = 0; u < RP; ++u)
#pragma unroll
          for (int w = 0; w < NP; ++w) {
            const uint32_t nxt = (w + 1 < NP) ? A[u][w + 1] : 0u;
            A[u][w] &= __builtin_amdgcn_alignbit(A[u][w], nxt, 31);  // (A_w << 1) | (A_{w+1} >> 31)
          }
      }
#pragma unroll
      for (int u = 0; u < RP; ++u) {
        const int64_t i = rbase + r + 4 * u;
        if (i >= row1) break;
        if (i == j) val[u] = __dadd_rn((double)(Lx[u] - 1), (double)(1 - d) / 3.0);  // kernels.py:96
        if (jin) store_f(o, i - row0, j, val[u]);
        if (MIRROR) tile[r + 4 * u][lane] = val[u];
      }
    }
  }
  if (MIRROR && !diag_tile) {
    __syncthreads();
    // transpose: row j = J*64 + c of K gets columns I*64 + lane
    const int64_t icol = rbase + lane;
    for (int c = wave; c < 64; c += 4) {
      const int64_t jr = cbase + c;
      if (jr >= q.n) break;
      if (icol < row1) store_f(o, jr - row0, icol, tile[lane][c]);
    }
  }
}

// ------------------------------------------------------------------ WDS
// c_st = sum_{i=1}^{L-k} sum_{s=0}^{S} [s+i<L] delta_s * ([x[i+s:i+s+k]==y[i:i+k]] +
// [x[i:i+k]==y[i+s:i+s+k]]), accumulated in exactly that (i, s) order; K += beta_k*c_st
// (kernels.py:115-135).  Zero terms are skipped: adding +0.0 never changes an fp64 sum.
template <int NW, int SMAX>
__global__ __launch_bounds__(256) void gram_wds_kernel(SeqSpec q, int64_t row0, int64_t row1, int d,
                                                       int S, int span, Coef cf, OutSpec o) {
  constexpr int WS = SeqTile<NW>::WORDS;
  __shared__ uint32_t srow[16][WS];
  __shared__ uint32_t scol[64][WS];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t rbase = row0 + (int64_t)blockIdx.y * 16;
  const int64_t cbase = (int64_t)blockIdx.x * 64;
  for (int r = wave; r < 16; r += 4) stage_seq<NW>(srow[r], q, rbase + r);
  for (int c = wave; c < 64; c += 4) stage_seq<NW>(scol[c], q, cbase + c);
  __syncthreads();
  const int64_t j = cbase + lane;
  if (j >= q.n) return;
  for (int r = wave; r < 16; r += 4) {
    const int64_t i = rbase + r;
    if (i >= row1) break;
    const bool rowx = i <= j;
    const uint32_t *xs = rowx ? srow[r] : scol[lane];
    const uint32_t *ys = rowx ? scol[lane] : srow[r];
    const int Lx = q.lens[rowx ? i : j], Ly = q.lens[rowx ? j : i];
    const int Lr = span > 0 ? span : Lx;  // summation length L (get_WDShifts_d's argument)
    uint64_t M1[SMAX + 1][NW], M2[SMAX + 1][NW], W1[SMAX + 1][NW], W2[SMAX + 1][NW];
#pragma unroll
    for (int s = 0; s <= SMAX; ++s) {
      if (s <= S) {
        match_mask<NW>(xs, Lx, s, ys, Ly, 0, M1[s]);  // x_{i+s} == y_i
        match_mask<NW>(xs, Lx, 0, ys, Ly, s, M2[s]);  // x_i == y_{i+s}
        if (s > 0 && Lx - s == Ly) {
          // ragged rows: x[i+s:i+s+k] and y[i:i+k] are clipped to the SAME length Ly - i
          // near the end, and Python compares the clipped slices (kernels.py:133): a
          // suffix match counts.  Positions past the end of y match vacuously.
          uint64_t tail[NW];
          range_mask<NW>(tail, Ly, 64 * NW);
#pragma unroll
          for (int w = 0; w < NW; ++w) M1[s][w] |= tail[w];
        }
      } else {
#pragma unroll
        for (int w = 0; w < NW; ++w) { M1[s][w] = 0; M2[s][w] = 0; }
      }
#pragma unroll
      for (int w = 0; w < NW; ++w) { W1[s][w] = M1[s][w]; W2[s][w] = M2[s][w]; }
    }
    double val = 0.0;
    for (int k = 1; k <= d; ++k) {
      if (k > 1) {
#pragma unroll
        for (int s = 0; s <= SMAX; ++s) {
          uint64_t t1[NW], t2[NW];
          shr_bits<NW>(M1[s], k - 1, t1);
          shr_bits<NW>(M2[s], k - 1, t2);
#pragma unroll
          for (int w = 0; w < NW; ++w) { W1[s][w] &= t1[w]; W2[s][w] &= t2[w]; }
        }
      }
      uint64_t V[NW];
      range_mask<NW>(V, 1, Lr - k + 1);
      uint64_t any[NW];
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        uint64_t a = 0;
#pragma unroll
        for (int s = 0; s <= SMAX; ++s) a |= W1[s][w] | W2[s][w];
        any[w] = a & V[w];
      }
      double cst = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        uint64_t bits = any[w];
        while (bits) {
          const int b = __builtin_ctzll(bits);
          bits &= bits - 1;
          const int ii = 64 * w + b;
#pragma unroll
          for (int s = 0; s <= SMAX; ++s) {
            if (s <= S && s + ii < Lr) {
              const int m = (int)((W1[s][w] >> b) & 1ull) + (int)((W2[s][w] >> b) & 1ull);
              if (m) cst = __dadd_rn(cst, __dmul_rn(cf.b[s], (double)m));
            }
          }
        }
      }
      val = __dadd_rn(val, __dmul_rn(cf.a[k - 1], cst));
    }
    store_f(o, i - row0, j, val);
  }
}

// v from lane l - 1 (lanes 1..63; lane 0 gets 0): DPP wave_shr:1 on both halves, a VALU
// move instead of the LDS-routed ds_bpermute that __shfl_up becomes
__device__ __forceinline__ double wave_shr1(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// ------------------------------------------------------------------ SS (substring)
// One wave per pair.  Bottom-up B_t(r, j) = B_t(x[:r], y[:j]) for t = 1..k-1 over an
// anti-diagonal sweep: lane l of a 64-row strip owns row r, at step st it computes
// column j = st - l.  B_t(r,j) = ((lam*B_t(r-1,j) + lam*B_t(r,j-1)) - lam2*B_t(r-1,j-1))
// + [x_{r-1}==y_{j-1}] lam2*B_{t-1}(r-1,j-1)   (kernels.py:337-342)
// K = sum_{i=k..n} lam2 * S_i,  S_i = sum_{j: y_j == x_{i-1}} B_{k-1}(i-1, j)  (kernels.py:359-364)
template <int KMAX>
__global__ __launch_bounds__(256) void gram_ss_kernel(SeqSpec q, int64_t row0, int64_t row1, int kk,
                                                      double lam, double lam2, int mirror,
                                                      OutSpec o) {
  extern __shared__ __align__(16) double ssm[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = row0 + blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (j >= q.n || i >= row1) return;
  if (mirror && j < i) return;
  const int ML = q.maxlen;
  // per-wave LDS: rowbuf[KMAX-1][ML+1], Sbuf[ML+2], ybytes[ML+4]
  const int per = (KMAX - 1) * (ML + 1) + (ML + 2) + (ML + 4 + 7) / 8;
  double *rowbuf = ssm + (size_t)wave * per;
  double *Sbuf = rowbuf + (KMAX - 1) * (ML + 1);
  uint8_t *yb = (uint8_t *)(Sbuf + ML + 2);
  const int64_t ia = min(i, j), ib = max(i, j);
  const uint8_t *xsrc = q.codes + ia * q.ldc;
  const uint8_t *ysrc = q.codes + ib * q.ldc;
  const int nx = q.lens[ia], ny = q.lens[ib];
  double result;
  if (kk == 0) {
    result = 1.0;  // K_k(.., 0, ..) returns 1 (kernels.py:354-355)
  } else if (nx < kk || ny < kk) {
    result = 0.0;  // kernels.py:357-358
  } else {
    for (int c = lane; c < ny; c += 64) yb[c] = ysrc[c];
    for (int r = lane; r <= nx + 1; r += 64) Sbuf[r] = 0.0;
    __builtin_amdgcn_wave_barrier();
    for (int s0 = 0; s0 <= nx; s0 += 64) {
      const int r = s0 + lane;  // row = number of x symbols consumed
      const bool live = r <= nx;
      const uint32_t xprev = (r >= 1 && live) ? xsrc[r - 1] : 0x1FFu;  // x_{r-1}
      const uint32_t xcur = (r < nx) ? xsrc[r] : 0x1FFu;               // x_r (for S_{r+1})
      double last[KMAX - 1], diag[KMAX - 1];
#pragma unroll
      for (int t = 0; t < KMAX - 1; ++t) { last[t] = 0.0; diag[t] = 0.0; }
      double sacc = 0.0;
      const bool store_row = (lane == 63) && (s0 + 64 <= nx);
      for (int st = 0; st <= ny + 63; ++st) {
        const int jc = st - lane;
        const bool act = live && jc >= 0 && jc <= ny;
        double up[KMAX - 1];
#pragma unroll
        for (int t = 0; t < KMAX - 1; ++t) {
          const double fromleft = wave_shr1(last[t]);
          double u = fromleft;
          if (lane == 0) u = (s0 == 0 || jc < 0 || jc > ny) ? 0.0 : rowbuf[t * (ML + 1) + jc];
          up[t] = u;
        }
        if (act) {
          double cur[KMAX - 1];
          const bool match = (r >= 1 && jc >= 1) && (xprev == yb[jc - 1]);
#pragma unroll
          for (int t = 0; t < KMAX - 1; ++t) {
            const int lvl = t + 1;
            double v = 0.0;
            if (lvl < kk && r >= lvl && jc >= lvl && r >= 1 && jc >= 1) {
              v = __dadd_rn(__dmul_rn(lam, up[t]), __dmul_rn(lam, last[t]));
              v = __dsub_rn(v, __dmul_rn(lam2, diag[t]));
              if (match) {
                const double prevlvl = (t == 0) ? 1.0 : diag[t - 1];
                v = __dadd_rn(v, __dmul_rn(lam2, prevlvl));
              }
            }
            cur[t] = v;
          }
          if (jc < ny && r < nx && yb[jc] == xcur) {
            double bkm1 = 1.0;  // B_0 == 1
#pragma unroll
            for (int t = 0; t < KMAX - 1; ++t)
              if (t == kk - 2) bkm1 = cur[t];
            sacc = __dadd_rn(sacc, bkm1);
          }
#pragma unroll
          for (int t = 0; t < KMAX - 1; ++t) {
            diag[t] = up[t];
            last[t] = cur[t];
          }
          if (store_row) {
#pragma unroll
            for (int t = 0; t < KMAX - 1; ++t) rowbuf[t * (ML + 1) + jc] = cur[t];
          }
          if (jc == ny && r < nx) Sbuf[r + 1] = sacc;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();
    double K = 0.0;
    if (lane == 0) {
      for (int ii = kk; ii <= nx; ++ii) K = __dadd_rn(K, __dmul_rn(lam2, Sbuf[ii]));
    }
    result = K;
  }
  if (lane == 0) {
    store_f(o, i - row0, j, result);
    if (mirror && j != i && j >= row0 && j < row1) store_f(o, j - row0, i, result);
  }
}

// ------------------------------------------------------------------ SS, grouped sweep
// The same recurrences, 64 / LPP pairs a wave: lane s of a pair's LPP-lane group owns the
// DP rows r = s R .. s R + R - 1 (r = 0..n_x, row 0 the zero boundary) and at step st
// computes column c = st - s of each of its rows in row order.  Row r - 1 at column c is
// the row above in the same lane, or for the lane's first row lane s - 1's last row,
// published at step st - 1 and moved by DPP wave_shr:1 (across a group boundary it lands
// on a lane whose first row is row 0, which never reads it); the diagonal is the row
// above's previous value.  The strip kernel above ran one pair a wave in 64-row strips:
// at L = 101 two strips of ny + 64 steps each with 38 of 64 lanes live in the second, and
// KMAX - 1 >= kk - 1 levels; here ML + LPP steps of R rows and exactly NL levels per
// lane, so every lane stays busy.  Per cell the operation order is the strip kernel's
// (bit-identical), S_{r+1} accumulates in column order, K sums S_i in row order.
template <int LPP, int R, int NL>
__global__ __launch_bounds__(256) void gram_ssg_kernel(SeqSpec q, int64_t row0, int64_t row1,
                                                       int kk, double lam, double lam2,
                                                       int mirror, OutSpec o, int bmode) {
  constexpr int G = 64 / LPP;
  extern __shared__ __align__(16) double gsm[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane / LPP, s = lane % LPP;
  const int64_t i = row0 + blockIdx.y;
  const int64_t jb = (mirror ? i : 0) + ((int64_t)blockIdx.x * 4 + wave) * G;
  if (i >= row1 || jb >= q.n) return;  // wave-uniform
  const int ML = q.maxlen;
  const int SW = ML + 2;  // S slots per group
  double *Ssh = gsm + (size_t)(wave * G + g) * SW;
  uint8_t *ysh = (uint8_t *)(gsm + (size_t)4 * G * SW) + (size_t)(wave * G + g) * (ML + 1);
  const int64_t j = jb + g;
  const bool pv = j < q.n;
  const int64_t ia = pv ? min(i, j) : i, ib = pv ? max(i, j) : i;
  const uint8_t *xs = q.codes + ia * q.ldc;
  const uint8_t *ys = q.codes + ib * q.ldc;
  const int nx = pv ? q.lens[ia] : -1, ny = pv ? q.lens[ib] : -1;
  // a pair takes part in the sweep unless its value is a constant (kernels.py:354-358);
  // bmode (B_{kk-1}, levels 1..kk-1 computed, kernels.py:331-335): prefixes of >= kk-1
  const bool dp = bmode ? (pv && kk >= 2 && nx >= kk - 1 && ny >= kk - 1)
                        : (pv && kk >= 1 && nx >= kk && ny >= kk);
  double bval = 0.0;  // bmode: B_{kk-1}(x, y) at the cell (n_x, n_y), held by its row's lane
  for (int c = s; c < ny; c += LPP) ysh[c] = ys[c];
  // x_{r-1} and x_r of the lane's rows, packed 4 a word (0x1FF-like sentinel 0xFF:
  // never equal to a code of y, which the match tests compare as bytes)
  uint32_t xw[(R + 4) / 4];
#pragma unroll
  for (int w = 0; w < (R + 4) / 4; ++w) xw[w] = 0xFFFFFFFFu;
#pragma unroll
  for (int k = 0; k <= R; ++k) {  // xw byte k = x_{r0 + k - 1}
    const int rr = s * R + k - 1;
    const uint32_t v = (dp && rr >= 0 && rr < nx) ? (uint32_t)xs[rr] : 0xFFu;
    xw[k >> 2] = (xw[k >> 2] & ~(0xFFu << (8 * (k & 3)))) | (v << (8 * (k & 3)));
  }
  __builtin_amdgcn_wave_barrier();
  double last[R][NL], sacc[R], pub[NL], pup[NL];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    sacc[k] = 0.0;
#pragma unroll
    for (int t = 0; t < NL; ++t) last[k][t] = 0.0;
  }
#pragma unroll
  for (int t = 0; t < NL; ++t) {
    pub[t] = 0.0;
    pup[t] = 0.0;
  }
  const int r0 = s * R;
  const int steps = ML + LPP;
  for (int st = 0; st < steps; ++st) {
    const int c = st - s;
    double up[NL];
#pragma unroll
    for (int t = 0; t < NL; ++t) up[t] = wave_shr1(pub[t]);
    if (dp && c >= 0 && c <= ny) {
      const uint32_t yprev = c >= 1 ? (uint32_t)ysh[c - 1] : 0x1FFu;
      const uint32_t ycur = c < ny ? (uint32_t)ysh[c] : 0x1FFu;
      double above[NL], adiag[NL];
#pragma unroll
      for (int t = 0; t < NL; ++t) {
        above[t] = up[t];
        adiag[t] = pup[t];
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int r = r0 + k;
        if (r <= nx) {
          const uint32_t xprev = (xw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
          const uint32_t xcur = (xw[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu;
          const bool match = r >= 1 && c >= 1 && xprev == yprev;
          double cur[NL];
#pragma unroll
          for (int t = 0; t < NL; ++t) {
            const int lvl = t + 1;
            double v = 0.0;
            if (lvl < kk && r >= lvl && c >= lvl) {
              v = __dadd_rn(__dmul_rn(lam, above[t]), __dmul_rn(lam, last[k][t]));
              v = __dsub_rn(v, __dmul_rn(lam2, adiag[t]));
              if (match) {
                const double prevlvl = (t == 0) ? 1.0 : adiag[t - 1];
                v = __dadd_rn(v, __dmul_rn(lam2, prevlvl));
              }
            }
            cur[t] = v;
          }
          if (c < ny && r < nx && ycur == xcur) {
            double bkm1 = 1.0;  // B_0 == 1
#pragma unroll
            for (int t = 0; t < NL; ++t)
              if (t == kk - 2) bkm1 = cur[t];
            sacc[k] = __dadd_rn(sacc[k], bkm1);
          }
          if (bmode && r == nx && c == ny) {
#pragma unroll
            for (int t = 0; t < NL; ++t)
              if (t == kk - 2) bval = cur[t];
          }
#pragma unroll
          for (int t = 0; t < NL; ++t) {
            adiag[t] = last[k][t];
            above[t] = cur[t];
            last[k][t] = cur[t];
          }
        }
      }
#pragma unroll
      for (int t = 0; t < NL; ++t) {
        pup[t] = up[t];
        pub[t] = last[R - 1][t];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < R; ++k)
    if (dp && r0 + k < nx) Ssh[r0 + k + 1] = sacc[k];
  if (bmode && dp && nx >= r0 && nx < r0 + R) Ssh[0] = bval;
  __builtin_amdgcn_wave_barrier();
  if (s == 0 && pv) {
    double K = 0.0;
    if (bmode) {
      K = kk == 1 ? 1.0 : dp ? Ssh[0] : 0.0;  // B_0 == 1; short prefixes: 0 (kernels.py:331-335)
    } else if (kk == 0) {
      K = 1.0;  // K_k(.., 0, ..) returns 1 (kernels.py:354-355)
    } else if (dp) {
      for (int ii = kk; ii <= nx; ++ii) K = __dadd_rn(K, __dmul_rn(lam2, Ssh[ii]));
    }
    store_f(o, i - row0, j, K);
    if (mirror && j != i && j >= row0 && j < row1) store_f(o, j - row0, i, K);
  }
}

// ------------------------------------------------------------------ LA (intended)
// Local-alignment kernel with the reference's three defects removed (KMG_LA_INTENDED;
// oracle cpu_ref.la_intended_pair documents the semantics; parity unpinned): five DP
// arrays, cells (r, c) for r in 1..n_x, c in 1..n_y on x[r-1], y[c-1], gap opening factor
// exp(-beta e) and extension exp(-beta d).  One wave per pair (x = row min(i, j), y = row
// max(i, j): the reference's j >= i fill, kernels.py:293-297), the SS kernel's
// anti-diagonal sweep: lane l of a 64-row strip owns row r = s0 + l and at step st
// computes column c = st - l; its left neighbour is its own previous cell, "up" comes
// from lane l - 1 by a shuffle (lane 0: the previous strip's last row, kept in LDS), the
// diagonal is the previous step's "up".  Every cell is evaluated in the oracle's order
// with separately rounded products (no FMA): bit-identical sums, the final log within
// an ulp of libm's.
struct LaCoef {
  double es[16];   // exp(beta * S[a][b]), a * 4 + b (kernels.py:223)
  double eo, ee;   // exp(-beta e), exp(-beta d)
  double inv_beta; // 1 / beta (the reference's (1/beta) * log(...))
};

template <bool SMITH>
__global__ __launch_bounds__(256) void gram_la_kernel(SeqSpec q, int64_t row0, int64_t row1,
                                                      LaCoef cf, int mirror, OutSpec o) {
  extern __shared__ __align__(16) double lsm[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = row0 + blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * (blockDim.x >> 6) + wave;
  if (j >= q.n || i >= row1) return;
  if (mirror && j < i) return;
  const int ML = q.maxlen;
  // per wave: rowbuf[4][ML + 1] (M, X, Y, X2 of the strip's last row), result slot, y bytes
  const int per = 4 * (ML + 1) + 1 + (ML + 8) / 8;
  double *rowbuf = lsm + (size_t)wave * per;
  double *res = rowbuf + 4 * (ML + 1);
  uint8_t *yb = (uint8_t *)(res + 1);
  const int64_t ia = min(i, j), ib = max(i, j);
  const uint8_t *xs = q.codes + ia * q.ldc;
  const uint8_t *ys = q.codes + ib * q.ldc;
  const int nx = q.lens[ia], ny = q.lens[ib];
  for (int c = lane; c < ny; c += 64) yb[c] = ys[c];
  if (lane == 0) *res = 1.0;  // n_x or n_y == 0: cell [n_x, n_y] is the zero boundary
  __builtin_amdgcn_wave_barrier();
  const double eo = cf.eo, ee = cf.ee;
  for (int s0 = 0; s0 <= nx; s0 += 64) {
    const int r = s0 + lane;
    const bool live = r <= nx;
    const uint32_t xr = (r >= 1 && live) ? xs[r - 1] : 0u;
    // left (own previous cell) and diagonal values; row 0 / column 0 are zero
    double lM = 0.0, lX = 0.0, lY = 0.0, lX2 = 0.0, lY2 = 0.0;
    double dM = 0.0, dX = 0.0, dY = 0.0;
    const bool store_row = (lane == 63) && (s0 + 64 <= nx);
    for (int st = 0; st <= ny + 63; ++st) {
      const int c = st - lane;
      double uM = wave_shr1(lM), uX = wave_shr1(lX);
      double uY = wave_shr1(lY), uX2 = wave_shr1(lX2);
      if (lane == 0) {
        const bool rb = s0 > 0 && c >= 0 && c <= ny;
        uM = rb ? rowbuf[c] : 0.0;
        uX = rb ? rowbuf[(ML + 1) + c] : 0.0;
        uY = rb ? rowbuf[2 * (ML + 1) + c] : 0.0;
        uX2 = rb ? rowbuf[3 * (ML + 1) + c] : 0.0;
      }
      if (live && c >= 0 && c <= ny) {
        double M = 0.0, X = 0.0, Y = 0.0, X2 = 0.0, Y2 = 0.0;
        if (r >= 1 && c >= 1) {
          const double sub = cf.es[(xr & 3u) * 4 + (yb[c - 1] & 3u)];  // ACGT (host-checked)
          if (SMITH) {
            M = __dmul_rn(sub, fmax(fmax(fmax(1.0, dX), dY), dM));
            X = fmax(__dmul_rn(eo, uM), __dmul_rn(ee, uX));
            Y = fmax(fmax(__dmul_rn(eo, lM), __dmul_rn(eo, lX)), __dmul_rn(ee, lY));
            X2 = fmax(uM, uX2);
            Y2 = fmax(fmax(lM, lX2), lY2);
          } else {
            M = __dmul_rn(sub, __dadd_rn(__dadd_rn(__dadd_rn(1.0, dX), dY), dM));
            X = __dadd_rn(__dmul_rn(eo, uM), __dmul_rn(ee, uX));
            Y = __dadd_rn(__dmul_rn(eo, __dadd_rn(lM, lX)), __dmul_rn(ee, lY));
            X2 = __dadd_rn(uM, uX2);
            Y2 = __dadd_rn(__dadd_rn(lM, lX2), lY2);
          }
        }
        dM = uM; dX = uX; dY = uY;
        lM = M; lX = X; lY = Y; lX2 = X2; lY2 = Y2;
        if (store_row) {
          rowbuf[c] = M;
          rowbuf[(ML + 1) + c] = X;
          rowbuf[2 * (ML + 1) + c] = Y;
          rowbuf[3 * (ML + 1) + c] = X2;
        }
        if (r == nx && c == ny && r >= 1 && c >= 1)
          *res = SMITH ? fmax(fmax(fmax(1.0, X2), Y2), M)
                       : __dadd_rn(__dadd_rn(__dadd_rn(1.0, X2), Y2), M);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    const double result = __dmul_rn(cf.inv_beta, log(*res));
    store_f(o, i - row0, j, result);
    if (mirror && j != i && j >= row0 && j < row1) store_f(o, j - row0, i, result);
  }
}

// LA, grouped sweep (the SS layout above): 64 / LPP pairs a wave, lane s of a group owns
// the DP rows s R .. s R + R - 1; up (M, X, Y, X2 of row r - 1 at column c) comes from the
// row above in the lane or, for its first row, from lane s - 1's last row of the previous
// step (DPP wave_shr:1); the diagonal is the previous up.  Per cell the strip kernel's
// operation order (bit-identical).
template <int LPP, int R, bool SMITH>
__global__ __launch_bounds__(256) void gram_lag_kernel(SeqSpec q, int64_t row0, int64_t row1,
                                                       LaCoef cf, int mirror, OutSpec o) {
  constexpr int G = 64 / LPP;
  extern __shared__ __align__(16) double gsm[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane / LPP, s = lane % LPP;
  const int64_t i = row0 + blockIdx.y;
  const int64_t jb = (mirror ? i : 0) + ((int64_t)blockIdx.x * 4 + wave) * G;
  const bool wlive = i < row1 && jb < q.n;  // wave-uniform (the block syncs once below)
  const int ML = q.maxlen;
  double *res = gsm + (wave * G + g);
  uint8_t *ysh = (uint8_t *)(gsm + 4 * G) + (size_t)(wave * G + g) * (ML + 1);
  const int64_t j = jb + g;
  const bool pv = wlive && j < q.n;
  const int64_t ia = pv ? min(i, j) : 0, ib = pv ? max(i, j) : 0;
  const uint8_t *xs = q.codes + ia * q.ldc;
  const uint8_t *ys = q.codes + ib * q.ldc;
  const int nx = pv ? q.lens[ia] : -1, ny = pv ? q.lens[ib] : -1;
  for (int c = s; c < ny; c += LPP) ysh[c] = ys[c];
  if (s == 0) *res = 1.0;  // n_x or n_y == 0: cell [n_x, n_y] is the zero boundary
  // the substitution factors in LDS (a dynamically indexed kernel-argument array would be
  // materialised in VGPRs with a select chain per read)
  double *es = gsm + 4 * G + (4 * G * (ML + 1) + 7) / 8;
  if (threadIdx.x < 16) es[threadIdx.x] = cf.es[threadIdx.x];
  __syncthreads();
  uint32_t xw[(R + 3) / 4];  // byte k: x_{r0 + k - 1} & 3 (ACGT, host-checked)
#pragma unroll
  for (int w = 0; w < (R + 3) / 4; ++w) xw[w] = 0u;
  const int r0 = s * R;
#pragma unroll
  for (int k = 0; k < R; ++k) {
    const int rr = r0 + k - 1;
    const uint32_t v = (pv && rr >= 0 && rr < nx) ? (uint32_t)xs[rr] & 3u : 0u;
    xw[k >> 2] |= v << (8 * (k & 3));
  }
  if (!wlive) return;
  __builtin_amdgcn_wave_barrier();
  const double eo = cf.eo, ee = cf.ee;
  double lM[R], lX[R], lY[R], lX2[R], lY2[R];
#pragma unroll
  for (int k = 0; k < R; ++k) lM[k] = lX[k] = lY[k] = lX2[k] = lY2[k] = 0.0;
  double pM = 0.0, pX = 0.0, pY = 0.0, pX2 = 0.0;  // published: last row at this column
  double qM = 0.0, qX = 0.0, qY = 0.0;             // previous up (first row's diagonal)
  const int steps = ML + LPP;
  for (int st = 0; st < steps; ++st) {
    const int c = st - s;
    const double uM0 = wave_shr1(pM), uX0 = wave_shr1(pX), uY0 = wave_shr1(pY),
                 uX20 = wave_shr1(pX2);
    if (pv && c >= 0 && c <= ny) {
      const uint32_t yc = c >= 1 ? (uint32_t)ysh[c - 1] & 3u : 0u;
      double uM = uM0, uX = uX0, uX2 = uX20;  // row above at column c (Y: left only)
      double dM = qM, dX = qX, dY = qY;                  // row above at column c - 1
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int r = r0 + k;
        {  // rows past n_x: don't-care values (only rows below them read them), no branch
          double M, X, Y, X2, Y2;
          {
            const uint32_t xr = (xw[k >> 2] >> (8 * (k & 3))) & 3u;
            const double sub = es[xr * 4 + yc];
            if (SMITH) {
              M = __dmul_rn(sub, fmax(fmax(fmax(1.0, dX), dY), dM));
              X = fmax(__dmul_rn(eo, uM), __dmul_rn(ee, uX));
              Y = fmax(fmax(__dmul_rn(eo, lM[k]), __dmul_rn(eo, lX[k])), __dmul_rn(ee, lY[k]));
              X2 = fmax(uM, uX2);
              Y2 = fmax(fmax(lM[k], lX2[k]), lY2[k]);
            } else {
              M = __dmul_rn(sub, __dadd_rn(__dadd_rn(__dadd_rn(1.0, dX), dY), dM));
              X = __dadd_rn(__dmul_rn(eo, uM), __dmul_rn(ee, uX));
              Y = __dadd_rn(__dmul_rn(eo, __dadd_rn(lM[k], lX[k])), __dmul_rn(ee, lY[k]));
              X2 = __dadd_rn(uM, uX2);
              Y2 = __dadd_rn(__dadd_rn(lM[k], lX2[k]), lY2[k]);
            }
            const bool in = r >= 1 && c >= 1;  // row 0 / column 0: the zero boundary
            M = in ? M : 0.0;
            X = in ? X : 0.0;
            Y = in ? Y : 0.0;
            X2 = in ? X2 : 0.0;
            Y2 = in ? Y2 : 0.0;
          }
          if (r == nx && c == ny && r >= 1 && c >= 1)
            *res = SMITH ? fmax(fmax(fmax(1.0, X2), Y2), M)
                         : __dadd_rn(__dadd_rn(__dadd_rn(1.0, X2), Y2), M);
          // this row at c - 1 is the next row's diagonal, this row at c its up
          dM = lM[k];
          dX = lX[k];
          dY = lY[k];
          uM = M;
          uX = X;
          uX2 = X2;
          lM[k] = M;
          lX[k] = X;
          lY[k] = Y;
          lX2[k] = X2;
          lY2[k] = Y2;
        }
      }
      qM = uM0;
      qX = uX0;
      qY = uY0;
      pM = lM[R - 1];
      pX = lX[R - 1];
      pY = lY[R - 1];
      pX2 = lX2[R - 1];
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (s == 0 && pv) {
    const double result = __dmul_rn(cf.inv_beta, log(*res));
    store_f(o, i - row0, j, result);
    if (mirror && j != i && j >= row0 && j < row1) store_f(o, j - row0, i, result);
  }
}

hipError_t launch_gram_la(const SeqSpec &q, int64_t row0, int64_t row1, double e, double d,
                          double beta, int smith, int mirror, const OutSpec &o, hipStream_t s,
                          int lpp) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  const int ML = q.maxlen;
  if (rows > 65535) return hipErrorNotSupported;
  static const int S[4][4] = {{4, 0, 0, 0}, {0, 9, -3, -1}, {0, -3, 6, 2}, {0, -1, -2, 5}};
  LaCoef cf;
  for (int a = 0; a < 4; ++a)
    for (int b = 0; b < 4; ++b) cf.es[a * 4 + b] = std::exp(beta * (double)S[a][b]);
  cf.eo = std::exp(-beta * e);
  cf.ee = std::exp(-beta * d);
  cf.inv_beta = 1.0 / beta;
  // grouped sweep while a group's rows cover the sequences (LPP x R >= ML + 1)
  auto grouped = [&](auto lpp_c, auto r_c) -> hipError_t {
    constexpr int LPP = decltype(lpp_c)::value, R = decltype(r_c)::value, G = 64 / LPP;
    const size_t lds = (size_t)4 * G * sizeof(double) + ((4 * G * (ML + 1) + 7) / 8) * 8 + 16 * 8;
    const int64_t cols = mirror ? q.n - row0 : q.n;  // mirror: columns from row i on
    const dim3 grid((unsigned)((cols + 4 * G - 1) / (4 * G)), (unsigned)rows);
    if (smith)
      hipLaunchKernelGGL((gram_lag_kernel<LPP, R, true>), grid, dim3(256), (lds + 15) & ~(size_t)15,
                         s, q, row0, row1, cf, mirror, o);
    else
      hipLaunchKernelGGL((gram_lag_kernel<LPP, R, false>), grid, dim3(256), (lds + 15) & ~(size_t)15,
                         s, q, row0, row1, cf, mirror, o);
    return hipGetLastError();
  };
  // 16 lanes x 8 rows a pair by default (N = 1000, L = 101: 7.2 ms sum form against 11.9 at
  // 8 x 13 and 7.6 at 32 x 4; profiles/r03j_ss_la_lpp_ab.jsonl); KMG_LA_LPP for the A/B
  if (lpp == 8 && ML + 1 <= 8 * 13)
    return grouped(std::integral_constant<int, 8>{}, std::integral_constant<int, 13>{});
  if (lpp == 32 && ML + 1 <= 32 * 4)
    return grouped(std::integral_constant<int, 32>{}, std::integral_constant<int, 4>{});
  if (lpp == 64 && ML + 1 <= 64 * 2)
    return grouped(std::integral_constant<int, 64>{}, std::integral_constant<int, 2>{});
  if (ML + 1 <= 16 * 8)
    return grouped(std::integral_constant<int, 16>{}, std::integral_constant<int, 8>{});
  // longer sequences: the 64-row strip kernel, as many waves a block as the boundary rows'
  // LDS allows (4 up to length ~1250, 1 up to ~5100)
  const size_t per_wave = (size_t)(4 * (ML + 1) + 1 + (ML + 8) / 8) * sizeof(double);
  const int W = (int)std::min<size_t>(4, (160 * 1024) / per_wave);
  if (W < 1) return hipErrorNotSupported;
  const dim3 grid((unsigned)((q.n + W - 1) / W), (unsigned)rows);
  if (smith)
    hipLaunchKernelGGL((gram_la_kernel<true>), grid, dim3(64 * W), per_wave * W, s, q, row0, row1, cf,
                       mirror, o);
  else
    hipLaunchKernelGGL((gram_la_kernel<false>), grid, dim3(64 * W), per_wave * W, s, q, row0, row1, cf,
                       mirror, o);
  return hipGetLastError();
}

// ------------------------------------------------------------------ argument checks
// stats[0] = max symbol code over every row's first len symbols, stats[1] = min len (both
// must be preset by the caller to 0 / INT_MAX): the C ABI's alphabet / length checks on
// device-resident rows (kmgram.h: KMG_EINVAL for alphabet errors)
__global__ __launch_bounds__(256) void row_stats_kernel(SeqSpec q, uint32_t *stats) {
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= q.n) return;
  const int len = min(max(q.lens[j], 0), (int)q.ldc);
  uint32_t mx = 0;
  for (int t = lane; t < len; t += 64) mx = max(mx, (uint32_t)q.codes[j * q.ldc + t]);
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
  if (lane == 0) {
    atomicMax(&stats[0], mx);
    atomicMin(&stats[1], (uint32_t)len);
  }
}

hipError_t launch_row_stats(const SeqSpec &q, uint32_t *stats, hipStream_t s) {
  if (q.n == 0) return hipSuccess;
  hipLaunchKernelGGL(row_stats_kernel, dim3((unsigned)((q.n + 3) / 4)), dim3(256), 0, s, q, stats);
  return hipGetLastError();
}

// ------------------------------------------------------------------ GP (k=1, g=0)
// phi_c(x) = [letter c occurs in x[0:window]] (gappy_k with k=1, g=0, kernels.py:420-433);
// K_raw = <phi_x, phi_y>, then normalize_K (kernels.py:454).
__global__ void gappy1_diag_kernel(SeqSpec q, int window, double *diagv, double *dsq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q.n) return;
  const int L = min(q.lens[i], window);
  uint32_t m = 0;
  for (int t = 0; t < L; ++t) m |= 1u << (q.codes[i * q.ldc + t] & 3u);
  const double v = (double)__popc(m);
  diagv[i] = v;
  dsq[i] = __builtin_sqrt(v);
}

__global__ void gappy1_gram_kernel(SeqSpec q, int64_t row0, int64_t row1, int window, OutSpec o) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = row0 + blockIdx.y;
  if (j >= q.n || i >= row1) return;
  auto mask = [&](int64_t s) {
    const int L = min(q.lens[s], window);
    uint32_t m = 0;
    for (int t = 0; t < L; ++t) m |= 1u << (q.codes[s * q.ldc + t] & 3u);
    return m;
  };
  const double raw = (double)__popc(mask(i) & mask(j));
  const bool norm = o.normalize && o.diagv[0] != 1.0;
  double v = raw;
  if (norm) v = (i == j) ? 1.0 : raw / (o.dsq[i] * o.dsq[j]);
  store_f(o, i - row0, j, v);
}

// ------------------------------------------------------------------ dense helpers
__global__ void dense_diag_sqrt_kernel(const double *K, int64_t n, int64_t ld, double *dsq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dsq[i] = __builtin_sqrt(K[i * ld + i]);
}

__global__ void dense_normalize_kernel(double *K, int64_t n, int64_t ld, const double *dsq) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (j >= n || j < i) return;
  if (j == i) {
    K[i * ld + i] = 1.0;  // np.fill_diagonal(K, np.ones(n))
  } else {
    const double v = K[i * ld + j] / (dsq[i] * dsq[j]);  // K[i,j] /= (d * diag[j])
    K[i * ld + j] = v;
    K[j * ld + i] = v;  // K[j,i] = K[i,j]
  }
}

__global__ void dense_rowmean_kernel(const double *K, int64_t n, int64_t ld, double *rowmean) {
  __shared__ double red[256];
  const int64_t i = blockIdx.x;
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += blockDim.x) s += K[i * ld + j];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) rowmean[i] = red[0] / (double)n;
}

__global__ void dense_colmean_kernel(const double *K, int64_t n, int64_t ld, double *colmean) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s += K[i * ld + j];
  colmean[j] = s / (double)n;
}

__global__ void dense_total_kernel(const double *rowmean, int64_t n, double *tot) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) s += rowmean[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) tot[0] = red[0] / (double)n;
}

__global__ void dense_center_kernel(const double *K, int64_t ldk, double *out, int64_t ldo,
                                    int64_t n, const double *rowmean, const double *colmean,
                                    const double *tot) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (j >= n) return;
  out[i * ldo + j] = ((K[i * ldk + j] - rowmean[i]) - colmean[j]) + tot[0];
}

// ------------------------------------------------------------------ launchers
static bool pick_nw(int maxlen, int &nw) {
  if (maxlen <= 128) { nw = 2; return true; }
  if (maxlen <= 256) { nw = 4; return true; }
  return false;
}

static Coef make_coef(const double *a, const double *b) {
  Coef c;
  for (int t = 0; t < KMG_MAX_COEF; ++t) {
    c.a[t] = a ? a[t] : 0.0;
    c.b[t] = b ? b[t] : 0.0;
  }
  return c;
}

hipError_t launch_gram_wd(const SeqSpec &q, int64_t row0, int64_t row1, int d, int span,
                          const double *beta, const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  int nw;
  if (!pick_nw(q.maxlen, nw)) return hipErrorNotSupported;
  const Coef cf = make_coef(beta, nullptr);
  const dim3 grid((unsigned)((q.n + 63) / 64), (unsigned)((rows + 15) / 16));
  if (nw == 2)
    hipLaunchKernelGGL((gram_wd_kernel<2>), grid, dim3(256), 0, s, q, row0, row1, d, span, cf, o);
  else
    hipLaunchKernelGGL((gram_wd_kernel<4>), grid, dim3(256), 0, s, q, row0, row1, d, span, cf, o);
  return hipGetLastError();
}

hipError_t launch_gram_wd_packed(const SeqSpec &q, const Packed &pk, int64_t row0, int64_t row1,
                                 int d, int span, const double *beta, const OutSpec &o,
                                 hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  const int need = (q.maxlen + 15) / 16;  // code words a pair compares
  if (need > pk.cw) return hipErrorInvalidValue;
  const Coef cf = make_coef(beta, nullptr);
  // the whole square: upper tiles + transposed copies
  const bool mirror = row0 == 0 && row1 == q.n;
  const dim3 grid((unsigned)((q.n + 63) / 64), (unsigned)((rows + 63) / 64));
#define KMG_WDP(NC_)                                                                             \
  do {                                                                                           \
    if (mirror)                                                                                  \
      hipLaunchKernelGGL((gram_wdp_kernel<NC_, true>), grid, dim3(256), 0, s, q, pk, row0, row1, \
                         d, span, cf, o);                                                        \
    else                                                                                         \
      hipLaunchKernelGGL((gram_wdp_kernel<NC_, false>), grid, dim3(256), 0, s, q, pk, row0,     \
                         row1, d, span, cf, o);                                                  \
  } while (0)
  // plane words per pair: ceil(code words / 2)
  if (need <= 4) KMG_WDP(2);
  else if (need <= 8) KMG_WDP(4);
  else if (need <= 16) KMG_WDP(8);
  else return hipErrorNotSupported;
#undef KMG_WDP
  return hipGetLastError();
}

hipError_t launch_gram_wds(const SeqSpec &q, int64_t row0, int64_t row1, int d, int S, int span,
                           const double *beta, const double *delta, const OutSpec &o,
                           hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  int nw;
  if (!pick_nw(q.maxlen, nw)) return hipErrorNotSupported;
  const Coef cf = make_coef(beta, delta);
  const dim3 grid((unsigned)((q.n + 63) / 64), (unsigned)((rows + 15) / 16));
#define KMG_WDS(NW_, SM_) \
  hipLaunchKernelGGL((gram_wds_kernel<NW_, SM_>), grid, dim3(256), 0, s, q, row0, row1, d, S, span, cf, o)
  if (nw == 2) {
    if (S <= 1) KMG_WDS(2, 1);
    else if (S <= 3) KMG_WDS(2, 3);
    else if (S <= 7) KMG_WDS(2, 7);
    else if (S <= 15) KMG_WDS(2, 15);
    else return hipErrorNotSupported;
  } else {
    if (S <= 1) KMG_WDS(4, 1);
    else if (S <= 3) KMG_WDS(4, 3);
    else if (S <= 7) KMG_WDS(4, 7);
    else return hipErrorNotSupported;
  }
#undef KMG_WDS
  return hipGetLastError();
}

hipError_t launch_gram_ss(const SeqSpec &q, int64_t row0, int64_t row1, int kk, double lam,
                          double lam2, int mirror, const OutSpec &o, hipStream_t s, int lpp,
                          int bmode) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || q.n == 0) return hipSuccess;
  const int ML = q.maxlen;
  if (rows > 65535) return hipErrorInvalidValue;
  if (bmode) {
    // B_kk needs levels 1..kk: the sweep of K_{kk+1}, reading level kk at the corner
    if (kk < 0 || kk > 32) return hipErrorNotSupported;
    kk += 1;
  }
  // grouped sweep whenever the rows fit one group (LPP x R >= ML + 1) and kk - 1 <= 32
  // levels: NL levels exactly for kk <= 9, rounded up to 12 / 16 / 24 / 32 above
  const int nl = kk >= 2 ? kk - 1 : 1;
  auto grouped = [&](auto lpp_c, auto r_c, auto nl_c) -> hipError_t {
    constexpr int LPP = decltype(lpp_c)::value, R = decltype(r_c)::value, NL = decltype(nl_c)::value;
    constexpr int G = 64 / LPP;
    const size_t lds = (size_t)4 * G * ((ML + 2) * sizeof(double) + (ML + 1));
    const int64_t cols = mirror ? q.n - row0 : q.n;  // mirror: columns from row i on
    const dim3 grid((unsigned)((cols + 4 * G - 1) / (4 * G)), (unsigned)rows);
    hipLaunchKernelGGL((gram_ssg_kernel<LPP, R, NL>), grid, dim3(256), (lds + 15) & ~(size_t)15, s,
                       q, row0, row1, kk, lam, lam2, mirror, o, bmode);
    return hipGetLastError();
  };
#define KMG_SSG(LPP_, R_, NL_) \
  grouped(std::integral_constant<int, LPP_>{}, std::integral_constant<int, R_>{}, \
          std::integral_constant<int, NL_>{})
  // defaults from interleaved A/B at N = 1000, L = 101 (profiles/r03j_ss_la_lpp_ab.jsonl):
  // fewer rows a lane keep the cell registers small (k = 5: 8 lanes x 13 rows 23.4 ms,
  // 16 x 7 10.6 ms); KMG_SS_LPP forces another group width for the A/B
  if (lpp == 8 && nl <= 4 && ML + 1 <= 8 * 13) return KMG_SSG(8, 13, 4);
  if (lpp == 16 && nl <= 8 && ML + 1 <= 16 * 7) return KMG_SSG(16, 7, 8);
  if (lpp == 32 && nl <= 4 && ML + 1 <= 32 * 4) return KMG_SSG(32, 4, 4);
  if (lpp == 64 && nl <= 8 && ML + 1 <= 64 * 2) return KMG_SSG(64, 2, 8);
  if (lpp == 32 && nl > 8 && nl <= 16 && ML + 1 <= 32 * 4) return KMG_SSG(32, 4, 16);
  if (nl <= 4 && ML + 1 <= 16 * 7) {
    switch (nl) {
      case 1: return KMG_SSG(16, 7, 1);
      case 2: return KMG_SSG(16, 7, 2);
      case 3: return KMG_SSG(16, 7, 3);
      default: return KMG_SSG(16, 7, 4);
    }
  }
  if (nl <= 8 && ML + 1 <= 32 * 4) {
    switch (nl) {
      case 5: return KMG_SSG(32, 4, 5);
      case 6: return KMG_SSG(32, 4, 6);
      case 7: return KMG_SSG(32, 4, 7);
      default: return KMG_SSG(32, 4, 8);
    }
  }
  if (nl <= 32 && ML + 1 <= 64 * 2)
    return nl <= 12 ? KMG_SSG(64, 2, 12) : nl <= 16 ? KMG_SSG(64, 2, 16)
                    : nl <= 24 ? KMG_SSG(64, 2, 24) : KMG_SSG(64, 2, 32);
#undef KMG_SSG
  if (bmode) return hipErrorNotSupported;
  // longer sequences: the strip kernel (64-row strips, the boundary row in LDS), as many
  // waves (pairs) a block as their LDS allows (4 up to length ~300 at k = 16, 1 to ~1200)
  const int kmx = kk <= 2 ? 2 : kk <= 4 ? 4 : kk <= 8 ? 8 : 16;
  const size_t per_wave = (size_t)((kmx - 1) * (ML + 1) + (ML + 2) + (ML + 4 + 7) / 8) * 8;
  const int W = (int)std::min<size_t>(4, (160 * 1024) / per_wave);
  if (W < 1) return hipErrorNotSupported;
  const dim3 grid((unsigned)((q.n + W - 1) / W), (unsigned)rows);
  auto lds_for = [&](int) { return per_wave * W; };
#define KMG_SS(KM_)                                                                          \
  hipLaunchKernelGGL((gram_ss_kernel<KM_>), grid, dim3(64 * W), lds_for(KM_), s, q, row0, row1, kk, \
                     lam, lam2, mirror, o)
  if (kk <= 2) KMG_SS(2);
  else if (kk <= 4) KMG_SS(4);
  else if (kk <= 8) KMG_SS(8);
  else if (kk <= 16) KMG_SS(16);
  else return hipErrorNotSupported;
#undef KMG_SS
  return hipGetLastError();
}

hipError_t launch_gram_gappy1(const SeqSpec &q, int64_t row0, int64_t row1, int window,
                              const OutSpec &o, double *diagv, double *dsq, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (q.n == 0) return hipSuccess;
  hipLaunchKernelGGL(gappy1_diag_kernel, dim3((unsigned)((q.n + 255) / 256)), dim3(256), 0, s, q,
                     window, diagv, dsq);
  if (rows <= 0) return hipGetLastError();
  hipLaunchKernelGGL(gappy1_gram_kernel, dim3((unsigned)((q.n + 255) / 256), (unsigned)rows),
                     dim3(256), 0, s, q, row0, row1, window, o);
  return hipGetLastError();
}

hipError_t launch_normalize_dense(double *K, int64_t n, int64_t ld, hipStream_t s) {
  if (n == 0) return hipSuccess;
  double *dsq = nullptr;
  hipError_t e = hipMallocAsync((void **)&dsq, sizeof(double) * n, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(dense_diag_sqrt_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, K,
                     n, ld, dsq);
  hipLaunchKernelGGL(dense_normalize_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)n),
                     dim3(256), 0, s, K, n, ld, dsq);
  e = hipGetLastError();
  (void)hipFreeAsync(dsq, s);
  return e;
}

hipError_t launch_center_dense(const double *K, int64_t ldk, double *out, int64_t ld_out,
                               int64_t n, double *rowmean, double *colmean, double *tot,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(dense_rowmean_kernel, dim3((unsigned)n), dim3(256), 0, s, K, n, ldk, rowmean);
  hipLaunchKernelGGL(dense_colmean_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, K, n,
                     ldk, colmean);
  hipLaunchKernelGGL(dense_total_kernel, dim3(1), dim3(256), 0, s, rowmean, n, tot);
  hipLaunchKernelGGL(dense_center_kernel, dim3((unsigned)((n + 255) / 256), (unsigned)n), dim3(256),
                     0, s, K, ldk, out, ld_out, n, rowmean, colmean, tot);
  return hipGetLastError();
}

}  // namespace kmg
