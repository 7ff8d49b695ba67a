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
// Sequences are read 2-bit packed (Packed, kmg_internal.h): a workgroup stages its row's
// record (52 bytes at L = 101) in LDS and derives every window's k-mer code from it.
//
// Mismatch (m=1) uses the closed form K(x,y) = sum_{a,b} w[ham(x_a, y_b)],
// w = (1+3k, 4, 2, 0, ...)  (= <Phi_x, Phi_y> of kernels.py:161-175) and
// enumerates the Hamming<=2 neighbourhood through the "drop one letter" index
// (kmg_index.hip): list (p, key_p(z)) holds every occurrence that equals z outside
// position p, in 4 sub-bins by its letter at p.
#include "kmg_internal.h"
#include "kmg_rowacc.h"

#include <algorithm>
#include <type_traits>

namespace kmg {

__device__ __forceinline__ uint32_t letter_at_g(uint32_t code, int p, int k) {
  return (code >> (2 * (k - 1 - p))) & 3u;
}
__device__ __forceinline__ uint32_t drop_letter_g(uint32_t code, int p, int k) {
  const uint64_t c = code;
  const int lo_bits = 2 * (k - 1 - p);
  return (uint32_t)(((c >> (lo_bits + 2)) << lo_bits) | (c & ((1ull << lo_bits) - 1ull)));
}

// ------------------------------------------------------------------ spectrum
// One workgroup of 1024 threads owns (row i, column chunk c); PACK16: two 16-bit counters
// per LDS word (valid when every K_ij <= 65535, i.e. P_i * P_j <= 65535; the host checks
// P_max <= 255), so a 20000-column chunk is 40 KB and two rows are in flight per CU.
// Gather: lpw lanes per row window (a power of two filling the block: 8 at 94 windows);
// the window's posting list is read as aligned 16-byte pieces of 8 entries, lane s of the
// window taking pieces s, s + lpw, ...; the first two pieces of every lane are issued
// before the accumulator is cleared, so the clear overlaps the entry loads.  Only pieces
// holding entries of the list are read.
// Store: 16 bytes per lane and step, every store instruction of a wave covering 1 KB of
// the row (int32 / float32: 4 columns a lane; float64: 2), so every line is written whole.
// NT: non-temporal stores (measured faster for multi-chunk and float64 K; plain stores
// faster for a single-chunk int32 K, profiles/r02t_sp_store.jsonl).
// ROWS > 1 (KMG_SP_ROWS; full-width dtypes only): one workgroup owns ROWS consecutive rows of
// the chunk, their accumulators side by side in LDS, the windows of all its rows over its lane
// groups, so the per-workgroup costs (accumulator clear, descriptors, barriers) are shared.
template <bool PACK16, int DT, bool NT, int ROWS>
__global__ __launch_bounds__(1024) void gram_sp_kernel(IndexGeom g, Packed pk,
                                                       const uint32_t *__restrict__ off,
                                                       const uint16_t *__restrict__ ent,
                                                       int64_t row0, int64_t rows,
                                                       int chunk_major, OutSpec o) {
  extern __shared__ __align__(16) uint32_t acc_all[];
  // chunk_major: chunk-major grid (all rows of chunk 0 first, so the lists in flight all
  // belong to one chunk's slice of the index: 3.7 MB at N=100000 instead of all 18.6 MB,
  // which the XCD's L2 keeps despite the K stores streaming through it; FETCH_SIZE 4.5 ->
  // 0.96 GB per launch, config 4 Gram 6.66 -> 5.85 ms = 6.8 TB/s), else row-major
  const int64_t groups = (rows + ROWS - 1) / ROWS;  // row groups of the launch
  const int64_t gl = chunk_major ? (int64_t)blockIdx.x % groups : blockIdx.x / g.nchunks;
  const int c = chunk_major ? (int)((int64_t)blockIdx.x / groups) : (int)(blockIdx.x - gl * g.nchunks);
  const int64_t il0 = gl * ROWS;
  const int nr = (int)min((int64_t)ROWS, rows - il0);  // rows of this workgroup
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  if (col0 + cw <= o.col_lo) return;  // the whole chunk lies below the written columns
  const int words = PACK16 ? (((g.chunk + 7) >> 3) << 2) : (((g.chunk + 3) >> 2) << 2);
  const uint32_t *__restrict__ o_c = off + (size_t)c * g.nkeys;
  const uint4 *__restrict__ e4 = (const uint4 *)ent;
  const int nwr = nr * g.pmax;  // windows of the workgroup's rows
  // lanes per window: a power of two, >= 2, so that the windows of the rows fill the block
  int lpw = 2;
  while (lpw < 16 && (lpw << 1) * ROWS * g.pmax <= (int)blockDim.x) lpw <<= 1;
  const int sub = threadIdx.x & (lpw - 1);
  const int nwin = blockDim.x / lpw;
  int a = threadIdx.x / lpw;
  uint32_t *acc = acc_all;  // the accumulator of window a's row
  auto add = [&](uint32_t j0) {
    if (PACK16)
      atomicAdd(&acc[j0 >> 1], 1u << ((j0 & 1) << 4));
    else
      atomicAdd(&acc[j0], 1u);
  };
  // entries of piece q (halfwords [8q, 8q + 8)) that fall in [beg, end)
  auto piece = [&](const uint4 &v, uint32_t q, uint32_t beg, uint32_t len) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      const uint32_t rel = 8u * q + (uint32_t)h - beg;
      if (rel < len) add((w[h >> 1] >> ((h & 1) * 16)) & 0xFFFFu);
    }
  };
  auto window = [&](int aw, uint32_t &b, uint32_t &l) {  // window aw: list + accumulator
    const int r = ROWS == 1 ? 0 : aw / g.pmax;
    const int aa = aw - r * g.pmax;
    acc = acc_all + r * words;
    l = 0;
    const uint32_t u = pk_window(pk.w + (row0 + il0 + r) * pk.ldp, pk.cw, aa, g.k);
    if (u != KMG_INVALID) {
      b = o_c[u];
      l = o_c[u + 1] - b;
    }
  };
  uint32_t beg = 0, len = 0;
  if (a < nwr) window(a, beg, len);
  uint32_t q0 = beg >> 3;
  uint4 p0 = make_uint4(0, 0, 0, 0), p1 = p0;
  // only pieces that hold entries of the list are read
  if (len && 8u * (q0 + sub) < beg + len) p0 = e4[q0 + sub];
  if (len && 8u * (q0 + sub + lpw) < beg + len) p1 = e4[q0 + sub + lpw];
  uint4 *acc4 = (uint4 *)acc_all;
  for (int w = threadIdx.x; w < ((ROWS * words) >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  for (;;) {
    if (len) {
      if (8u * (q0 + sub) < beg + len) piece(p0, q0 + sub, beg, len);
      if (8u * (q0 + sub + lpw) < beg + len) piece(p1, q0 + sub + lpw, beg, len);
      for (uint32_t q = q0 + 2 * lpw + sub; 8u * q < beg + len; q += lpw) piece(e4[q], q, beg, len);
    }
    a += nwin;
    if (a >= nwr) break;  // more windows than lane groups (long sequences)
    window(a, beg, len);
    q0 = beg >> 3;
    if (len && 8u * (q0 + sub) < beg + len) p0 = e4[q0 + sub];
    if (len && 8u * (q0 + sub + lpw) < beg + len) p1 = e4[q0 + sub + lpw];
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  const int qs = (int)max((int64_t)0, o.col_lo - col0);  // a multiple of 8 (host check)
  for (int r = 0; r < nr; ++r) {
  acc = acc_all + r * words;
  const int64_t il = il0 + r, i = row0 + il;
  if constexpr (DT == KMG_U8) {
    // raw off-diagonal counts as uint8, diagonal column stored as 0 (see emit_row), 16
    // columns = 16 B per lane and step from the packed 16-bit counters
    static_assert(PACK16, "8-bit slabs need the packed accumulator");
    uint8_t *prow = (uint8_t *)o.out + il * o.ld + col0;
    bool big = false;
    for (int q = qs + threadIdx.x * 16; q < cw; q += blockDim.x * 16) {
      uint32_t v[16];
      if (q + 16 <= cw) {
        const uint4 a = *(const uint4 *)&acc[q >> 1], b = *(const uint4 *)&acc[(q >> 1) + 4];
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int h = 0; h < 16; ++h) v[h] = (w[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
      } else {
#pragma unroll
        for (int h = 0; h < 16; ++h)
          v[h] = q + h < cw ? (acc[(q + h) >> 1] >> (16 * ((q + h) & 1))) & 0xFFFFu : 0u;
      }
#pragma unroll
      for (int h = 0; h < 16; ++h) {
        const bool dg = col0 + q + h == i;
        v[h] = (dg || q + h >= cw) ? 0u : u8_slab_entry(o, i, col0 + q + h, v[h], big);
      }
      uint8_t *d = prow + q;
      if (q + 16 <= cw && (((uintptr_t)d) & 15) == 0) {
        uint4 x;
        x.x = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
        x.y = v[4] | (v[5] << 8) | (v[6] << 16) | (v[7] << 24);
        x.z = v[8] | (v[9] << 8) | (v[10] << 16) | (v[11] << 24);
        x.w = v[12] | (v[13] << 8) | (v[14] << 16) | (v[15] << 24);
        *(uint4 *)d = x;
      } else {
        for (int h = 0; h < 16 && q + h < cw; ++h) d[h] = (uint8_t)v[h];
      }
    }
    if (big && o.ovf) atomicOr(o.ovf, 1u);
  } else if constexpr (DT == KMG_U16) {
    // raw counts as uint16 (multi-GPU round slabs, never normalised here): with PACK16 the
    // LDS words are the uint16 pairs themselves (column 2w in the low half = little-endian
    // order), 8 columns = 16 B per lane and step; P_max <= 255 bounds every count by 65025
    static_assert(PACK16, "16-bit slabs need the packed accumulator");
    uint16_t *prow = (uint16_t *)o.out + il * o.ld + col0;
    for (int q = qs + threadIdx.x * 8; q < cw; q += blockDim.x * 8) {
      const uint4 w = *(const uint4 *)&acc[q >> 1];
      uint16_t *d = prow + q;
      if (q + 8 <= cw && (((uintptr_t)d) & 15) == 0) {
        if constexpr (NT) {
          typedef int v4i __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(__builtin_bit_cast(v4i, w), (v4i *)d);
        } else {
          *(uint4 *)d = w;
        }
      } else {
        const uint32_t x[4] = {w.x, w.y, w.z, w.w};
        for (int h = 0; h < 8 && q + h < cw; ++h) d[h] = (uint16_t)(x[h >> 1] >> (16 * (h & 1)));
      }
    }
  } else if constexpr (DT == KMG_F64) {
    // two columns (16 B) per lane and step, so every store instruction of a wave covers
    // 1 KB of the row contiguously (whole lines: no partial-line writes)
    typedef double v2d __attribute__((ext_vector_type(2)));
    double *prow = (double *)o.out + il * o.ld + col0;
    const bool al = (((uintptr_t)prow) & 15) == 0;
    const double di = norm ? o.dsq[i] : 1.0;
    for (int q = qs + threadIdx.x * 2; q < cw; q += blockDim.x * 2) {
      uint32_t v0, v1;
      if (PACK16) {
        const uint32_t w = acc[q >> 1];
        v0 = w & 0xFFFFu; v1 = w >> 16;
      } else {
        const uint2 w = *(const uint2 *)&acc[q];
        v0 = w.x; v1 = w.y;
      }
      const int64_t c0 = o.col_seq0 + col0 + q;  // the column's sequence (column blocks)
      const bool two = q + 1 < cw;
      double r0 = (double)v0, r1 = (double)v1;
      if (norm) {  // normalize_K: K[i,j] / (sqrt(K[i,i]) * sqrt(K[j,j])), diagonal := 1
        r0 = (i == c0) ? 1.0 : (double)v0 / (di * o.dsq[c0]);
        r1 = !two ? 0.0 : (i == c0 + 1) ? 1.0 : (double)v1 / (di * o.dsq[c0 + 1]);
      }
      if (al && two) {
        const v2d x = {r0, r1};
        if constexpr (NT)
          __builtin_nontemporal_store(x, (v2d *)(prow + q));
        else
          *(v2d *)(prow + q) = x;
      } else {
        prow[q] = r0;
        if (two) prow[q + 1] = r1;
      }
    }
  } else {
    for (int q = qs + threadIdx.x * 4; q < cw; q += blockDim.x * 4) {
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
  }
  }  // rows of the workgroup
}

// ------------------------------------------------------------------ mismatch m=1
// Slot layout (kmg_index.hip slot_pack_kernel): every 4-bin group (copy p, chunk, key) of
// the rotated drop-one-letter index is ONE 128-byte line: uint16 e1, e2, e3, tot (ends of
// the letter-0/1/2 bins relative to the group start, and the group total; tot = 0xFFFF:
// too large for 16-bit counts, CSR only) followed by the first KMG_SLOT_INLINE entries.
// Sub-lists of a row k-mer u (NSUB = k + 3k(k-1)/2), walked copy-major so the lists in
// flight on an XCD read one copy's table:
//   type 1 (p): group key_p(u): letter u_p bin -> Hamming 0 (counted on p = 0 only, w0),
//               other letters -> Hamming 1 at p (w1)
//   type 2 (p, q < p, ci): key_p(u) with letter q replaced by the ci-th other letter:
//               letters != u_p -> Hamming 2 at {q, p} (w2); the u_p bin is skipped
// Every Hamming <= 2 neighbour of u is visited exactly once with its weight.
// Two lanes per list; lane gl takes the line's 16-byte pieces gl, gl+2, gl+4, gl+6, so
// step j covers halfwords [16j, 16j+16) of every list of the wave and is skipped when no
// list reaches it.  Per slot: SDWA column address + interval test + ds_add.  The in-bin
// Hamming-0 adds (copy 0 only) are taken from the CSR after the loop.  D lists in flight
// per lane pair (a ring unrolled at compile time); grid chunk-major.
template <int K, int D>
__global__ __launch_bounds__(1024) void gram_mm1_kernel(IndexGeom g, Packed pk,
                                                        const uint4 *__restrict__ slots,
                                                        const uint32_t *__restrict__ off,
                                                        const uint16_t *__restrict__ ent,
                                                        int64_t row0, int64_t rows, int w0,
                                                        int w1, int w2, OutSpec o) {
  constexpr int G = 2, CH = 4;
  constexpr int NSUB = K + 3 * K * (K - 1) / 2;
  extern __shared__ __align__(16) uint32_t smem[];  // acc first: LDS offset 0 (col_addr_sdwa)
  int c;
  int64_t il;
  rowacc_block(g, o, row0, rows, c, il);
  const int64_t i = row0 + il;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  if (col0 + cw <= o.col_lo) return;  // the whole chunk lies below the written columns
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;
  uint32_t *rotk = smem + accw;   // [P][K]: rot_p(u_a)
  uint32_t *sub = rotk + P * K;   // [NSUB]: p | q << 8 | ci << 16 (q = 0xFF: type 1)
  uint32_t *srec = sub + NSUB;    // packed row record
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  stage_record(pk, i, srec);
  for (int s = threadIdx.x; s < NSUB; s += blockDim.x) {
    // copy-major: copy p owns 1 + 3p sub-lists (type 1, then (q < p, ci))
    int pp = 0;
    while ((pp + 1) + 3 * (pp + 1) * pp / 2 <= s) ++pp;
    const int r = s - (pp + 3 * pp * (pp - 1) / 2);
    sub[s] = r == 0 ? ((uint32_t)pp | (0xFFu << 8))
                    : ((uint32_t)pp | ((uint32_t)((r - 1) / 3) << 8) | ((uint32_t)((r - 1) % 3) << 16));
  }
  __syncthreads();
  for (int t = threadIdx.x; t < P * K; t += blockDim.x) {
    const int a = t / K, p = t - a * K;
    const uint32_t u = pk_window(srec, pk.cw, a, K);
    // an invalid window (host-checked ACGT input has none) enumerates the lists of
    // k-mer 0 with zero weights below
    rotk[t] = u == KMG_INVALID ? 0xFFFFFFFFu : (drop_letter_g(u, p, K) << 2) | letter_at_g(u, p, K);
  }
  __syncthreads();

  const uint32_t chunk_groups = (uint32_t)c * (g.nkeys >> 2);
  const uint32_t copy_groups = (uint32_t)g.nchunks * (g.nkeys >> 2);
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int lane = threadIdx.x & 63;
  const int total = P * NSUB;

  auto describe = [&](int L, uint32_t &gidx, uint32_t &meta) {
    const int Lc = L < total ? L : total - 1;
    const int s = Lc / P;
    const int a = Lc - s * P;
    const uint32_t d = sub[s];
    const int p = d & 0xFF;
    const bool t1 = ((d >> 8) & 0xFF) == 0xFF;
    const int q = t1 ? 0 : (int)((d >> 8) & 0xFF);
    const uint32_t rkr = rotk[a * K + p];
    const bool valid = L < total && rkr != 0xFFFFFFFFu;
    const uint32_t rk = valid ? rkr : 0u;
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
    for (int j = 0; j < CH; ++j) b[j] = sp[2 * j];
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
  auto process = [&](const uint4(&b)[CH], uint32_t gidx, uint32_t meta) {
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
      const uint32_t wd[4] = {b[j].x, b[j].y, b[j].z, b[j].w};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        // active: a valid inline entry outside the query letter's bin (weight wb); the
        // in-bin entries (weight wa: Hamming 0, copy 0 only) are added below
        const uint32_t rel = (uint32_t)(16 * j + v) - lo_l;  // = t - lo
        const int t = 16 * j + 8 * gl + v - 4;
        const uint32_t ad = (v & 1) ? col_addr_sdwa<1>(wd[v >> 1]) : col_addr_sdwa<0>(wd[v >> 1]);
        if (t >= 0 && (uint32_t)t < lim && rel >= span)
          __hip_atomic_fetch_add((__attribute__((address_space(3))) int32_t *)(uintptr_t)ad, wb,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    if (wa && !big) {  // in-bin inline entries [lo, min(hi, lim)) with weight wa, from the CSR
      const uint32_t o0 = off[(size_t)gidx * 4];
      const uint32_t e1x = o0 + min(hi, lim);
      for (uint32_t e = o0 + lo + (uint32_t)gl; e < e1x; e += G) atomicAdd(&acc[ent[e]], wa);
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
  emit_row<true>(o, il, i, col0, cw, (const int32_t *)acc, norm);
}

// ------------------------------------------------------------------ mismatch m=1, pair table
// Drop-two-letters formulation (PairGeom, kmg_internal.h).  For a row k-mer u and a pair
// p < q, group key_pq(u) holds every occurrence z that agrees with u outside {p, q}, in 16
// sub-bins (z_p, z_q), z_p-major.  Weights, an inclusion-exclusion that leaves every entry
// of every group with the same weight w2 and NO per-entry test:
//   every entry of every group -> w2.  A Hamming-2 neighbour at {a, b} sits in group
//     (a, b) only; a Hamming-1 neighbour at r in the k-1 groups (p, q) holding r; the
//     row's own k-mer (Hamming 0) in all k(k-1)/2.
//   corrections, in the pairs (0, r) only (k-1 of the 36 lists of a window):
//     row u_0 of (0, r) minus the exact bin (z_0 = u_0, z_r != u_r: Hamming 1 at r)
//       -> + c = w1 - (k-1) w2;
//     r = 1: the exact bin (u_0, u_1) (Hamming 0) -> + h0 = w0 - k(k-1)/2 w2, and the
//       column bins (z_0 != u_0, z_1 = u_1: Hamming 1 at 0) -> + c.
// Net: every Hamming <= 2 neighbour gets exactly w[ham] (the closed form of
// <Phi_x, Phi_y>, kernels.py:161-175, 211-215).  The pack kernel fills the tail of a
// group's last line with lane-spread dummy columns (64 LDS words past the accumulator),
// so a lane adds w2 for every halfword of its pieces: one SDWA + one ds_add per entry.
// Per row: k(k-1)/2 lists per window (36 at k = 9, against 117 one-line lists of the
// drop-one table), each a few whole lines.
// Four lanes per list (the per-list decode is shared by fewer lanes than entries: 8 lanes
// doubled the VALU work per line); per list (pipelined): a 32-byte summary record (L2)
// gives the group's first line and line count nl (DPP sums over the 4 lanes), then lane gl
// loads the group header and its pieces [2 gl nl, 2 gl nl + 2 nl) with buffer loads
// (pieces past them fall outside the buffer: no traffic), builds 64-bit masks of its
// entries from the 16 bin-end bytes and adds the weights with LDS atomics.
__device__ __forceinline__ uint64_t span_mask(int a, int b) {  // bits [a, b) of 0..63
  const int lo = min(max(a, 0), 64), hi = min(max(b, 0), 64);
  const uint64_t mh = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
  const uint64_t ml = lo >= 64 ? ~0ull : ((1ull << lo) - 1ull);
  return mh & ~ml;
}
__device__ __forceinline__ uint32_t nibble_sum(uint32_t x) {
  const uint32_t y = (x & 0x0F0F0F0Fu) + ((x >> 4) & 0x0F0F0F0Fu);
  return (y * 0x01010101u) >> 24;
}
// sum over each aligned group of 4 lanes, result in all 4 (DPP quad swaps)
__device__ __forceinline__ uint32_t sum4(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
  return v;
}
// start / end of sub-bin b from the header dwords (bin ends as bytes, e[15] = n)
__device__ __forceinline__ int bin_end(const uint32_t (&h)[4], int b) {
  const int q = b >> 2;  // select, not an indexed load: keeps h in registers
  const uint32_t w = q == 0 ? h[0] : q == 1 ? h[1] : q == 2 ? h[2] : h[3];
  return (int)((w >> (8 * (b & 3))) & 0xFFu);
}
__device__ __forceinline__ int bin_start(const uint32_t (&h)[4], int b) {
  return b == 0 ? 0 : bin_end(h, b - 1);
}

template <int K, int D>
__global__ __launch_bounds__(1024) void gram_mm2_kernel(PairGeom pg, IndexGeom g, Packed pk,
                                                        const uint32_t *__restrict__ summary,
                                                        const uint4 *__restrict__ lines,
                                                        uint32_t line_bytes,
                                                        const uint32_t *__restrict__ xoff,
                                                        const uint16_t *__restrict__ xent,
                                                        int64_t row0, int64_t rows, int w0, int w1,
                                                        int w2, OutSpec o) {
  // G lanes per list; a lane takes 2 nl of the group's 8 nl 16-byte pieces, MAXP of them
  // in registers: groups of > 3 lines (n > 184) go the exact-index way like wide ones
  constexpr int G = 4, MAXP = 6, MAXNL = MAXP * G / 8;
  constexpr int NP = K * (K - 1) / 2;
  constexpr uint32_t NK2 = 1u << (2 * (K - 2));
  // one dynamic LDS block, accumulator first: col_addr_sdwa needs acc at LDS offset 0, so
  // this kernel declares no static __shared__ variable
  extern __shared__ __align__(16) uint32_t smem[];
  int c;
  int64_t il;
  rowacc_block(g, o, row0, rows, c, il);
  const int64_t i = row0 + il;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  if (col0 + cw <= o.col_lo) return;  // the whole chunk lies below the written columns
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int P = g.pmax;
  int32_t *acc = (int32_t *)smem;  // [accw] + 64 dummy words (the pack kernel's padding)
  uint32_t *rowk = smem + accw + 64;  // [P] row k-mers (KMG_INVALID: skipped)
  uint32_t *srec = rowk + P;     // packed row record
  uint32_t *spq = srec + pk.ldp; // [NP] p | q << 8 of every pair
  uint4 *acc4 = (uint4 *)acc;
  for (int w = threadIdx.x; w < (accw >> 2) + 16; w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  stage_record(pk, i, srec);
  if (threadIdx.x < NP) spq[threadIdx.x] = pg.pq[threadIdx.x];
  __syncthreads();
  for (int a = threadIdx.x; a < P; a += blockDim.x) rowk[a] = pk_window(srec, pk.cw, a, K);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t rl =
      __builtin_amdgcn_make_buffer_rsrc((void *)lines, (short)0, (int)line_bytes, 0x00020000);
  const int ngrp = blockDim.x / G, grp = threadIdx.x / G, gl = threadIdx.x % G;
  const int total = NP * P;
  const uint32_t chunk_base = (uint32_t)c * NK2;
  const uint32_t pair_stride = (uint32_t)g.nchunks * NK2;
  const int cc = w1 - (K - 1) * w2;   // Hamming 1: on top of the w2 of its K-1 groups
  const int h0 = w0 - NP * w2;        // Hamming 0: on top of the w2 of all NP groups

  // the lists of this lane group: L = grp + t * ngrp, pair-major (pi, a) = divmod(L, P),
  // walked incrementally (no division per list)
  int nx_pi = grp / P, nx_a = grp - (grp / P) * P, nx_L = grp;
  // describe the next list of the stream and advance it; meta = u_p | u_q << 2 |
  // valid << 4 | special (p == 0) << 5 | q << 8
  auto describe_next = [&](uint32_t &gidx, uint32_t &meta) {
    const bool in = nx_L < total;
    const uint32_t pq = spq[in ? nx_pi : 0];
    const int p = pq & 0xFF, q = pq >> 8;
    const uint32_t u = rowk[in ? nx_a : 0];
    const bool valid = in && u != KMG_INVALID;
    const uint32_t uu = valid ? u : 0u;
    gidx = (uint32_t)(in ? nx_pi : 0) * pair_stride + chunk_base + pair_key(uu, K, p, q);
    meta = ((uu >> (2 * (K - 1 - p))) & 3u) | (((uu >> (2 * (K - 1 - q))) & 3u) << 2) |
           ((valid ? 1u : 0u) << 4) | ((p == 0 ? 1u : 0u) << 5) | ((uint32_t)q << 8);
    nx_L += ngrp;
    nx_a += ngrp;
    while (nx_a >= P) {
      nx_a -= P;
      ++nx_pi;
    }
  };
  // summary dwords 2 gl, 2 gl + 1 of the group's record (dword 0: base line, dwords 1..4:
  // line-count nibbles of groups 0..31)
  auto load_summary = [&](uint32_t gidx) -> uint2 {
    return ((const uint2 *)summary)[(size_t)(gidx >> 5) * 4 + gl];
  };
  // nibble sum of word w (1..4) over the groups before r, and group r's own nibble
  auto nib_part = [&](uint32_t sw, int w, int r, uint32_t &part, uint32_t &own) {
    const int below = r - 8 * (w - 1);
    const uint32_t m = below >= 8 ? 0xFFFFFFFFu : (below <= 0 ? 0u : ((1u << (4 * below)) - 1u));
    part += nibble_sum(sw & m);
    own += (below >= 0 && below < 8) ? (sw >> (4 * below)) & 15u : 0u;
  };
  // base line and line count of the group from the 4 lanes' summary dwords
  auto decode = [&](uint2 sw, uint32_t gidx, uint32_t meta, uint32_t &base, uint32_t &nl) {
    const int r = (int)(gidx & 31u);
    uint32_t part = 0, own = 0;
    if (gl == 0) {
      part = sw.x;
      nib_part(sw.y, 1, r, part, own);
    } else if (gl == 1) {
      nib_part(sw.x, 2, r, part, own);
      nib_part(sw.y, 3, r, part, own);
    } else if (gl == 2) {
      nib_part(sw.x, 4, r, part, own);
    }
    base = sum4(part);
    nl = (meta & 16u) ? sum4(own) : 0u;
  };
  // header (piece 0) and this lane's pieces [gl * 2nl, gl * 2nl + 2nl)
  auto load_lines = [&](uint32_t base, uint32_t nl, uint4 &hdr, uint4(&d)[MAXP]) {
    const uint32_t np = nl <= (uint32_t)MAXNL ? 2u * nl : 0u;  // pieces of this lane
    const uint32_t first = (uint32_t)gl * np;
    hdr = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rl, nl ? base * 128u : 0xFFFFFFF0u, 0, 0));
#pragma unroll
    for (int s = 0; s < MAXP; ++s) {
      const uint32_t off = (uint32_t)s < np ? (base * 128u + (first + (uint32_t)s) * 16u) : 0xFFFFFFF0u;
      d[s] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rl, off, 0, 0));
    }
  };
  // correction of sub-bin (zp, zq) on top of w2 (pairs (0, r) only; see above)
  auto bin_corr = [&](uint32_t meta, uint32_t zp, uint32_t zq) -> int {
    if (!(meta & 32u)) return 0;
    const uint32_t up = meta & 3u, uq = (meta >> 2) & 3u;
    const int r = (int)(meta >> 8);
    if (zp == up) return zq == uq ? (r == 1 ? h0 : 0) : cc;
    return (r == 1 && zq == uq) ? cc : 0;
  };
  // wide group (> 255 entries): every bin straight from the exact index
  auto wide = [&](uint32_t gidx, uint32_t meta) {
    const uint32_t key = gidx & (NK2 - 1u);
    const int pi = (int)(gidx / pair_stride);
    const int p = spq[pi] & 0xFF, q = spq[pi] >> 8;
    const uint32_t *xo = xoff + (size_t)c * ((size_t)NK2 << 4);
    for (uint32_t b = 0; b < 16; ++b) {
      const int w = (meta & 16u) ? w2 + bin_corr(meta, b >> 2, b & 3u) : 0;
      if (!w) continue;
      const uint32_t z = pair_insert(key, K, p, q, b >> 2, b & 3u);
      const uint32_t e1 = xo[z + 1];
      for (uint32_t e = xo[z] + (uint32_t)gl; e < e1; e += G) atomicAdd(&acc[xent[e]], w);
    }
  };
  auto add = [&](uint32_t ad, int w) {
    __hip_atomic_fetch_add((__attribute__((address_space(3))) int32_t *)(uintptr_t)ad, w,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto process = [&](const uint4 &hdr, const uint4(&d)[MAXP], uint32_t nl, uint32_t gidx,
                     uint32_t meta) {
    if (nl == 0) return;
    const uint32_t hd[4] = {hdr.x, hdr.y, hdr.z, hdr.w};
    // wide marker (byte 14 = 0xFF, byte 15 = 0) or more lines than the lanes hold
    if ((hdr.w >> 16) == 0x00FFu || nl > (uint32_t)MAXNL) {
      wide(gidx, meta);
      return;
    }
    const int np = 2 * (int)nl;  // pieces of this lane; piece 0 of the group is the header
    // pieces [1, pe) hold the n entries (the last one padded with dummy columns): + w2 for
    // every halfword of them
    const int n = (int)(hdr.w >> 24);
    const int pe = min(np, ((n + 7) >> 3) + 1 - gl * np);  // this lane's live pieces: sp < pe
    const int p0 = gl == 0 ? 1 : 0;
#pragma unroll
    for (int sp = 0; sp < MAXP; ++sp) {
      if (!__any(sp < pe)) break;
      if (sp >= p0 && sp < pe) {
        const uint32_t wd[4] = {d[sp].x, d[sp].y, d[sp].z, d[sp].w};
#pragma unroll
        for (int v = 0; v < 8; ++v)
          add((v & 1) ? col_addr_sdwa<1>(wd[v >> 1]) : col_addr_sdwa<0>(wd[v >> 1]), w2);
      }
    }
    if (!__any(meta & 32u)) return;
    if (!(meta & 32u)) return;
    // corrections of a pair (0, r) list: row u_0 (minus / plus the exact bin) and, for
    // r = 1, the column bins (z_0 != u_0, z_1 = u_1)
    const int up = (int)(meta & 3u), uq = (int)((meta >> 2) & 3u), r = (int)(meta >> 8);
    const int t0 = 8 * gl * np - 8;  // entry index of the lane's first halfword
    const uint64_t rm = span_mask(bin_start(hd, 4 * up) - t0, bin_end(hd, 4 * up + 3) - t0);
    const uint64_t bm = span_mask(bin_start(hd, 4 * up + uq) - t0, bin_end(hd, 4 * up + uq) - t0);
    uint64_t cm = 0;
    if (r == 1) {
#pragma unroll
      for (int zp = 0; zp < 4; ++zp)
        if (zp != up) cm |= span_mask(bin_start(hd, 4 * zp + uq) - t0, bin_end(hd, 4 * zp + uq) - t0);
    }
    const int wb = r == 1 ? h0 : 0;
    const uint64_t any = rm | cm;
#pragma unroll
    for (int sp = 0; sp < MAXP; ++sp) {
      const uint32_t m8 = sp < np ? (uint32_t)(any >> (8 * sp)) & 0xFFu : 0u;
      if (!__any(m8 != 0u)) continue;
      const uint32_t wd[4] = {d[sp].x, d[sp].y, d[sp].z, d[sp].w};
#pragma unroll
      for (int v = 0; v < 8; ++v) {
        if (m8 & (1u << v)) {
          const int j = 8 * sp + v;
          const int w = ((bm >> j) & 1ull) ? wb : cc;
          if (w) add((v & 1) ? col_addr_sdwa<1>(wd[v >> 1]) : col_addr_sdwa<0>(wd[v >> 1]), w);
        }
      }
    }
  };

  // ring of D lists per lane group, unrolled so no loaded register is ever copied: slot r
  // holds the lines of its current list (loaded one round ago) and the summary of its next
  // list (loaded one round ago); per round and slot: atomics of the current list, decode
  // of the next list's summary + its line loads, then the summary load of the list after.
  uint4 dat[D][MAXP], hdr[D];
  uint32_t nl[D], gid[D], met[D], gidn[D], metn[D];
  uint2 swn[D];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    describe_next(gid[r], met[r]);
    swn[r] = load_summary(gid[r]);
  }
#pragma unroll
  for (int r = 0; r < D; ++r) {
    uint32_t base;
    decode(swn[r], gid[r], met[r], base, nl[r]);
    load_lines(base, nl[r], hdr[r], dat[r]);
  }
#pragma unroll
  for (int r = 0; r < D; ++r) {
    describe_next(gidn[r], metn[r]);
    swn[r] = load_summary(gidn[r]);
  }
  for (int L = grp; L < total; L += D * ngrp) {
#pragma unroll
    for (int r = 0; r < D; ++r) {
      process(hdr[r], dat[r], nl[r], gid[r], met[r]);
      uint32_t base;
      decode(swn[r], gidn[r], metn[r], base, nl[r]);
      gid[r] = gidn[r];
      met[r] = metn[r];
      load_lines(base, nl[r], hdr[r], dat[r]);
      describe_next(gidn[r], metn[r]);
      swn[r] = load_summary(gidn[r]);
    }
  }
  __syncthreads();

  const bool norm = o.normalize && o.diagv[0] != 1.0;
  emit_row<true>(o, il, i, col0, cw, (const int32_t *)acc, norm);
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

// raw self-kernel K_ii for every sequence (diagonal used by normalize_K), any max distance
__global__ __launch_bounds__(64) void diag_ham_kernel(IndexGeom g, Packed pk,
                                                      const int64_t *__restrict__ wtab,
                                                      double *__restrict__ diagv,
                                                      double *__restrict__ dsq) {
  __shared__ int64_t w_s[33];
  __shared__ uint32_t xk[4096];
  __shared__ uint32_t srec[1024];
  const int lane = threadIdx.x;
  const int64_t i = blockIdx.x;
  if (lane <= g.k) w_s[lane] = wtab[lane];
  stage_record(pk, i, srec);
  __syncthreads();
  const int P = min(g.pmax, 4096);
  for (int a = lane; a < P; a += 64) xk[a] = pk_window(srec, pk.cw, a, g.k);
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
// block, k-mers derived from the packed record in LDS; per lane only the histogram of
// distances 0..M2 is kept (int32) and weighted once at the end.  Same integer sum as
// diag_ham_kernel.
template <int M2>
__global__ __launch_bounds__(256) void diag_ham_small_kernel(IndexGeom g, Packed pk,
                                                             const int64_t *__restrict__ wtab,
                                                             double *__restrict__ diagv,
                                                             double *__restrict__ dsq) {
  extern __shared__ __align__(16) uint32_t xk_all[];  // [4][pmax] k-mers, then [4][ldp] records
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + wave;
  const bool valid = i < g.n;
  uint32_t *xk = xk_all + wave * g.pmax;
  uint32_t *srec = xk_all + 4 * g.pmax + wave * pk.ldp;
  const int P = g.pmax;
  if (valid) {
    const uint32_t *rec = pk.w + i * pk.ldp;
    for (int t = lane; t < (int)pk.ldp; t += 64) srec[t] = rec[t];
  }
  __syncthreads();
  if (valid)
    for (int a = lane; a < P; a += 64) xk[a] = pk_window(srec, pk.cw, a, g.k);
  __syncthreads();
  if (!valid) return;
  const uint32_t mask55 = (g.k >= 16) ? 0x55555555u : (0x55555555u & ((1u << (2 * g.k)) - 1u));
  // K_ii = sum_{a,b} w[ham(x_a, x_b)] is symmetric in (a, b): count b > a twice and a = b
  // once.  Lane l takes the windows a = l and a = P - 1 - l (and so on in strides of 128),
  // whose b > a tails add up to ~P iterations for every lane (half the work of the full
  // a x b square, no lane idling through a second, shorter stride)
  int cnt[M2 + 1];
#pragma unroll
  for (int d = 0; d <= M2; ++d) cnt[d] = 0;
  auto tail = [&](int a) {
    const uint32_t xa = xk[a];
    if (xa == KMG_INVALID) return;
    cnt[0] += 1;  // b = a
    for (int b = a + 1; b < P; ++b) {
      const uint32_t yb = xk[b];
      const int h = (yb == KMG_INVALID) ? 64 : ham2bit(xa, yb, mask55);
#pragma unroll
      for (int d = 0; d <= M2; ++d) cnt[d] += (h == d) ? 2 : 0;
    }
  };
  for (int a0 = 0; a0 < (P + 1) / 2; a0 += 64) {
    const int a = a0 + lane, a2 = P - 1 - a;
    if (a < (P + 1) / 2) {
      tail(a);
      if (a2 != a) tail(a2);
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
#define KMG_DISPATCH_DT(DT, ...)                       \
  switch (DT) {                                        \
    case KMG_I32: { constexpr int D = KMG_I32; __VA_ARGS__; } break; \
    case KMG_F32: { constexpr int D = KMG_F32; __VA_ARGS__; } break; \
    default: { constexpr int D = KMG_F64; __VA_ARGS__; } break;      \
  }

// ------------------------------------------------------------------ multi-GPU assembly
// One pass over the round slab S (R rows x w columns; row y = K row c0 + y at columns >= c0):
// a 64 x 64 tile of S is read once (coalesced rows), written to K's rows c0 + y at columns
// c0 + j (upper part, coalesced) and, for j >= R (K rows below the round), transposed from
// LDS into K[c0 + j][c0 + y] (the mirror, coalesced along y).  Rows of S at or past n - c0
// (padding of the last round) are skipped.
template <typename T>
__global__ __launch_bounds__(256) void tri_unpack_kernel(const T *__restrict__ S, int64_t w,
                                                         int64_t R, int64_t c0, int64_t n,
                                                         T *__restrict__ K, int64_t ld) {
  __shared__ T tile[64][65];
  const int64_t j0 = (int64_t)blockIdx.x * 64;  // S column (K column / mirror row c0 + j)
  const int64_t y0 = (int64_t)blockIdx.y * 64;  // S row (K row / mirror column c0 + y)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t yend = min(R, n - c0);
  for (int r = wv; r < 64; r += 4) {
    const int64_t y = y0 + r, j = j0 + lane;
    if (y < yend && j < w) {
      const T v = S[y * w + j];
      K[(c0 + y) * ld + c0 + j] = v;
      tile[r][lane] = v;
    }
  }
  if (j0 + 64 <= R) return;  // no column of this tile lies below the round (block-uniform)
  __syncthreads();
  for (int r = wv; r < 64; r += 4) {
    const int64_t j = j0 + r, y = y0 + lane;
    if (j >= R && j < w && y < yend) K[(c0 + j) * ld + c0 + y] = tile[lane][r];
  }
}

// The same assembly from a uint16 slab of raw counts, widened to K's dtype on the way, as
// two streaming passes with 16-byte accesses on both sides: (1) rows — K[c0 + y][c0 + j] =
// S[y][j], 8 columns a thread; (2) mirror — 64 x 64 tiles of S[:, R:] through LDS into
// K[c0 + j][c0 + y0 .. + 64) (256 / 512 contiguous bytes per output row).  With
// normalisation every element is K_ij / (sqrt(K_ii) * sqrt(K_jj)), diagonal 1: the Gram
// kernels' fused epilogue (emit4 / emit_row) bit for bit, and symmetric because the
// product of the two square roots is commutative.  (The round-2 single-pass 64 x 64 kernel
// with 4-byte accesses moved ~3.3 TB/s.)
template <typename TO>
__device__ __forceinline__ TO widen16(uint32_t v, int64_t gr, int64_t gc, bool norm,
                                      const double *__restrict__ dsq) {
  if constexpr (std::is_same<TO, int32_t>::value) {
    return (int32_t)v;
  } else {
    const double d = !norm ? (double)v : (gr == gc) ? 1.0 : (double)v / (dsq[gr] * dsq[gc]);
    return (TO)d;
  }
}

template <typename TO>
__device__ __forceinline__ void store_out(TO *p, const TO (&v)[16 / sizeof(TO)]) {
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i x;
  __builtin_memcpy(&x, v, 16);
  *(v4i *)p = x;
}

// 8 slab elements of type TI (uint16 / uint8) from src, vector load when aligned
template <typename TI>
__device__ __forceinline__ void load8(const TI *src, int cnt, uint32_t (&v)[8]) {
  if constexpr (sizeof(TI) == 2) {
    if (cnt == 8 && (((uintptr_t)src) & 15) == 0) {
      const uint4 x = *(const uint4 *)src;
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int h = 0; h < 8; ++h) v[h] = (xs[h >> 1] >> (16 * (h & 1))) & 0xFFFFu;
      return;
    }
  } else {
    if (cnt == 8 && (((uintptr_t)src) & 7) == 0) {
      const uint2 x = *(const uint2 *)src;
#pragma unroll
      for (int h = 0; h < 8; ++h) v[h] = ((h < 4 ? x.x : x.y) >> (8 * (h & 3))) & 0xFFu;
      return;
    }
  }
#pragma unroll
  for (int h = 0; h < 8; ++h) v[h] = h < cnt ? (uint32_t)src[h] : 0u;
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void tri_rows16_kernel(const TI *__restrict__ S, int64_t w,
                                                         int64_t yend, int64_t c0,
                                                         TO *__restrict__ K, int64_t ld,
                                                         int normalize,
                                                         const double *__restrict__ diagv,
                                                         const double *__restrict__ dsq) {
  constexpr int V = 16 / (int)sizeof(TO);  // outputs per 16-byte store
  const int64_t per_row = (w + 7) >> 3;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per_row * yend) return;
  const bool norm = normalize && diagv[0] != 1.0;
  const int64_t y = t / per_row, j = (t - y * per_row) * 8;
  const TI *src = S + y * w + j;
  const int64_t gr = c0 + y, gc = c0 + j;
  TO *dst = K + gr * ld + gc;
  const int cnt = (int)min((int64_t)8, w - j);
  uint32_t v[8];
  load8<TI>(src, cnt, v);
  if constexpr (sizeof(TI) == 1) {  // 8-bit slabs leave the diagonal out: K_ii from diagv
#pragma unroll
    for (int h = 0; h < 8; ++h)
      if (gc + h == gr) v[h] = (uint32_t)diagv[gr];
  }
  if (cnt == 8 && (((uintptr_t)dst) & 15) == 0) {
#pragma unroll
    for (int b = 0; b < 8; b += V) {
      TO o[V];
#pragma unroll
      for (int q = 0; q < V; ++q) o[q] = widen16<TO>(v[b + q], gr, gc + b + q, norm, dsq);
      store_out<TO>(dst + b, o);
    }
  } else {
    for (int h = 0; h < cnt; ++h) dst[h] = widen16<TO>(v[h], gr, gc + h, norm, dsq);
  }
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void tri_mirror16_kernel(const TI *__restrict__ S, int64_t w,
                                                           int64_t R, int64_t yend, int64_t c0,
                                                           TO *__restrict__ K, int64_t ld,
                                                           int normalize,
                                                           const double *__restrict__ diagv,
                                                           const double *__restrict__ dsq) {
  constexpr int V = 16 / (int)sizeof(TO);
  __shared__ uint32_t tile[64][65];  // [y][j]
  const int64_t j0 = R + (int64_t)blockIdx.x * 64;  // S column of the tile (>= R)
  const int64_t y0 = (int64_t)blockIdx.y * 64;
  const bool norm = normalize && diagv[0] != 1.0;
  // load: 64 rows x 8 chunks of 8 columns
  for (int c = threadIdx.x; c < 512; c += blockDim.x) {
    const int r = c >> 3, q8 = (c & 7) * 8;
    const int64_t y = y0 + r, j = j0 + q8;
    uint32_t v[8];
    const TI *src = S + y * w + j;
    if (y < yend && j < w) {
      load8<TI>(src, (int)min((int64_t)8, w - j), v);
    } else {
#pragma unroll
      for (int h = 0; h < 8; ++h) v[h] = 0u;
    }
#pragma unroll
    for (int h = 0; h < 8; ++h) tile[r][q8 + h] = v[h];
  }
  __syncthreads();
  // store: output row c0 + j0 + jj, columns c0 + y0 + [0, 64): 64 / V chunks of 16 bytes
  constexpr int CPR = 64 / V;
  for (int c = threadIdx.x; c < 64 * CPR; c += blockDim.x) {
    const int jj = c / CPR, yy = (c - jj * CPR) * V;
    const int64_t j = j0 + jj;
    if (j >= w) continue;
    const int64_t gr = c0 + j, gc = c0 + y0 + yy;
    TO *dst = K + gr * ld + gc;
    const int cnt = (int)min((int64_t)V, yend - (y0 + yy));
    if (cnt <= 0) continue;
    TO o[V];
#pragma unroll
    for (int q = 0; q < V; ++q) o[q] = widen16<TO>(tile[yy + q][jj], gr, gc + q, norm, dsq);
    if (cnt == V && (((uintptr_t)dst) & 15) == 0) {
      store_out<TO>(dst, o);
    } else {
      for (int q = 0; q < cnt; ++q) dst[q] = o[q];
    }
  }
}

hipError_t launch_tri_unpack16(const uint16_t *S, int64_t w, int64_t R, int64_t c0, int64_t n,
                               void *K, int64_t ld, int dt, int normalize, const double *diagv,
                               const double *dsq, hipStream_t s) {
  if (w <= 0 || R <= 0 || c0 >= n) return hipSuccess;
  if (normalize && (!diagv || !dsq)) return hipErrorInvalidValue;
  const int64_t yend = std::min(R, n - c0);
  const int64_t items = ((w + 7) >> 3) * yend;
  const dim3 g1((unsigned)((items + 255) / 256));
  const bool mir = w > R;
  const dim3 g2((unsigned)(mir ? (w - R + 63) / 64 : 0), (unsigned)((yend + 63) / 64));
  if (g2.y > 65535u || (items + 255) / 256 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
#define KMG_UNPACK(T)                                                                            \
  do {                                                                                           \
    hipLaunchKernelGGL((tri_rows16_kernel<uint16_t, T>), g1, dim3(256), 0, s, S, w, yend, c0,    \
                       (T *)K, ld, dt == KMG_I32 ? 0 : normalize, diagv, dsq);                   \
    if (mir)                                                                                     \
      hipLaunchKernelGGL((tri_mirror16_kernel<uint16_t, T>), g2, dim3(256), 0, s, S, w, R, yend, \
                         c0, (T *)K, ld, dt == KMG_I32 ? 0 : normalize, diagv, dsq);             \
  } while (0)
  if (dt == KMG_I32)
    KMG_UNPACK(int32_t);
  else if (dt == KMG_F32)
    KMG_UNPACK(float);
  else if (dt == KMG_F64)
    KMG_UNPACK(double);
  else
    return hipErrorInvalidValue;
#undef KMG_UNPACK
  return hipGetLastError();
}

// escapes of uint8 round slabs: one thread per (list, entry); K[r][c] and its mirror
// K[c][r] get the count widened exactly as tri_rows16_kernel / tri_mirror16_kernel widen
// slab values (normalize_K's formula for normalised output)
template <typename TO>
__global__ __launch_bounds__(256) void tri_patch8_kernel(const uint4 *__restrict__ esc,
                                                         const uint32_t *__restrict__ counts,
                                                         int64_t stride, int64_t max_count,
                                                         TO *__restrict__ K, int64_t ld,
                                                         int normalize,
                                                         const double *__restrict__ diagv,
                                                         const double *__restrict__ dsq) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int set = (int)blockIdx.y;
  const int64_t cnt = min((int64_t)counts[set], min(stride, max_count));
  if (t >= cnt) return;
  const bool norm = normalize && diagv[0] != 1.0;
  const uint4 e = esc[(int64_t)set * stride + t];
  const int64_t r = e.x, c = e.y;
  K[r * ld + c] = widen16<TO>(e.z, r, c, norm, dsq);
  K[c * ld + r] = widen16<TO>(e.z, c, r, norm, dsq);
}

hipError_t launch_tri_patch8(const uint4 *esc, const uint32_t *counts, int nsets, int64_t stride,
                             int64_t max_count, void *K, int64_t ld, int dt, int normalize,
                             const double *diagv, const double *dsq, hipStream_t s) {
  const int64_t m = std::min(stride, max_count);
  if (nsets <= 0 || m <= 0) return hipSuccess;
  if (!diagv || (normalize && !dsq) || nsets > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((m + 255) / 256), (unsigned)nsets);
  if (dt == KMG_I32)
    hipLaunchKernelGGL((tri_patch8_kernel<int32_t>), grid, dim3(256), 0, s, esc, counts, stride,
                       max_count, (int32_t *)K, ld, 0, diagv, dsq);
  else if (dt == KMG_F32)
    hipLaunchKernelGGL((tri_patch8_kernel<float>), grid, dim3(256), 0, s, esc, counts, stride,
                       max_count, (float *)K, ld, normalize, diagv, dsq);
  else
    hipLaunchKernelGGL((tri_patch8_kernel<double>), grid, dim3(256), 0, s, esc, counts, stride,
                       max_count, (double *)K, ld, normalize, diagv, dsq);
  return hipGetLastError();
}

hipError_t launch_tri_unpack8(const uint8_t *S, int64_t w, int64_t R, int64_t c0, int64_t n,
                              void *K, int64_t ld, int dt, int normalize, const double *diagv,
                              const double *dsq, hipStream_t s) {
  if (w <= 0 || R <= 0 || c0 >= n) return hipSuccess;
  if (!diagv || (normalize && !dsq)) return hipErrorInvalidValue;
  const int64_t yend = std::min(R, n - c0);
  const int64_t items = ((w + 7) >> 3) * yend;
  const dim3 g1((unsigned)((items + 255) / 256));
  const bool mir = w > R;
  const dim3 g2((unsigned)(mir ? (w - R + 63) / 64 : 0), (unsigned)((yend + 63) / 64));
  if (g2.y > 65535u || (items + 255) / 256 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
#define KMG_UNPACK8(T)                                                                           \
  do {                                                                                           \
    hipLaunchKernelGGL((tri_rows16_kernel<uint8_t, T>), g1, dim3(256), 0, s, S, w, yend, c0,     \
                       (T *)K, ld, dt == KMG_I32 ? 0 : normalize, diagv, dsq);                   \
    if (mir)                                                                                     \
      hipLaunchKernelGGL((tri_mirror16_kernel<uint8_t, T>), g2, dim3(256), 0, s, S, w, R, yend,  \
                         c0, (T *)K, ld, dt == KMG_I32 ? 0 : normalize, diagv, dsq);             \
  } while (0)
  if (dt == KMG_I32)
    KMG_UNPACK8(int32_t);
  else if (dt == KMG_F32)
    KMG_UNPACK8(float);
  else if (dt == KMG_F64)
    KMG_UNPACK8(double);
  else
    return hipErrorInvalidValue;
#undef KMG_UNPACK8
  return hipGetLastError();
}

hipError_t launch_tri_unpack(const void *S, int64_t w, int64_t R, int64_t c0, int64_t n, void *K,
                             int64_t ld, int esz, hipStream_t s) {
  if (w <= 0 || R <= 0 || c0 >= n) return hipSuccess;
  const int64_t ry = std::min(R, n - c0);
  const dim3 grid((unsigned)((w + 63) / 64), (unsigned)((ry + 63) / 64));
  if (grid.y > 65535u) return hipErrorInvalidValue;
  if (esz == 8)
    hipLaunchKernelGGL(tri_unpack_kernel<uint64_t>, grid, dim3(256), 0, s, (const uint64_t *)S, w,
                       R, c0, n, (uint64_t *)K, ld);
  else
    hipLaunchKernelGGL(tri_unpack_kernel<uint32_t>, grid, dim3(256), 0, s, (const uint32_t *)S, w,
                       R, c0, n, (uint32_t *)K, ld);
  return hipGetLastError();
}

// In-place mirror of a full square K built with OutSpec::tri: K[i][j] = K[j][i] for every
// j < (i / chunk) * chunk, the blocks left of row i's own column chunk that the mismatch
// kernels skipped (rowacc_block).  Row j < (i / chunk) * chunk did compute column i (its
// own chunk is left of i's), so every source entry exists.  64 x 64 tiles through LDS: the
// source K[j0.., i0..] is read along its rows and the target K[i0.., j0..] written along
// its rows, 16 bytes per lane each way.
template <typename T>
__global__ __launch_bounds__(256) void mirror_chunks_kernel(T *__restrict__ K, int64_t ld,
                                                            int64_t n, int chunk, int64_t ti0) {
  constexpr int V = 16 / (int)sizeof(T), CPR = 64 / V;
  __shared__ T tile[64][64 + 1];  // [j - j0][i - i0]
  const int64_t i0 = (ti0 + (int64_t)blockIdx.y) * 64, j0 = (int64_t)blockIdx.x * 64;
  const int64_t imax = min(n - 1, i0 + 63);
  if (j0 >= (imax / chunk) * chunk) return;  // no target entry in this tile
  for (int c = threadIdx.x; c < 64 * CPR; c += blockDim.x) {
    const int r = c / CPR, q = (c - r * CPR) * V;
    const int64_t j = j0 + r, i = i0 + q;
    if (j >= n) continue;
    const T *src = K + j * ld + i;
    if (i + V <= n && (((uintptr_t)src) & 15) == 0) {
      const uint4 x = *(const uint4 *)src;
      const T *v = (const T *)&x;
#pragma unroll
      for (int h = 0; h < V; ++h) tile[r][q + h] = v[h];
    } else {
      for (int h = 0; h < V && i + h < n; ++h) tile[r][q + h] = src[h];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 64 * CPR; c += blockDim.x) {
    const int r = c / CPR, q = (c - r * CPR) * V;
    const int64_t i = i0 + r, j = j0 + q;
    if (i >= n) continue;
    const int64_t cs = (i / chunk) * chunk;
    if (j >= cs) continue;
    T o[V];
#pragma unroll
    for (int h = 0; h < V; ++h) o[h] = tile[q + h][r];
    T *dst = K + i * ld + j;
    if (j + V <= cs && (((uintptr_t)dst) & 15) == 0) {
      *(uint4 *)dst = *(const uint4 *)o;
    } else {
      for (int h = 0; h < V && j + h < cs; ++h) dst[h] = o[h];
    }
  }
}

hipError_t launch_mirror_chunks(void *K, int64_t ld, int64_t n, int chunk, int esz,
                                hipStream_t s) {
  if (n <= chunk) return hipSuccess;
  if (esz != 8 && esz != 4) return hipErrorInvalidValue;
  if ((n + 63) / 64 > 65535) return hipErrorInvalidValue;
  // one launch per row chunk c >= 1: its 64-row tiles x the column tiles left of c * chunk
  // (a square grid over all tile pairs would start ~57 % of its blocks only to leave)
  for (int64_t c0 = chunk; c0 < n; c0 += chunk) {
    const int64_t ti0 = c0 / 64, ti1 = (std::min(n, c0 + chunk) + 63) / 64;
    const dim3 grid((unsigned)((c0 + 63) / 64), (unsigned)(ti1 - ti0));
    if (esz == 8)
      hipLaunchKernelGGL(mirror_chunks_kernel<uint64_t>, grid, dim3(256), 0, s, (uint64_t *)K, ld,
                         n, chunk, ti0);
    else
      hipLaunchKernelGGL(mirror_chunks_kernel<uint32_t>, grid, dim3(256), 0, s, (uint32_t *)K, ld,
                         n, chunk, ti0);
  }
  return hipGetLastError();
}

// Column-block assembly (kmg_gram_blocks gather 5 / 6): a rank's column block K[:, C] (n
// rows x w columns) is, K being symmetric, its row slab K[C, :] stored column-major; this
// copies it into the slab's rows of K.  One 64 x 64 tile a workgroup: read along the block's
// rows, written along K's rows, 16 bytes a lane each way (as mirror_chunks_kernel).
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T *__restrict__ M, int64_t ldm,
                                                        int64_t rows, int64_t w,
                                                        T *__restrict__ K, int64_t ldk) {
  constexpr int V = 16 / (int)sizeof(T), CPR = 64 / V;
  __shared__ T tile[64][64 + 1];  // [i - i0][j - j0]
  const int64_t j0 = (int64_t)blockIdx.x * 64, i0 = (int64_t)blockIdx.y * 64;
  for (int c = threadIdx.x; c < 64 * CPR; c += blockDim.x) {
    const int r = c / CPR, q = (c - r * CPR) * V;
    const int64_t i = i0 + r, j = j0 + q;
    if (i >= rows || j >= w) continue;
    const T *src = M + i * ldm + j;
    if (j + V <= w && (((uintptr_t)src) & 15) == 0) {
      const uint4 x = *(const uint4 *)src;
      const T *v = (const T *)&x;
#pragma unroll
      for (int h = 0; h < V; ++h) tile[r][q + h] = v[h];
    } else {
      for (int h = 0; h < V && j + h < w; ++h) tile[r][q + h] = src[h];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 64 * CPR; c += blockDim.x) {
    const int r = c / CPR, q = (c - r * CPR) * V;
    const int64_t j = j0 + r, i = i0 + q;  // K row j, columns i ..
    if (j >= w || i >= rows) continue;
    T o[V];
#pragma unroll
    for (int h = 0; h < V; ++h) o[h] = tile[q + h][r];
    T *dst = K + j * ldk + i;
    if (i + V <= rows && (((uintptr_t)dst) & 15) == 0) {
      *(uint4 *)dst = *(const uint4 *)o;
    } else {
      for (int h = 0; h < V && i + h < rows; ++h) dst[h] = o[h];
    }
  }
}

hipError_t launch_transpose(const void *M, int64_t ldm, int64_t rows, int64_t w, void *K,
                            int64_t ldk, int esz, hipStream_t s) {
  if (rows <= 0 || w <= 0) return hipSuccess;
  if (esz != 8 && esz != 4) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((w + 63) / 64), (unsigned)((rows + 63) / 64));
  if ((rows + 63) / 64 > 65535 || (w + 63) / 64 > 0x7FFFFFFFLL) return hipErrorInvalidValue;
  if (esz == 8)
    hipLaunchKernelGGL(transpose_kernel<uint64_t>, grid, dim3(256), 0, s, (const uint64_t *)M, ldm,
                       rows, w, (uint64_t *)K, ldk);
  else
    hipLaunchKernelGGL(transpose_kernel<uint32_t>, grid, dim3(256), 0, s, (const uint32_t *)M, ldm,
                       rows, w, (uint32_t *)K, ldk);
  return hipGetLastError();
}

hipError_t launch_gram_spectrum(const IndexGeom &g, const Packed &pk, const uint32_t *off,
                                const uint16_t *ent, int64_t row0, int64_t row1, const OutSpec &o,
                                hipStream_t s, int store, int order, int rows_per) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (o.tri) return hipErrorInvalidValue;  // (the spectrum grid has its own row orders)
  const int64_t nblk = rowacc_blocks(g, o, row0, rows);
  if (nblk * 1024 >= (1LL << 32)) return hipErrorInvalidValue;  // AQL grid size is 32-bit
  const bool pack = g.pmax <= 255;
  const int words = pack ? (((g.chunk + 7) >> 3) << 2) : (((g.chunk + 3) >> 2) << 2);
  // rows a workgroup (KMG_SP_ROWS 0 auto, 2 or 4): full-width dtypes, all accumulators in LDS
  if (rows_per == 0) rows_per = g.chunk <= 16384 ? 2 : 1;  // auto (kmg_api.cpp Tuning::sp_rows)
  int rpw = (rows_per == 2 || rows_per == 4) && o.dtype != KMG_U16 && o.dtype != KMG_U8 ? rows_per : 1;
  while (rpw > 1 && (size_t)rpw * words * 4 > 160 * 1024) rpw >>= 1;
  const size_t lds = (size_t)words * 4 * rpw;
  const int64_t nb = rpw > 1 ? ((rows + rpw - 1) / rpw) * g.nchunks : nblk;
  const dim3 grid((unsigned)nb);
  // store policy: 0 auto (plain for a single-chunk int32 K, else non-temporal), 1 NT, 2 plain
  const bool nt = store == 1 || (store == 0 && !(o.dtype == KMG_I32 && g.nchunks == 1));
  const int cmj = (order == 1 && g.nchunks > 1) ? 1 : 0;
  if (o.dtype == KMG_U16 || o.dtype == KMG_U8) {  // raw round slab (kmg_gram_blocks)
    if (!pack) return hipErrorInvalidValue;
    if (o.dtype == KMG_U16)
      hipLaunchKernelGGL((gram_sp_kernel<true, KMG_U16, false, 1>), grid, dim3(1024), lds, s, g, pk,
                         off, ent, row0, rows, cmj, o);
    else
      hipLaunchKernelGGL((gram_sp_kernel<true, KMG_U8, false, 1>), grid, dim3(1024), lds, s, g, pk,
                         off, ent, row0, rows, cmj, o);
    return hipGetLastError();
  }
#define KMG_SP(PK, NTV, R)                                                                        \
  KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_sp_kernel<PK, D, NTV, R>), grid, dim3(1024),  \
                                              lds, s, g, pk, off, ent, row0, rows, cmj, o))
#define KMG_SP_R(R)                                                                    \
  if (pack) {                                                                          \
    if (nt) { KMG_SP(true, true, R); } else { KMG_SP(true, false, R); }                \
  } else {                                                                             \
    if (nt) { KMG_SP(false, true, R); } else { KMG_SP(false, false, R); }              \
  }
  if (rpw == 4) {
    KMG_SP_R(4)
  } else if (rpw == 2) {
    KMG_SP_R(2)
  } else {
    KMG_SP_R(1)
  }
#undef KMG_SP_R
#undef KMG_SP
  return hipGetLastError();
}

hipError_t launch_gram_mismatch1_slots(const IndexGeom &g, const Packed &pk, const uint4 *slots,
                                       const uint32_t *off, const uint16_t *ent, int64_t row0,
                                       int64_t row1, int w0, int w1, int w2, const OutSpec &o,
                                       hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (g.k < 8 || g.k > 12 || !g.rot) return hipErrorNotSupported;
  if (w0 > 255 || w1 > 255 || w2 > 255) return hipErrorNotSupported;
  const int64_t nblk = rowacc_blocks(g, o, row0, rows);
  if (nblk * 1024 >= (1LL << 32)) return hipErrorInvalidValue;  // AQL grid size is 32-bit
  const int nsub = g.k + 3 * g.k * (g.k - 1) / 2;
  const size_t lds = (size_t)((((g.chunk + 3) >> 2) << 2) + g.pmax * g.k + nsub + pk.ldp) * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk);
  switch (g.k) {
#define KMG_MM(KK)                                                                               \
  case KK:                                                                                       \
    hipLaunchKernelGGL((gram_mm1_kernel<KK, 2>), grid, dim3(1024), lds, s, g, pk, slots, off,    \
                       ent, row0, rows, w0, w1, w2, o);                                          \
    break;
    KMG_MM(8) KMG_MM(9) KMG_MM(10) KMG_MM(11) KMG_MM(12)
#undef KMG_MM
  }
  return hipGetLastError();
}

hipError_t launch_gram_mismatch1_pairs(const PairGeom &pg, const IndexGeom &g, const Packed &pk,
                                       const uint32_t *summary, const uint4 *lines,
                                       int64_t nlines, const uint32_t *xoff, const uint16_t *xent,
                                       int64_t row0, int64_t row1, int w0, int w1, int w2,
                                       const OutSpec &o, hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (pg.k < 3 || pg.k > 12 || pg.k != g.k) return hipErrorNotSupported;
  const int64_t nblk = rowacc_blocks(g, o, row0, rows);
  if (nblk * 1024 >= (1LL << 32)) return hipErrorInvalidValue;  // AQL grid size is 32-bit
  if (nlines * 128 >= 0xFFFFFFF0LL) return hipErrorInvalidValue;  // 32-bit buffer offsets
  const size_t lds = (size_t)((((g.chunk + 3) >> 2) << 2) + 64 + g.pmax + pk.ldp + KMG_PAIRS_MAX) * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk);
  const uint32_t lb = (uint32_t)(nlines * 128);
  switch (pg.k) {
#define KMG_MM2(KK)                                                                               \
  case KK:                                                                                        \
    hipLaunchKernelGGL((gram_mm2_kernel<KK, 2>), grid, dim3(1024), lds, s, pg, g, pk, summary, lines, \
                       lb, xoff, xent, row0, rows, w0, w1, w2, o);                                \
    break;
    KMG_MM2(3) KMG_MM2(4) KMG_MM2(5) KMG_MM2(6) KMG_MM2(7) KMG_MM2(8) KMG_MM2(9) KMG_MM2(10)
    KMG_MM2(11) KMG_MM2(12)
#undef KMG_MM2
  }
  return hipGetLastError();
}

hipError_t launch_gram_hamming(const IndexGeom &g, const uint32_t *kmers, int64_t row0,
                               int64_t row1, const int64_t *wtab, const OutSpec &o,
                               hipStream_t s) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (rows > 65535) return hipErrorInvalidValue;  // grid.y
  const dim3 grid((unsigned)((g.n + 63) / 64), (unsigned)rows);
  KMG_DISPATCH_DT(o.dtype, hipLaunchKernelGGL((gram_ham_kernel<D>), grid, dim3(256), 0, s, g,
                                              kmers, row0, wtab, o));
  return hipGetLastError();
}

hipError_t launch_diag_hamming(const IndexGeom &g, const Packed &pk, const int64_t *wtab,
                               int max_dist, double *diagv, double *dsq, hipStream_t s) {
  if (g.n == 0) return hipSuccess;
  if (pk.ldp > 1024) return hipErrorInvalidValue;
  if (max_dist <= 4 && g.pmax <= 4096) {
    const dim3 grid((unsigned)((g.n + 3) / 4));
    const size_t lds = (size_t)4 * (g.pmax + pk.ldp) * sizeof(uint32_t);
#define KMG_DIAG(M2_)                                                                          \
  case M2_:                                                                                    \
    hipLaunchKernelGGL((diag_ham_small_kernel<M2_>), grid, dim3(256), lds, s, g, pk, wtab,      \
                       diagv, dsq);                                                            \
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
  hipLaunchKernelGGL(diag_ham_kernel, dim3((unsigned)g.n), dim3(64), 0, s, g, pk, wtab, diagv, dsq);
  return hipGetLastError();
}

}  // namespace kmg
