// kmg_nbhd.hip — mismatch (k, 1) Gram through NEIGHBOURHOOD LISTS (gfx950).
//
// get_mismatch_K (kernels.py:196-217) reduces to the closed form
//   K(x, y) = sum_{a, b} w[ham(x_a, y_b)],  w = (1 + 3k, 4, 2) for m = 1
// (kmgram.params.mismatch_weights), i.e. for row i's window k-mer u every column window at
// Hamming distance <= 2 of u adds w[ham] to its column.  The drop-one slot table and the
// drop-two pair lines (kmg_gram.hip, kmg_pairs.hip) read those column windows as many
// short posting groups (117 or 36 random 128-byte lines a window and chunk, 1.6-2x the
// entries a window needs: a Hamming-1 neighbour sits in k - 1 pair groups, Hamming 0 in all
// of them).  This formulation materialises, once per build, for every (column chunk c,
// k-mer u) the NEIGHBOURHOOD LIST of u:
//
//   [ occurrences of u | of its 3k Hamming-1 neighbours | of its 9 k(k-1)/2 Hamming-2 ]
//
// as uint16 columns inside the chunk, each of the three segments padded to whole 16-byte
// pieces (8 columns) with dummy columns (LDS words past the accumulator).  Every column
// window then appears exactly once per list, and a row window reads ONE contiguous list
// (N=200000, k=9: ~25000 entries, 50 KB over all chunks) instead of 117 random lines per
// chunk: the Gram kernel streams HBM, 16 bytes a lane, 1 KB per wave instruction.
//
//   nb_count_kernel   per (c, u): n0, n1, n2 from the exact index (1 + 3k + 9k(k-1)/2
//                     lookups of its bin offsets, L2-resident) -> pieces and segment ends
//   launch_scan       list starts (in pieces; < 2^32: checked by the host)
//   list fills        (launch_nb_fill picks one)
//     nb_fill_grouped_kernel  default: one workgroup per 16 k-mers sharing a (k-2)-letter
//                     prefix, the 211 prefix ranges' sub-bin offsets in LDS; one wave a list:
//                     DPP prefix sum of its 352 runs, lane-per-run copies from the index
//     nb_fill_pieces_kernel   past 8.5 occurrences a k-mer and chunk: the ranges as an LDS
//                     image (16-byte loads), each list assembled 16 bytes a lane from it
//     nb_fill_kernel, nb_fill_ranges_kernel   the per-list and range-major forms (measured
//                     slower; KMG_NB_FILL 1 / 6)
//   gram_nb_kernel   per (row i, chunk c): row windows -> (list start, pieces, segment
//                     ends) in LDS, a prefix sum over the row's lists, then every wave streams
//                     an equal share of the row's pieces (four 16-byte loads in flight per
//                     lane), adding the segment's weight for each of the 8 columns of a piece
//                     into the LDS accumulator; fused normalize_K epilogue (emit_row).
//
// Roofline: the lists are read from HBM once per (row, chunk) -- 2 B per (row window,
// neighbour occurrence): N=20000 ~466 KB a row against the 160 KB float64 K row; the bound is
// HBM (table reads + K writes), not the Infinity-Cache line rate of the table formulations.
#include "kmg_rowacc.h"

namespace kmg {

namespace {
constexpr int NB_FILL_THREADS = 256;

__device__ __forceinline__ int nb_neighbours(int k) { return 1 + 3 * k + 9 * k * (k - 1) / 2; }

// neighbour t of u (t < nb_neighbours(k)) and its segment: t = 0 u itself; then the 3k
// Hamming-1 k-mers (position p, letter xor d = 1..3); then the Hamming-2 k-mers of the pairs
// p < q in order (0,1), (0,2), (1,2), (0,3), ... (q-major), 9 letter xors each
__device__ __forceinline__ uint32_t nb_neighbour(uint32_t u, int k, int t, int &seg) {
  if (t == 0) {
    seg = 0;
    return u;
  }
  t -= 1;
  if (t < 3 * k) {
    seg = 1;
    const int p = t / 3, d = t - 3 * p + 1;
    return u ^ ((uint32_t)d << (2 * (k - 1 - p)));
  }
  seg = 2;
  t -= 3 * k;
  const int pi = t / 9, r = t - 9 * pi;
  int q = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)pi)) * 0.5f);  // pi = q(q-1)/2 + p
  while (q * (q - 1) / 2 > pi) --q;
  while ((q + 1) * q / 2 <= pi) ++q;
  const int p = pi - q * (q - 1) / 2;
  const int d1 = r / 3 + 1, d2 = r - 3 * (r / 3) + 1;
  return u ^ ((uint32_t)d1 << (2 * (k - 1 - p))) ^ ((uint32_t)d2 << (2 * (k - 1 - q)));
}

// the same inclusive wave scan on DPP row shifts and row broadcasts (VALU only, no LDS
// permutes): Hillis-Steele inside each 16-lane row, then lane 15 into row 1 (and 47 into row
// 3), then lane 31 into rows 2 and 3
__device__ __forceinline__ uint32_t nb_wave_incl_scan_dpp(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return (uint32_t)x;
}

__device__ __forceinline__ uint32_t nb_wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}
}  // namespace

// per (chunk, k-mer): pieces of its neighbourhood list and the segment ends (in pieces)
__global__ __launch_bounds__(256) void nb_count_kernel(int k, int64_t nbins,
                                                       const uint32_t *__restrict__ xoff,
                                                       uint32_t *__restrict__ hist,
                                                       uint2 *__restrict__ seg) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nbins) return;
  const uint32_t nkeys = 1u << (2 * k);
  const uint32_t u = (uint32_t)b & (nkeys - 1u);
  const uint32_t *off = xoff + (b - u);
  auto cnt = [&](uint32_t v) { return off[v + 1] - off[v]; };
  const uint32_t n0 = cnt(u);
  uint32_t n1 = 0, n2 = 0;
  for (int p = 0; p < k; ++p) {
    const int sp = 2 * (k - 1 - p);
#pragma unroll
    for (uint32_t d = 1; d <= 3; ++d) n1 += cnt(u ^ (d << sp));
    for (int q = p + 1; q < k; ++q) {
      const int sq = 2 * (k - 1 - q);
#pragma unroll
      for (uint32_t d1 = 1; d1 <= 3; ++d1)
#pragma unroll
        for (uint32_t d2 = 1; d2 <= 3; ++d2) n2 += cnt(u ^ (d1 << sp) ^ (d2 << sq));
    }
  }
  const uint32_t p0 = (n0 + 7) >> 3, p1 = (n1 + 7) >> 3, p2 = (n2 + 7) >> 3;
  hist[b] = p0 + p1 + p2;
  seg[b] = make_uint2(p0, p0 + p1);
}

// One WAVE per (chunk, k-mer) bin, four waves a workgroup, grid-stride over the bins.
//  1. lane l owns the neighbours t in [l R, l R + R) (R = ceil(nb / 64)): their posting
//     ranges (all loads issued before any is used), a wave prefix sum gives each run's start
//     in the unpadded concatenation; starts and sources go to the wave's LDS tables;
//  2. the runs are copied by groups of LG lanes, one run a group (LG ~ the mean run length:
//     chunk x P / 4^k occurrences of a k-mer, 7 at N=20000 and k = 9), 64 / LG runs a step
//     and NB_STEPS steps' loads in flight; the runs of a step are consecutive in the list, so
//     a wave's 2-byte stores land on ~128 contiguous bytes.
// (Round 4's first forms -- a workgroup per bin with one dependent load per copied entry,
// and an entry-parallel copy through an LDS run map, ~60 VALU per entry -- took 1.7-3.0 ms
// per 262144 bins at N=20000.)
constexpr int NB_MAXR = 10;    // neighbours a lane in step 1: ceil(631 / 64) at k = 12
constexpr int NB_MAXN = 640;   // neighbour tables per wave (631 at k = 12, + the end)
constexpr int NB_STEPS = 8;

template <int LG>
__global__ __launch_bounds__(NB_FILL_THREADS) void nb_fill_kernel(
    int k, int64_t nbins, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint16_t *__restrict__ table,
    uint32_t pad_col) {
  constexpr int G = 64 / LG;  // runs a step
  __shared__ uint32_t npre_all[NB_FILL_THREADS / 64][NB_MAXN];
  __shared__ uint32_t nsrc_all[NB_FILL_THREADS / 64][NB_MAXN];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = lane / LG, gl = lane % LG;
  uint32_t *npre = npre_all[wave];
  uint32_t *nsrc = nsrc_all[wave];
  const uint32_t nkeys = 1u << (2 * k);
  const int nbn = nb_neighbours(k);
  const int R = (nbn + 63) >> 6;
  const int t0 = lane * R;
  const int t2 = 1 + 3 * k;  // first Hamming-2 neighbour
  const int64_t wstride = (int64_t)gridDim.x * (NB_FILL_THREADS / 64);
  for (int64_t b = (int64_t)blockIdx.x * (NB_FILL_THREADS / 64) + wave; b < nbins; b += wstride) {
    const uint32_t start = nboff[b], tot = nboff[b + 1] - start;
    if (tot == 0) continue;  // wave-uniform
    const uint32_t u = (uint32_t)b & (nkeys - 1u);
    const uint32_t *off = xoff + (b - u);
    const uint2 sg = nbseg[b];
    uint32_t src[NB_MAXR], cnt[NB_MAXR];
#pragma unroll
    for (int j = 0; j < NB_MAXR; ++j) {
      cnt[j] = 0;
      src[j] = 0;
      if (j < R && t0 + j < nbn) {
        int sgm;
        const uint32_t v = nb_neighbour(u, k, t0 + j, sgm);
        src[j] = off[v];
        cnt[j] = off[v + 1] - src[j];
      }
    }
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < NB_MAXR; ++j) s += cnt[j];
    const uint32_t inc = nb_wave_incl_scan(s);
    const uint32_t total = __shfl(inc, 63, 64);
    {
      uint32_t r = inc - s;
#pragma unroll
      for (int j = 0; j < NB_MAXR; ++j) {
        if (j < R && t0 + j < nbn) {
          npre[t0 + j] = r;
          nsrc[t0 + j] = src[j];
        }
        r += cnt[j];
      }
    }
    if (lane == 0) npre[nbn] = total;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const uint32_t n0 = npre[1];
    const uint32_t pre2 = t2 < nbn ? npre[t2] : total;
    uint16_t *dst = table + (size_t)start * 8u;
    // (segment base - unpadded segment start) per segment
    const uint32_t dlt0 = 0u, dlt1 = sg.x * 8u - n0, dlt2 = sg.y * 8u - pre2;
    for (int t00 = 0; t00 < nbn; t00 += G * NB_STEPS) {
      uint32_t sa[NB_STEPS], pa[NB_STEPS], ca[NB_STEPS];
#pragma unroll
      for (int q = 0; q < NB_STEPS; ++q) {
        const int t = t00 + q * G + grp;
        ca[q] = 0;
        if (t < nbn) {
          const uint32_t p0 = npre[t];
          ca[q] = npre[t + 1] - p0;
          sa[q] = nsrc[t];
          pa[q] = p0 + (t == 0 ? dlt0 : t < t2 ? dlt1 : dlt2);
        }
      }
      // first LG entries of every run of the steps: loads first, then the stores
      uint16_t v[NB_STEPS];
#pragma unroll
      for (int q = 0; q < NB_STEPS; ++q)
        if ((uint32_t)gl < ca[q]) v[q] = xent[sa[q] + gl];
#pragma unroll
      for (int q = 0; q < NB_STEPS; ++q)
        if ((uint32_t)gl < ca[q]) dst[pa[q] + gl] = v[q];
      // runs longer than LG (rare at the chosen LG)
#pragma unroll
      for (int q = 0; q < NB_STEPS; ++q)
        for (uint32_t e = LG + gl; e < ca[q]; e += LG) dst[pa[q] + e] = xent[sa[q] + e];
    }
    // dummy columns after each segment, spread over 64 LDS words of the Gram kernel
    if (lane < 24) {
      const int sgi = lane >> 3, e = lane & 7;
      const uint32_t segb = sgi == 0 ? 0u : sgi == 1 ? sg.x * 8u : sg.y * 8u;
      const uint32_t segn = sgi == 0 ? n0 : sgi == 1 ? pre2 - n0 : total - pre2;
      const uint32_t segend = sgi == 0 ? sg.x * 8u : sgi == 1 ? sg.y * 8u : tot * 8u;
      const uint32_t pos = segb + segn + (uint32_t)e;
      if (pos < segend) dst[pos] = (uint16_t)(pad_col + (pos & 63u));
    }
    __builtin_amdgcn_wave_barrier();  // the next bin overwrites the tables
  }
}

// ------------------------------------------------------------------ grouped list fill
// The lists of the 4^S k-mers u = (prefix P, suffix s_u) that share their first k - S letters
// are built together by one workgroup.  Every Hamming <= 2 neighbour of such a u is
// (prefix w, suffix s) with ham(w, P) + ham(s, s_u) <= 2, and the 4^S bins of one prefix w
// are ADJACENT in the exact index (key order): the workgroup loads the m_S = 1 + 3(k-S) +
// 9 C(k-S, 2) ranges [w 4^S, (w + 1) 4^S) of bins into LDS once (k = 9, S = 2: 211 ranges of
// ~113 entries at N=20000), then every wave assembles lists from LDS: 352 runs a list in
// segment order, a wave prefix sum placing each run, lane-per-run copies LDS -> HBM.  Per
// list that is ~13 ranges' line requests instead of 352 runs' (the per-list fill above
// gathered each run from L2 / the Infinity Cache: ~2.5 ms at N=20000).  A group whose ranges
// overflow the LDS image (repetitive data) copies straight from the index (flat pointer).
template <int S>
__device__ __forceinline__ void nb_run_desc(int j, int k, int &r, uint32_t &dmask, int &h) {
  // run j of a list, segment order: (prefix range r, suffix xor dmask, Hamming class h)
  const int kp = k - S;
  if (j == 0) {
    r = 0; dmask = 0; h = 0;
    return;
  }
  j -= 1;
  if (j < 3 * S) {  // suffix Hamming 1, prefix 0
    const int ps = j / 3, d = j - 3 * ps + 1;
    r = 0; dmask = (uint32_t)d << (2 * (S - 1 - ps)); h = 1;
    return;
  }
  j -= 3 * S;
  if (j < 3 * kp) {  // prefix Hamming 1, suffix 0
    r = 1 + j; dmask = 0; h = 1;
    return;
  }
  j -= 3 * kp;
  h = 2;
  const int ns2 = 9 * S * (S - 1) / 2;
  if (j < ns2) {  // suffix Hamming 2 (S = 2), prefix 0
    r = 0; dmask = ((uint32_t)(j / 3 + 1) << 2) | (uint32_t)(j - 3 * (j / 3) + 1);
    return;
  }
  j -= ns2;
  if (j < 3 * kp * 3 * S) {  // prefix Hamming 1 x suffix Hamming 1
    const int rp = j / (3 * S), js = j - rp * 3 * S;
    const int ps = js / 3, d = js - 3 * ps + 1;
    r = 1 + rp; dmask = (uint32_t)d << (2 * (S - 1 - ps));
    return;
  }
  j -= 3 * kp * 3 * S;
  r = 1 + 3 * kp + j; dmask = 0;  // prefix Hamming 2, suffix 0
}

// copy one run of n uint16 entries to o (any alignment): WS = 1 one 2-byte store an entry;
// WS = 2 dword stores of entry pairs (o aligned to 4 bytes in the middle); WS = 4 also
// 8-byte stores of aligned quads
template <int WS, typename Src>
__device__ __forceinline__ void nb_copy_run(uint16_t *o, const Src *src, uint32_t n) {
  uint32_t e = 0;
  if constexpr (WS >= 2) {
    if (n && (((uintptr_t)o) & 2)) {
      o[0] = src[0];
      e = 1;
    }
    if constexpr (WS >= 4) {
      if (e + 1 < n && (((uintptr_t)(o + e)) & 4)) {
        *(uint32_t *)(o + e) = (uint32_t)src[e] | ((uint32_t)src[e + 1] << 16);
        e += 2;
      }
      for (; e + 3 < n; e += 4) {
        const uint32_t lo = (uint32_t)src[e] | ((uint32_t)src[e + 1] << 16);
        const uint32_t hi = (uint32_t)src[e + 2] | ((uint32_t)src[e + 3] << 16);
        *(uint2 *)(o + e) = make_uint2(lo, hi);
      }
    }
    for (; e + 1 < n; e += 2) *(uint32_t *)(o + e) = (uint32_t)src[e] | ((uint32_t)src[e + 1] << 16);
  }
  for (; e < n; ++e) o[e] = src[e];
}

// pieces of a list the piece fill assembles in LDS (longer lists: lane-per-run copies)
constexpr int NBP_MAXP = 640;

// LDS word where the piece fill's image starts (16-byte aligned), host and device
__host__ __device__ inline int nb_pieces_img_word(int k, int nt) {
  const int kp = k - 2, mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;
  const int nbn = 1 + 3 * k + 9 * k * (k - 1) / 2;
  const int tw = 2 * (nbn + 1) + NBP_MAXP;
  return (nbn + mr + mr * 17 + mr + 1 + nt / 64 + (nt / 64 * tw + 1) / 2 + 3) & ~3;
}

// the grouped fills' per-workgroup tables: rt[j] = run j of a list (prefix range | suffix xor
// << 16 | Hamming class << 24, segment order) and pm[r] = the prefix xor of range r
template <int S>
__device__ void nb_group_tables(int k, int nt, uint32_t *rt, uint32_t *pm) {
  const int kp = k - S;
  const int mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;
  const int nbn = nb_neighbours(k);
  for (int j = threadIdx.x; j < nbn; j += nt) {
    int r, h;
    uint32_t dm;
    nb_run_desc<S>(j, k, r, dm, h);
    rt[j] = (uint32_t)r | (dm << 16) | ((uint32_t)h << 24);
  }
  for (int r = threadIdx.x; r < mr; r += nt) {
    uint32_t w = 0;
    if (r > 0) {
      int t = r - 1;
      if (t < 3 * kp) {
        const int p = t / 3;
        w = (uint32_t)(t - 3 * p + 1) << (2 * (kp - 1 - p));
      } else {
        t -= 3 * kp;
        const int pi = t / 9, rr = t - 9 * pi;
        int q = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)pi)) * 0.5f);
        while (q * (q - 1) / 2 > pi) --q;
        while ((q + 1) * q / 2 <= pi) ++q;
        const int p = pi - q * (q - 1) / 2;
        w = ((uint32_t)(rr / 3 + 1) << (2 * (kp - 1 - p))) ^
            ((uint32_t)(rr - 3 * (rr / 3) + 1) << (2 * (kp - 1 - q)));
      }
    }
    pm[r] = w;
  }
}

// a group's range offsets into LDS (roff[r][q] = bin offset q of prefix range r), one word a
// lane: consecutive lanes read a range's SW + 1 consecutive offsets (a few lines a wave
// instruction instead of one line a lane), NLD loads in flight a thread before their stores
template <int SW, int NT>
__device__ __forceinline__ void nb_load_range_offsets(const uint32_t *__restrict__ xoff,
                                                      int64_t cbase, uint32_t P,
                                                      const uint32_t *pm, int mr, uint32_t *roff) {
  constexpr int NLD = 4;
  const int tot = mr * (SW + 1);
  for (int w0 = threadIdx.x; w0 < tot; w0 += NLD * NT) {
    uint32_t v[NLD];
#pragma unroll
    for (int t = 0; t < NLD; ++t) {
      const int w = w0 + t * NT;
      if (w < tot) {
        const int r = w / (SW + 1), q = w - r * (SW + 1);
        v[t] = xoff[cbase + (int64_t)(P ^ pm[r]) * SW + q];
      }
    }
#pragma unroll
    for (int t = 0; t < NLD; ++t) {
      const int w = w0 + t * NT;
      if (w < tot) roff[w] = v[t];
    }
  }
}

template <int S, int NT, int WS>
__global__ __launch_bounds__(NT) void nb_fill_grouped_kernel(
    int k, int64_t ngroups, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint16_t *__restrict__ table,
    uint32_t pad_col, int cap) {
  constexpr int SW = 1 << (2 * S);
  constexpr int NW = NT / 64;
  extern __shared__ __align__(16) uint32_t fsm[];
  const int kp = k - S;
  const int mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;  // prefix ranges
  const int nbn = nb_neighbours(k);
  uint32_t *rt = fsm;                        // [nbn] run j: r | suffix xor << 16 | class << 24
  uint32_t *pm = rt + nbn;                   // [mr] prefix xor of range r
  uint32_t *roff = pm + mr;                  // [mr][SW + 1] absolute index offsets
  uint32_t *rbase = roff + mr * (SW + 1);    // [mr + 1] LDS position of each range
  uint32_t *wtot = rbase + mr + 1;           // [NW] scan scratch
  uint16_t *ent = (uint16_t *)(wtot + NW);   // [cap] the ranges' entries
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t npref = 1u << (2 * kp);
  // the run and range tables, once per workgroup (the grid is persistent)
  nb_group_tables<S>(k, NT, rt, pm);
  __syncthreads();
  const int rpt = (mr + NT - 1) / NT;
  const int t2 = 1 + 3 * k;
  for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const uint32_t P = (uint32_t)(gi & (int64_t)(npref - 1u));
    const int64_t cbase = (gi - P) * SW;  // chunk c's first bin: c * 4^k
    if (nboff[gi * SW + SW] == nboff[gi * SW]) continue;  // all 4^S lists empty (uniform)
    // ---- 1. the ranges' bin offsets and sizes; their LDS positions (block scan): thread t
    // owns the ranges [t RPT, t RPT + RPT)
    nb_load_range_offsets<SW, NT>(xoff, cbase, P, pm, mr, roff);
    __syncthreads();
    uint32_t myn = 0;
    for (int r = threadIdx.x * rpt; r < min(mr, (int)(threadIdx.x + 1) * rpt); ++r)
      myn += roff[r * (SW + 1) + SW] - roff[r * (SW + 1)];
    {
      const uint32_t inc = nb_wave_incl_scan_dpp(myn);
      if (lane == 63) wtot[wave] = inc;
      __syncthreads();
      uint32_t base = 0, total = 0;
      for (int w2 = 0; w2 < NW; ++w2) {
        base += w2 < wave ? wtot[w2] : 0u;
        total += wtot[w2];
      }
      uint32_t run = base + inc - myn;
      for (int r = threadIdx.x * rpt; r < min(mr, (int)(threadIdx.x + 1) * rpt); ++r) {
        rbase[r] = run;
        run += roff[r * (SW + 1) + SW] - roff[r * (SW + 1)];
      }
      if (threadIdx.x == 0) rbase[mr] = total;
      __syncthreads();
    }
    const uint32_t etot = rbase[mr];
    const bool staged = etot <= (uint32_t)cap;
    // ---- 2. the ranges into LDS, one wave a range, all of a range's loads in flight
    if (staged) {
      for (int r = wave; r < mr; r += NW) {
        const uint32_t a = roff[r * (SW + 1)], n = roff[r * (SW + 1) + SW] - a, d = rbase[r];
        for (uint32_t j0 = 0; j0 < n; j0 += 256) {
          uint16_t v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t j = j0 + 64u * q + lane;
            if (j < n) v[q] = xent[a + j];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t j = j0 + 64u * q + lane;
            if (j < n) ent[d + j] = v[q];
          }
        }
      }
    }
    __syncthreads();
    // ---- 3. the 4^S lists, one wave a list, 64 runs at a time in segment order: lane j
    // places run j (wave prefix sum) and copies it
    for (int su = wave; su < SW; su += NW) {
      const int64_t b = cbase + (int64_t)P * SW + su;
      const uint32_t start = nboff[b], tot = nboff[b + 1] - start;
      if (tot == 0) continue;  // wave-uniform
      const uint2 sg = nbseg[b];
      uint16_t *dst = table + (size_t)start * 8u;
      uint32_t carry = 0, n0 = 0, pre2 = 0;
      for (int j0 = 0; j0 < nbn; j0 += 64) {
        const int j = j0 + lane;
        uint32_t cnt = 0, srcp = 0, h = 2;
        if (j < nbn) {
          const uint32_t d = rt[j];
          const uint32_t r = d & 0xFFFFu;
          h = d >> 24;
          const uint32_t *ro = roff + r * (SW + 1);
          const uint32_t sidx = (uint32_t)su ^ ((d >> 16) & 0xFFu);
          const uint32_t a0 = ro[sidx];
          cnt = ro[sidx + 1] - a0;
          srcp = staged ? rbase[r] + (a0 - ro[0]) : a0;
        }
        const uint32_t inc = nb_wave_incl_scan_dpp(cnt);
        const uint32_t pos = carry + inc - cnt;
        if (j0 == 0) {
          n0 = (uint32_t)__builtin_amdgcn_readlane((int)cnt, 0);
          pre2 = (uint32_t)__builtin_amdgcn_readlane((int)pos, t2 & 63);  // (t2 < 64 for k <= 21)
        }
        carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        const uint32_t dpos = (h == 0 ? 0u : h == 1 ? sg.x * 8u - n0 : sg.y * 8u - pre2) + pos;
        {
          uint16_t *o = dst + dpos;
          if (staged)
            nb_copy_run<WS>(o, ent + srcp, cnt);
          else
            nb_copy_run<WS>(o, xent + srcp, cnt);
        }
      }
      const uint32_t total = carry;
      // dummy columns after each segment, spread over 64 LDS words of the Gram kernel
      if (lane < 24) {
        const int sgi = lane >> 3, e = lane & 7;
        const uint32_t segb = sgi == 0 ? 0u : sgi == 1 ? sg.x * 8u : sg.y * 8u;
        const uint32_t segn = sgi == 0 ? n0 : sgi == 1 ? pre2 - n0 : total - pre2;
        const uint32_t segend = sgi == 0 ? sg.x * 8u : sgi == 1 ? sg.y * 8u : tot * 8u;
        const uint32_t pp = segb + segn + (uint32_t)e;
        if (pp < segend) dst[pp] = (uint16_t)(pad_col + (pp & 63u));
      }
    }
    __syncthreads();  // the next group overwrites the LDS image
  }
}

// ------------------------------------------------------------------ piece-assembled fill
// The lane-per-run copies above are bound by the texture-address unit, not by bytes: their
// 2-byte loads and stores cost ~25 TA cycles a wave instruction whatever the lane count, and
// a 16-list group issues ~2800 of them (PMC, profiles/r04t_pmc_fill.txt: TA busy 67 % of the
// kernel).  This form moves whole 16-byte pieces through the TA both ways:
//  1. the group's 211 prefix ranges (S = 2) into an LDS image with 16-byte loads, each range
//     at its source alignment mod 8 entries (~220 load instructions a group);
//  2. one wave a list: the 352 runs in segment order -> a wave prefix sum -> a table of the
//     non-empty runs (compacted by a ballot): destination end and (image offset - destination
//     start) as uint16, and for every 16-byte piece of the list the first run that reaches it;
//  3. lane p assembles list piece p from the image (8 LDS reads, the segment's dummy columns
//     in its padding) and writes it with one 16-byte store: a wave writes 1 KB of the list
//     per store instruction (~5 a list instead of ~90).
// Groups whose image exceeds the LDS, and lists of more than NBP_MAXP pieces, take the
// lane-per-run copy from the index.
template <int NL>
__global__ __launch_bounds__(NL * 64) void nb_fill_pieces_kernel(
    int k, int64_t ngroups, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint16_t *__restrict__ table,
    uint32_t pad_col, int cap) {
  constexpr int S = 2, SW = 16, NT = NL * 64, NW = NL, NH = SW / NL;
  extern __shared__ __align__(16) uint32_t fsm[];
  const int kp = k - S;
  const int mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;  // prefix ranges
  const int nbn = nb_neighbours(k);
  const int tw = 2 * (nbn + 1) + NBP_MAXP;           // uint16 table words a wave
  uint32_t *rt = fsm;                                 // [nbn] runs of a list
  uint32_t *pm = rt + nbn;                            // [mr] prefix xor of range r
  uint32_t *roff = pm + mr;                           // [mr][SW + 1] absolute index offsets
  uint32_t *rbase = roff + mr * (SW + 1);             // [mr + 1] image position of each range
  uint32_t *wtot = rbase + mr + 1;                    // [NW] scan scratch
  uint16_t *tabs = (uint16_t *)(wtot + NW);           // [NW][tw] re, rsd, pst
  uint16_t *img = (uint16_t *)(fsm + nb_pieces_img_word(k, NT));  // [cap], 16-byte aligned
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t npref = 1u << (2 * kp);
  nb_group_tables<S>(k, NT, rt, pm);
  __syncthreads();
  const int rpt = (mr + NT - 1) / NT;
  const int t2 = 1 + 3 * k;
  const int nfull = 1 + 3 * kp;  // ranges whose every sub-bin a half group takes
  const uint64_t ltmask = (1ull << lane) - 1ull;
  uint16_t *re = tabs + wave * tw;   // [nbn + 1] destination end of non-empty run idx
  uint16_t *rsd = re + nbn + 1;      // [nbn + 1] image offset - destination start
  uint16_t *pst = rsd + nbn + 1;     // [NBP_MAXP] first run reaching piece p
  for (int64_t bi = blockIdx.x; bi < ngroups * NH; bi += gridDim.x) {
    const int64_t gi = bi / NH;
    const int hh = (int)(bi - gi * NH);  // which NL of the group's 16 lists (suffixes)
    const uint32_t P = (uint32_t)(gi & (int64_t)(npref - 1u));
    const int64_t cbase = (gi - P) * SW;
    if (nboff[gi * SW + hh * NL + NL] == nboff[gi * SW + hh * NL]) continue;  // uniform
    // sub-bins [slo, shi) of range r the block's lists take: all 16 of the own prefix and the
    // Hamming-1 prefixes (suffix Hamming <= 1 reaches every first letter), only the block's
    // own suffixes [hh NL, hh NL + NL) of the Hamming-2 prefixes
    auto slo = [&](int r) { return r < nfull ? 0 : hh * NL; };
    auto shi = [&](int r) { return r < nfull ? SW : hh * NL + NL; };
    // ---- 1. ranges: offsets, image positions (n + 14 words each: 8-aligned + source phase)
    nb_load_range_offsets<SW, NT>(xoff, cbase, P, pm, mr, roff);
    __syncthreads();
    uint32_t myn = 0;
    for (int r = threadIdx.x * rpt; r < min(mr, (int)(threadIdx.x + 1) * rpt); ++r)
      myn += roff[r * (SW + 1) + shi(r)] - roff[r * (SW + 1) + slo(r)] + 14u;
    {
      const uint32_t inc = nb_wave_incl_scan_dpp(myn);
      if (lane == 63) wtot[wave] = inc;
      __syncthreads();
      uint32_t base = 0, total = 0;
      for (int w2 = 0; w2 < NW; ++w2) {
        base += w2 < wave ? wtot[w2] : 0u;
        total += wtot[w2];
      }
      uint32_t run = base + inc - myn;
      for (int r = threadIdx.x * rpt; r < min(mr, (int)(threadIdx.x + 1) * rpt); ++r) {
        const uint32_t a = roff[r * (SW + 1) + slo(r)];
        rbase[r] = ((run + 7u) & ~7u) + (a & 7u);
        run += roff[r * (SW + 1) + shi(r)] - a + 14u;
      }
      if (threadIdx.x == 0) rbase[mr] = total;
      __syncthreads();
    }
    const bool staged = rbase[mr] <= (uint32_t)cap;
    // ---- 2. the image: whole 16-byte pieces of each range, one wave a range
    if (staged) {
      for (int r = wave; r < mr; r += NW) {
        const uint32_t a = roff[r * (SW + 1) + slo(r)], n = roff[r * (SW + 1) + shi(r)] - a;
        if (n == 0) continue;
        const uint32_t fp = a >> 3, lp = (a + n + 7u) >> 3;
        uint16_t *d0 = img + (rbase[r] - (a & 7u));
        for (uint32_t pc = fp + (uint32_t)lane; pc < lp; pc += 64u)
          *(uint4 *)(d0 + 8u * (pc - fp)) = ((const uint4 *)xent)[pc];
      }
    }
    __syncthreads();
    // ---- 3. the block's NL lists, one wave a list
    for (int su = hh * NL + wave; su < hh * NL + NL; su += NW) {
      const int64_t b = cbase + (int64_t)P * SW + su;
      const uint32_t start = nboff[b], tot = nboff[b + 1] - start;
      if (tot == 0) continue;  // wave-uniform
      const uint2 sg = nbseg[b];
      uint16_t *dst = table + (size_t)start * 8u;
      const bool pieces = staged && tot <= (uint32_t)NBP_MAXP;  // wave-uniform
      uint32_t carry = 0, n0 = 0, pre2 = 0, nzc = 0;
      for (int j0 = 0; j0 < nbn; j0 += 64) {
        const int j = j0 + lane;
        uint32_t cnt = 0, a0 = 0, si = 0, h = 2;
        if (j < nbn) {
          const uint32_t d = rt[j];
          const uint32_t r = d & 0xFFFFu;
          h = d >> 24;
          const uint32_t *ro = roff + r * (SW + 1);
          const uint32_t sidx = (uint32_t)su ^ ((d >> 16) & 0xFFu);
          a0 = ro[sidx];
          cnt = ro[sidx + 1] - a0;
          si = rbase[r] + (a0 - ro[slo((int)r)]);
        }
        const uint32_t inc = nb_wave_incl_scan_dpp(cnt);
        const uint32_t pos = carry + inc - cnt;
        if (j0 == 0) {
          n0 = (uint32_t)__builtin_amdgcn_readlane((int)cnt, 0);
          pre2 = (uint32_t)__builtin_amdgcn_readlane((int)pos, t2 & 63);  // (t2 < 64 for k <= 21)
        }
        carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        const uint32_t dpos = (h == 0 ? 0u : h == 1 ? sg.x * 8u - n0 : sg.y * 8u - pre2) + pos;
        if (pieces) {
          const uint64_t bal = __ballot(cnt != 0u);
          const uint32_t idx = nzc + (uint32_t)__popcll(bal & ltmask);
          if (cnt) {
            re[idx] = (uint16_t)(dpos + cnt);
            rsd[idx] = (uint16_t)(si - dpos);
          }
          nzc += (uint32_t)__popcll(bal);
        } else {
          nb_copy_run<1>(dst + dpos, xent + a0, cnt);
        }
      }
      const uint32_t total = carry;
      if (pieces) {
        if (lane == 0) {
          re[nzc] = (uint16_t)(tot * 8u);  // sentinel: past every entry
          rsd[nzc] = 0;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        for (uint32_t idx = (uint32_t)lane; idx <= nzc; idx += 64u) {
          const uint32_t lo = idx ? re[idx - 1] : 0u, hi = re[idx];
          for (uint32_t p = (lo + 7u) >> 3; p < ((hi + 7u) >> 3); ++p) pst[p] = (uint16_t)idx;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        // dummy columns: [n0, sx), [e1, sy), [e2, tot * 8)
        const uint32_t sx = sg.x * 8u, sy = sg.y * 8u;
        const uint32_t e1 = sx + (pre2 - n0), e2 = sy + (total - pre2);
        for (uint32_t p = (uint32_t)lane; p < tot; p += 64u) {
          const uint32_t d0 = 8u * p;
          uint32_t jr = pst[p];
          uint32_t rej = re[jr], sdj = rsd[jr];
          // the next two runs (past the sentinel these read other table words, never used:
          // the sentinel's end lies past every entry)
          const uint32_t re1 = re[jr + 1], sd1 = rsd[jr + 1], re2 = re[jr + 2], sd2 = rsd[jr + 2];
          uint32_t w[4];
          const bool padp = (d0 + 8u > n0 && d0 < sx) || (d0 + 8u > e1 && d0 < sy) || d0 + 8u > e2;
          if (!padp && (re1 >= d0 + 8u || re2 >= d0 + 8u)) {
            // at most three runs reach the piece: branch-free selects
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const uint32_t d = d0 + (uint32_t)q;
              const uint32_t sd = d < rej ? sdj : d < re1 ? sd1 : sd2;
              const uint32_t v = img[(sd + d) & 0xFFFFu];
              if (q & 1) w[q >> 1] |= v << 16;
              else w[q >> 1] = v;
            }
          } else if (padp) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const uint32_t d = d0 + (uint32_t)q;
              if (d >= rej) {
                ++jr;
                rej = re[jr];
                sdj = rsd[jr];
              }
              uint32_t v;
              if ((d >= n0 && d < sx) || (d >= e1 && d < sy) || d >= e2)
                v = (pad_col + (d & 63u)) & 0xFFFFu;
              else
                v = img[(sdj + d) & 0xFFFFu];
              if (q & 1) w[q >> 1] |= v << 16;
              else w[q >> 1] = v;
            }
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const uint32_t d = d0 + (uint32_t)q;
              if (d >= rej) {  // runs are non-empty and contiguous here: one step
                ++jr;
                rej = re[jr];
                sdj = rsd[jr];
              }
              const uint32_t v = img[(sdj + d) & 0xFFFFu];
              if (q & 1) w[q >> 1] |= v << 16;
              else w[q >> 1] = v;
            }
          }
          *(uint4 *)(dst + d0) = make_uint4(w[0], w[1], w[2], w[3]);
        }
        __builtin_amdgcn_wave_barrier();  // the next list overwrites the tables
      } else if (lane < 24) {
        // dummy columns after each segment, spread over 64 LDS words of the Gram kernel
        const int sgi = lane >> 3, e = lane & 7;
        const uint32_t segb = sgi == 0 ? 0u : sgi == 1 ? sg.x * 8u : sg.y * 8u;
        const uint32_t segn = sgi == 0 ? n0 : sgi == 1 ? pre2 - n0 : total - pre2;
        const uint32_t segend = sgi == 0 ? sg.x * 8u : sgi == 1 ? sg.y * 8u : tot * 8u;
        const uint32_t pp = segb + segn + (uint32_t)e;
        if (pp < segend) dst[pp] = (uint16_t)(pad_col + (pp & 63u));
      }
    }
    __syncthreads();  // the next group overwrites the image
  }
}

// ------------------------------------------------------------------ range-major fill
// The grouped fill's copies run range-major: the 16 lists of a group (S = 2) take their runs
// from the 211 prefix ranges, and the 16 sub-bins of one range are contiguous in the index.
//  1. the ranges' sub-bin offsets (as the grouped fill);
//  2. one wave a list places its 352 runs (wave prefix sums in segment order) into an LDS
//     position table pos[list][run] and writes the segments' dummy tails;
//  3. one wave a range copies the range's entries 64 at a time (coalesced 2-byte loads),
//     each entry to every list that takes its sub-bin (1 list for the 189 Hamming-2 prefix
//     ranges, 7 for the 21 Hamming-1 ones, 16 for the group's own prefix): the sub-bin from
//     the 17 offsets held in SGPRs, the run from an inverse table inv[range][suffix xor].
// Per group ~420 load and ~700 store instructions, against ~2900 for lane-per-run copies
// whose lanes idle past the mean run (7 entries of a 64-run chunk whose longest has ~15).
__global__ __launch_bounds__(1024) void nb_fill_ranges_kernel(
    int k, int64_t ngroups, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint16_t *__restrict__ table,
    uint32_t pad_col) {
  constexpr int S = 2, SW = 16, NT = 1024, NW = NT / 64;
  extern __shared__ __align__(16) uint32_t fsm[];
  const int kp = k - S;
  const int mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;  // prefix ranges
  const int nbn = nb_neighbours(k);
  uint32_t *rt = fsm;                        // [nbn] run j: r | suffix xor << 16 | class << 24
  uint32_t *pm = rt + nbn;                   // [mr] prefix xor of range r
  uint32_t *roff = pm + mr;                  // [mr][17] absolute index offsets
  uint32_t *pos = roff + mr * (SW + 1);      // [SW][nbn] list position of run j (entries)
  uint32_t *lst = pos + SW * nbn;            // [SW] list start (pieces)
  uint16_t *inv = (uint16_t *)(lst + SW);    // [mr][16] run of (range, suffix xor); 0xFFFF none
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t npref = 1u << (2 * kp);
  for (int j = threadIdx.x; j < mr * SW; j += NT) inv[j] = 0xFFFFu;
  for (int r = threadIdx.x; r < mr; r += NT) {
    uint32_t w = 0;
    if (r > 0) {
      int t = r - 1;
      if (t < 3 * kp) {
        const int p = t / 3;
        w = (uint32_t)(t - 3 * p + 1) << (2 * (kp - 1 - p));
      } else {
        t -= 3 * kp;
        const int pi = t / 9, rr = t - 9 * pi;
        int q = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)pi)) * 0.5f);
        while (q * (q - 1) / 2 > pi) --q;
        while ((q + 1) * q / 2 <= pi) ++q;
        const int p = pi - q * (q - 1) / 2;
        w = ((uint32_t)(rr / 3 + 1) << (2 * (kp - 1 - p))) ^
            ((uint32_t)(rr - 3 * (rr / 3) + 1) << (2 * (kp - 1 - q)));
      }
    }
    pm[r] = w;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nbn; j += NT) {
    int r, h;
    uint32_t dm;
    nb_run_desc<S>(j, k, r, dm, h);
    rt[j] = (uint32_t)r | (dm << 16) | ((uint32_t)h << 24);
    inv[r * SW + (int)dm] = (uint16_t)j;
  }
  __syncthreads();
  const int t2 = 1 + 3 * k;
  for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const uint32_t P = (uint32_t)(gi & (int64_t)(npref - 1u));
    const int64_t cbase = (gi - P) * SW;  // chunk c's first bin: c * 4^k
    if (nboff[gi * SW + SW] == nboff[gi * SW]) continue;  // all 16 lists empty (uniform)
    // ---- 1. the ranges' sub-bin offsets
    for (int r = threadIdx.x; r < mr; r += NT) {
      const uint32_t *o = xoff + cbase + (int64_t)(P ^ pm[r]) * SW;
#pragma unroll
      for (int q = 0; q <= SW; ++q) roff[r * (SW + 1) + q] = o[q];
    }
    __syncthreads();
    // ---- 2. run positions of the 16 lists, one wave a list
    {
      const int su = wave;
      const int64_t b = cbase + (int64_t)P * SW + su;
      const uint32_t start = nboff[b], tot = nboff[b + 1] - start;
      if (lane == 0) lst[su] = start;
      if (tot > 0) {  // wave-uniform
        const uint2 sg = nbseg[b];
        uint32_t carry = 0, n0 = 0, pre2 = 0;
        for (int j0 = 0; j0 < nbn; j0 += 64) {
          const int j = j0 + lane;
          uint32_t cnt = 0, h = 2;
          if (j < nbn) {
            const uint32_t d = rt[j];
            const uint32_t *ro = roff + (d & 0xFFFFu) * (SW + 1);
            const uint32_t sidx = (uint32_t)su ^ ((d >> 16) & 0xFFu);
            cnt = ro[sidx + 1] - ro[sidx];
            h = d >> 24;
          }
          const uint32_t inc = nb_wave_incl_scan(cnt);
          const uint32_t p0 = carry + inc - cnt;
          if (j0 == 0) {
            n0 = __shfl(cnt, 0, 64);
            pre2 = __shfl(p0, t2 & 63, 64);  // (t2 = 1 + 3k < 64 for k <= 21)
          }
          carry += __shfl(inc, 63, 64);
          if (j < nbn)
            pos[su * nbn + j] = (h == 0 ? 0u : h == 1 ? sg.x * 8u - n0 : sg.y * 8u - pre2) + p0;
        }
        const uint32_t total = carry;
        if (lane < 24) {  // dummy columns after each segment (64 distinct LDS words)
          const int sgi = lane >> 3, e = lane & 7;
          const uint32_t segb = sgi == 0 ? 0u : sgi == 1 ? sg.x * 8u : sg.y * 8u;
          const uint32_t segn = sgi == 0 ? n0 : sgi == 1 ? pre2 - n0 : total - pre2;
          const uint32_t segend = sgi == 0 ? sg.x * 8u : sgi == 1 ? sg.y * 8u : tot * 8u;
          const uint32_t pp = segb + segn + (uint32_t)e;
          if (pp < segend) table[(size_t)start * 8u + pp] = (uint16_t)(pad_col + (pp & 63u));
        }
      }
    }
    __syncthreads();
    // ---- 3. range-major copies, one wave a range
    for (int r = wave; r < mr; r += NW) {
      const uint32_t myoff = lane <= SW ? roff[r * (SW + 1) + lane] : 0u;
      uint32_t so[SW + 1];
#pragma unroll
      for (int q = 0; q <= SW; ++q) so[q] = __builtin_amdgcn_readlane(myoff, q);
      const uint32_t base = so[0], n = so[SW] - base;
      const int hp = r == 0 ? 0 : r <= 3 * kp ? 1 : 2;
      for (uint32_t e0 = 0; e0 < n; e0 += 64) {
        const uint32_t e = e0 + lane;
        if (e >= n) continue;
        const uint16_t v = xent[base + e];
        int sb = 0;
#pragma unroll
        for (int q = 1; q < SW; ++q) sb += (base + e >= so[q]) ? 1 : 0;
        const uint32_t t = base + e - so[sb];
        const uint16_t *iv = inv + r * SW;
        if (hp == 2) {  // only the list with suffix sb
          table[(size_t)lst[sb] * 8u + pos[sb * nbn + iv[0]] + t] = v;
        } else if (hp == 1) {  // the lists within one suffix letter of sb
#pragma unroll
          for (int x = 0; x < 7; ++x) {
            const int dmx = x == 0 ? 0 : x <= 3 ? x : (x - 3) << 2;
            const int su = sb ^ dmx;
            table[(size_t)lst[su] * 8u + pos[su * nbn + iv[dmx]] + t] = v;
          }
        } else {  // the group's own prefix: every list
#pragma unroll
          for (int dmx = 0; dmx < SW; ++dmx) {
            const int su = sb ^ dmx;
            table[(size_t)lst[su] * 8u + pos[su * nbn + iv[dmx]] + t] = v;
          }
        }
      }
    }
    __syncthreads();  // the next group overwrites the tables
  }
}

// One workgroup per (row i, column chunk c) (rowacc_block: chunk-major, upper block
// triangle for a full square K).
// A16: 16-bit column counters, two a dword (the LDS of a chunk halves: two workgroups a CU
// at N=200000's 28572-column chunks instead of one).  Exact while no count reaches 2^16:
// K is a Gram matrix (K_ij = <phi(x_i), phi(x_j)>), so K_ij^2 <= K_ii K_jj, and a (row,
// chunk) whose K_ii x max_{j in chunk} K_jj < 2^32 cannot overflow; any other takes two
// passes over its list with 32-bit counters for half the chunk's columns each.
template <int K, int NB_UNROLL, bool A16>
__global__ __launch_bounds__(1024) void gram_nb_kernel(IndexGeom g, Packed pk,
                                                       const uint32_t *__restrict__ nboff,
                                                       const uint2 *__restrict__ nbseg,
                                                       const uint4 *__restrict__ table,
                                                       int64_t row0, int64_t rows, int w0, int w1,
                                                       int w2, OutSpec o,
                                                       const double *__restrict__ kdiag,
                                                       const double *__restrict__ kdmax) {
  extern __shared__ __align__(16) uint32_t smem[];
  int c;
  int64_t il;
  rowacc_block(g, o, row0, rows, c, il);
  const int64_t i = row0 + il;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  if (col0 + cw <= o.col_lo) return;  // the whole chunk lies below the written columns
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int accn = A16 ? (((accw >> 1) + 32 + 3) & ~3) : accw + 64;  // counter words (+ dummies)
  const int P = g.pmax;
  uint32_t *wst = smem + accn;        // [P] list start of window a (pieces)
  uint32_t *wcum = wst + P;           // [P + 1] pieces of windows < a
  uint32_t *ws0 = wcum + P + 1;       // [P] end of segment 0 (pieces, list-relative)
  uint32_t *ws1 = ws0 + P;            // [P] end of segment 1
  uint32_t *srec = ws1 + P;           // packed row record
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  stage_record(pk, i, srec);
  __syncthreads();
  const uint32_t cbase = (uint32_t)c << (2 * K);
  for (int a = threadIdx.x; a < P; a += blockDim.x) {
    const uint32_t u = pk_window(srec, pk.cw, a, K);
    uint32_t st = 0, n = 0, s0 = 0, s1 = 0;
    if (u != KMG_INVALID) {
      const uint32_t b = cbase + u;
      st = nboff[b];
      n = nboff[b + 1] - st;
      const uint2 sg = nbseg[b];
      s0 = sg.x;
      s1 = sg.y;
    }
    wst[a] = st;
    wcum[a + 1] = n;
    ws0[a] = s0;
    ws1[a] = s1;
  }
  __syncthreads();
  if (wave == 0) {  // inclusive prefix of wcum[1 .. P] (one wave, contiguous runs a lane)
    const int per = (P + 63) >> 6, lo = lane * per, hi = min(P, lo + per);
    uint32_t s = 0;
    for (int a = lo; a < hi; ++a) s += wcum[a + 1];
    uint32_t run = nb_wave_incl_scan(s) - s;
    for (int a = lo; a < hi; ++a) {
      run += wcum[a + 1];
      wcum[a + 1] = run;
    }
    if (lane == 0) wcum[0] = 0;
  }
  // 16-bit counters for this (row, chunk), or two 32-bit passes over column halves
  const bool c16 = A16 && kdiag[i] * kdmax[c] < 4294967296.0;
  const int npass = (!A16 || c16) ? 1 : 2;
  const uint32_t half = (uint32_t)((((cw + 1) >> 1) + 7) & ~7);  // pass 1's first column
  const bool norm = o.normalize && o.diagv[0] != 1.0;
  for (int pass = 0; pass < npass; ++pass) {
    // pass columns [plo, plo + pcw) (relative to col0); 32-bit counters at acc[x - plo]
    const uint32_t plo = npass == 1 ? 0u : pass * half;
    // (a chunk's last columns can be fewer than half: pass 0 takes them all, pass 1 none)
    const uint32_t ucw = (uint32_t)cw;
    const uint32_t pcw = npass == 1 ? ucw : pass ? (ucw > half ? ucw - half : 0u) : min(half, ucw);
    {
      uint4 *acc4 = (uint4 *)smem;
      for (int w = threadIdx.x; w < (accn >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    // this wave's share of the row's pieces; lane l takes pieces qb + l, qb + l + 64, ...
    const uint32_t T = wcum[P];
    const uint32_t qb = (uint32_t)(((uint64_t)T * wave) / nw), qe = (uint32_t)(((uint64_t)T * (wave + 1)) / nw);
    uint32_t q = qb + lane;
    int a = 0;  // window of piece q: the last a with wcum[a] <= q
    {
      int lo = 0, hi = P - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (wcum[mid] <= q) lo = mid;
        else hi = mid - 1;
      }
      a = lo;
    }
    uint32_t abeg = wcum[a], aend = wcum[a + 1], ast = wst[a], as0 = ws0[a], as1 = ws1[a];
    for (; q < qe; q += 64 * NB_UNROLL) {
      uint4 v[NB_UNROLL];
      int wt[NB_UNROLL];
#pragma unroll
      for (int t = 0; t < NB_UNROLL; ++t) {
        const uint32_t qq = q + 64u * t;
        wt[t] = 0;
        if (qq < qe) {
          while (qq >= aend) {
            ++a;
            abeg = aend;
            aend = wcum[a + 1];
            ast = wst[a];
            as0 = ws0[a];
            as1 = ws1[a];
          }
          const uint32_t rel = qq - abeg;
          v[t] = table[(uint64_t)ast + rel];
          wt[t] = rel < as0 ? w0 : rel < as1 ? w1 : w2;
        }
      }
#pragma unroll
      for (int t = 0; t < NB_UNROLL; ++t) {
        if (wt[t]) {
          const uint32_t x[4] = {v[t].x, v[t].y, v[t].z, v[t].w};
          if (!A16) {
            int32_t *acc = (int32_t *)smem;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              atomicAdd(&acc[x[h] & 0xFFFFu], wt[t]);
              atomicAdd(&acc[x[h] >> 16], wt[t]);
            }
          } else if (c16) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              const uint32_t xl = x[h] & 0xFFFFu, xh = x[h] >> 16;
              atomicAdd(&smem[xl >> 1], (uint32_t)wt[t] << ((xl & 1u) << 4));
              atomicAdd(&smem[xh >> 1], (uint32_t)wt[t] << ((xh & 1u) << 4));
            }
          } else {  // 32-bit counters of this pass's columns (dummies >= accw never land)
            int32_t *acc = (int32_t *)smem;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              const uint32_t xl = (x[h] & 0xFFFFu) - plo, xh = (x[h] >> 16) - plo;
              if (xl < pcw) atomicAdd(&acc[xl], wt[t]);
              if (xh < pcw) atomicAdd(&acc[xh], wt[t]);
            }
          }
        }
      }
    }
    __syncthreads();
    if (c16)
      emit_row<true, true>(o, il, i, col0, cw, (const int32_t *)smem, norm);
    else
      emit_row<true>(o, il, i, col0 + plo, (int)pcw, (const int32_t *)smem, norm);
    if (pass + 1 < npass) __syncthreads();
  }
}

// per column chunk, the largest raw diagonal K_jj of its columns (the 16-bit counters' bound)
__global__ __launch_bounds__(256) void chunk_dmax_kernel(const double *__restrict__ kdiag, int64_t n,
                                                         int chunk, double *__restrict__ dmax) {
  __shared__ double red[256];
  const int64_t c0 = (int64_t)blockIdx.x * chunk, c1 = min(n, c0 + chunk);
  double m = 0.0;
  for (int64_t j = c0 + threadIdx.x; j < c1; j += 256) m = fmax(m, kdiag[j]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) dmax[blockIdx.x] = red[0];
}

hipError_t launch_chunk_dmax(const double *kdiag, int64_t n, int chunk, int nchunks, double *dmax,
                             hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(chunk_dmax_kernel, dim3((unsigned)nchunks), dim3(256), 0, s, kdiag, n, chunk, dmax);
  return hipGetLastError();
}

int64_t nb_list_entries_bound(int k, int64_t occurrences, int64_t nbins) {
  // every occurrence sits in the lists of its 1 + 3k + 9k(k-1)/2 neighbours; a non-empty list
  // pads each of its three segments by at most 7 entries
  const int64_t e = (int64_t)(1 + 3 * k + 9 * k * (k - 1) / 2) * occurrences;
  return e + 21 * std::min(nbins, e);
}

size_t nb_gram_lds(const IndexGeom &g, const Packed &pk, bool a16) {
  const int accw = ((g.chunk + 3) >> 2) << 2;
  return (size_t)((a16 ? (((accw >> 1) + 32 + 3) & ~3) : accw + 64) + 4 * g.pmax + 1 + pk.ldp) * 4;
}

hipError_t launch_nb_count(const IndexGeom &g, const uint32_t *xoff, uint32_t *hist,
                           uint32_t *nboff, uint32_t *cursor, uint2 *nbseg, uint32_t *partials,
                           hipStream_t s) {
  const int64_t nbins = g.nbins();
  if (g.copies != 1 || g.k < 2 || g.k > 12) return hipErrorInvalidValue;
  hipLaunchKernelGGL(nb_count_kernel, dim3((unsigned)((nbins + 255) / 256)), dim3(256), 0, s, g.k,
                     nbins, xoff, hist, nbseg);
  return launch_scan(hist, nboff, cursor, nbins, partials, s);
}

hipError_t launch_nb_fill(const IndexGeom &g, const uint32_t *xoff, const uint16_t *xent,
                          const uint32_t *nboff, const uint2 *nbseg, uint16_t *table,
                          hipStream_t s, int form, int cap_override) {
  const int64_t nbins = g.nbins();
  if (g.copies != 1 || g.k < 2 || g.k > 12) return hipErrorInvalidValue;
  const uint32_t pad_col = (uint32_t)(((g.chunk + 3) >> 2) << 2);
  const double mean = (double)g.chunk * g.pmax / (double)g.nkeys;  // occurrences of a k-mer
  if (form == 6 && g.k >= 4) {
    // range-major grouped fill (S = 2)
    const int kp = g.k - 2, mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;
    const int nbn = 1 + 3 * g.k + 9 * g.k * (g.k - 1) / 2;
    const size_t lds = sizeof(uint32_t) * ((size_t)nbn + mr + (size_t)mr * 17 + 16 * (size_t)nbn + 16) +
                       sizeof(uint16_t) * (size_t)mr * 16;
    if (lds <= 160 * 1024) {
      const int64_t ngroups = nbins / 16;
      const int64_t blocks = std::min<int64_t>(ngroups, 256 * 8);
      hipLaunchKernelGGL(nb_fill_ranges_kernel, dim3((unsigned)blocks), dim3(1024), lds, s, g.k,
                         ngroups, xoff, xent, nboff, nbseg, table, pad_col);
      return hipGetLastError();
    }
  }
  // auto: the piece-assembled fill where a list's runs are long enough for its fixed cost per
  // group (~7 us of range offsets + image loads) to pay: N=200000 rank slab (7 chunks of
  // 28572 columns, 10.1 occurrences a k-mer and chunk) fill 9.1 -> 7.0 ms; at N=20000 (7.1)
  // the lane-per-run copies stay ahead, 1.25 vs 1.30 ms (profiles/r04_nb_fill.jsonl r04z)
  if (form == 0 && mean >= 8.5) form = 9;
  if ((form == 9 || form == 10) && g.k >= 4 && (((uintptr_t)xent) & 15u) == 0) {
    // piece-assembled grouped fill (S = 2): 16 lists a 1024-thread workgroup (form 9) or 8
    // lists a 512-thread one (form 10: half the LDS image, two workgroups a CU, measured
    // slower: each half group reloads the 211 ranges' offsets); the LDS left after the
    // tables is the image
    const int nl = form == 9 ? 16 : 8, nt = nl * 64;
    const int bpc = form == 9 ? 1 : 2;  // workgroups a CU the LDS is split for
    const size_t fixed = 4 * (size_t)nb_pieces_img_word(g.k, nt);
    const size_t avail = (size_t)160 * 1024 / bpc;
    int cap = fixed < avail ? (int)std::min<size_t>((avail - fixed) / 2, 65528) & ~7 : 0;
    if (cap_override >= 0) cap = std::min(cap, cap_override & ~7);
    if (cap >= 1024) {
      const size_t lds = fixed + 2 * (size_t)cap;
      const int64_t ngroups = nbins / 16;
      const int64_t blocks = std::min<int64_t>(ngroups * (16 / nl), 256 * bpc);
      if (nl == 16)
        hipLaunchKernelGGL(nb_fill_pieces_kernel<16>, dim3((unsigned)blocks), dim3(nt), lds, s, g.k,
                           ngroups, xoff, xent, nboff, nbseg, table, pad_col, cap);
      else
        hipLaunchKernelGGL(nb_fill_pieces_kernel<8>, dim3((unsigned)blocks), dim3(nt), lds, s, g.k,
                           ngroups, xoff, xent, nboff, nbseg, table, pad_col, cap);
      return hipGetLastError();
    }
  }
  if (form != 1 && g.k >= 4) {
    // grouped fill: S = 2 (16 lists a workgroup of 1024 threads) while the expected LDS
    // image stays <= 48 KB, else S = 1 (4 lists, 256 threads); the image is sized at 2x the
    // expectation (larger groups copy straight from the index)
    auto ranges = [&](int S) { const int kp = g.k - S; return 1 + 3 * kp + 9 * kp * (kp - 1) / 2; };
    const double e2 = ranges(2) * 16.0 * mean, e1 = ranges(1) * 4.0 * mean;  // LDS entries
    // S = 2 unless forced: it beat S = 1 at both sizes measured, also where the range image
    // overflows the LDS for part of the groups (N=200000 rank slab: fill 13.2 vs 23.3 ms;
    // N=20000: 1.44 vs 2.43 ms, profiles/r04_nb_fill.jsonl)
    const int S = form == 2 ? 1 : 2;
    const int SW = 1 << (2 * S), mr = ranges(S);
    const int nt = S == 2 ? 1024 : 512;
    const double e = S == 2 ? e2 : e1;
    int cap = (int)std::min(1.5 * e + 1024.0, S == 2 ? 40960.0 : 24576.0);
    cap = (cap + 7) & ~7;
    // no LDS range image by default: copying the runs straight from the index (L2 /
    // Infinity Cache) measured faster than staging them (N=20000 fill 1.49 -> 1.27 ms, rank
    // slab equal; profiles/r04_nb_fill.jsonl r04o); KMG_NB_CAP > 0 stages up to that many
    cap = cap_override >= 0 ? std::min(cap, cap_override & ~7) : 0;
    const int nbn = 1 + 3 * g.k + 9 * g.k * (g.k - 1) / 2;
    const int ws = form == 4 ? 2 : form == 5 ? 4 : 1;
    const size_t lds = sizeof(uint32_t) * ((size_t)nbn + mr + (size_t)mr * (SW + 1) + mr + 1 + nt / 64) +
                       2 * (size_t)cap;
    const int64_t ngroups = nbins / SW;
    const int64_t blocks = std::min<int64_t>(ngroups, 256 * 16);
    // store width: 1 / 2 / 4 entries (KMG_NB_FILL 3 / 4 / 5; auto 1: the wider stores measured
    // equal or slower, N=200000 rank slab fill 9.1 -> 15.1 ms, profiles/r04_nb_fill.jsonl r04n)
#define KMG_NBG(S_, NT_, WS_)                                                                  \
  hipLaunchKernelGGL((nb_fill_grouped_kernel<S_, NT_, WS_>), dim3((unsigned)blocks), dim3(NT_), \
                     lds, s, g.k, ngroups, xoff, xent, nboff, nbseg, table, pad_col, cap)
    if (S == 2) {
      if (ws == 1) KMG_NBG(2, 1024, 1);
      else if (ws == 2) KMG_NBG(2, 1024, 2);
      else KMG_NBG(2, 1024, 4);
    } else {
      KMG_NBG(1, 512, 4);
    }
#undef KMG_NBG
    return hipGetLastError();
  }
  const int64_t wpb = NB_FILL_THREADS / 64;
  // waves in flight: 32 a CU x 256 CUs, each walking bins in key order (neighbouring
  // k-mers share most of their neighbours' posting lines in L2)
  const int64_t fill_blocks = std::min<int64_t>((nbins + wpb - 1) / wpb, 8 * 256);
  // lanes a run: the mean occurrences of a k-mer in a chunk, to a power of two in [4, 32]
  const int lg = mean <= 4.0 ? 4 : mean <= 8.0 ? 8 : mean <= 16.0 ? 16 : 32;
#define KMG_NBF(LG_)                                                                             \
  hipLaunchKernelGGL(nb_fill_kernel<LG_>, dim3((unsigned)fill_blocks), dim3(NB_FILL_THREADS), 0, \
                     s, g.k, nbins, xoff, xent, nboff, nbseg, table, pad_col)
  if (lg == 4) KMG_NBF(4);
  else if (lg == 8) KMG_NBF(8);
  else if (lg == 16) KMG_NBF(16);
  else KMG_NBF(32);
#undef KMG_NBF
  return hipGetLastError();
}

hipError_t launch_gram_mismatch1_nb(const IndexGeom &g, const Packed &pk, const uint32_t *nboff,
                                    const uint2 *nbseg, const uint4 *table, int64_t row0,
                                    int64_t row1, int w0, int w1, int w2, const OutSpec &o,
                                    hipStream_t s, int threads, int unroll, const double *kdiag,
                                    const double *kdmax) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (g.k < 3 || g.k > 12 || g.copies != 1) return hipErrorNotSupported;
  if (threads != 512 && threads != 1024) return hipErrorInvalidValue;
  const bool a16 = kdiag != nullptr && kdmax != nullptr;
  const int64_t nblk = rowacc_blocks(g, o, row0, rows);
  if (nblk * threads >= (1LL << 32)) return hipErrorInvalidValue;  // AQL grid size is 32-bit
  if (g.chunk + 64 + 63 >= 65536) return hipErrorInvalidValue;      // uint16 columns + dummies
  const size_t lds = nb_gram_lds(g, pk, a16);
  if (lds > (threads == 512 ? 80 : 160) * 1024) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk);
  switch (g.k) {
#define KMG_NB(KK)                                                                              \
  case KK:                                                                                      \
    if (a16)                                                                                    \
      hipLaunchKernelGGL((gram_nb_kernel<KK, 4, true>), grid, dim3(threads), lds, s, g, pk,     \
                         nboff, nbseg, table, row0, rows, w0, w1, w2, o, kdiag, kdmax);         \
    else if (unroll == 8)                                                                       \
      hipLaunchKernelGGL((gram_nb_kernel<KK, 8, false>), grid, dim3(threads), lds, s, g, pk,    \
                         nboff, nbseg, table, row0, rows, w0, w1, w2, o, kdiag, kdmax);         \
    else                                                                                        \
      hipLaunchKernelGGL((gram_nb_kernel<KK, 4, false>), grid, dim3(threads), lds, s, g, pk,    \
                         nboff, nbseg, table, row0, rows, w0, w1, w2, o, kdiag, kdmax);         \
    break;
    KMG_NB(3) KMG_NB(4) KMG_NB(5) KMG_NB(6) KMG_NB(7) KMG_NB(8) KMG_NB(9) KMG_NB(10) KMG_NB(11)
    KMG_NB(12)
#undef KMG_NB
  }
  return hipGetLastError();
}

}  // namespace kmg
