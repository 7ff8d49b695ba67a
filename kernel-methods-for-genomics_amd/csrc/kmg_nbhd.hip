// kmg_nbhd.hip — mismatch (k, 1) Gram through NEIGHBOURHOOD LISTS (gfx950).
//
// get_mismatch_K (kernels.py:196-217) reduces to the closed form
//   K(x, y) = sum_{a, b} w[ham(x_a, y_b)],  w = (1 + 3k, 4, 2) for m = 1
// (kmgram.params.mismatch_weights), i.e. for row i's window k-mer u every column window at
// Hamming distance <= 2 of u adds w[ham] to its column.  This formulation materialises, once
// per build, for every (column chunk c, k-mer u) the NEIGHBOURHOOD LIST of u:
//
//   [ occurrences of u | of its 3k Hamming-1 neighbours | of its 9 k(k-1)/2 Hamming-2 ]
//
// as columns inside the chunk, so that a row window reads ONE contiguous list (N=200000,
// k=9: ~25000 entries over all chunks) and the Gram kernel streams HBM, 16 bytes a lane.
//
// List layout (in 16-byte pieces; nboff = list start, nbseg = (end of segment 0, end of
// segment 1), nbuse = (16-bit pieces, packed pieces), written by the fill):
//   [0, s0)            segment 0 as uint16 columns, 8 a piece (dummy columns pad the tail)
//   [s0, s1)           segment 1, the same
//   [s1, n16)          16-bit part of segment 2: the entries the packing left over
//   [n16, n16 + np)    PACKED part of segment 2: a piece = one uint16 column c (the minimum
//                      of its 15 columns) + 14 bytes o_1..o_14, columns c + o_t.  The sorted
//                      fill counting-sorts the segment by column >> 6 and cuts it into runs of
//                      15; a run spanning <= 254 columns becomes a packed piece, any other (and
//                      the last n2 mod 15 entries) go to the 16-bit part.
// Segment 2 holds ~93 % of a list's entries (k = 9), at ~0.115 entries a column of the chunk:
// 15 of them span ~122 columns, 0.5 % of the runs exceed 254 (1.078 B an entry against 2).
// A list whose segment 2 exceeds the fill's LDS sort buffer, or a k too sparse to pack
// (k >= 10: ~28 columns between entries), keeps the whole segment as 16-bit pieces
// (n16 = list size, np = 0).
//
//   nb_count_kernel   per (c, u): n0, n1, n2 from the exact index (1 + 3k + 9k(k-1)/2
//                     lookups of its bin offsets, L2-resident) -> 16-bit pieces and segment ends
//   launch_scan       list starts (in pieces; < 2^32: checked by the host)
//   list fills        (launch_nb_fill picks one; all take one workgroup per 16 k-mers sharing
//                     a (k-2)-letter prefix, the group's range offsets loaded once, one wave a list)
//     nb_fill_sorted_kernel   packed segment 2, where a list is read often enough to repay
//                     the sort (the host's reads rule): runs staged in a per-wave LDS buffer,
//                     segments 0 / 1 stored with 16-byte stores, segment 2 counting-sorted by
//                     column >> 6, then packed 15 entries a lane
//     nb_fill_staged_kernel   16-bit lists (the default elsewhere): the whole list staged in
//                     LDS, stored with 16-byte stores
//     nb_fill_grouped_kernel  lane-per-run copies straight from the index (forced, and the
//                     other fills' fallback for lists past their LDS buffers)
//     nb_fill_pieces_kernel   16-bit lists past 8.5 occurrences a k-mer and chunk where the
//                     staged fill's buffer is too small: the ranges as an LDS image
//   gram_nb_kernel   per (row i, chunk c): row windows -> (list start, pieces, segment
//                     ends) in LDS, prefix sums over the row's 16-bit and packed pieces, then
//                     every wave streams an equal share of each, 16 bytes a lane, adding the
//                     segment's weight for each column of a piece into the LDS accumulator;
//                     fused normalize_K epilogue (emit_row).
//
// Roofline: the lists are read from HBM once per (row, chunk): N=20000 ~270 KB a row (packed;
// 466 KB as 16-bit lists) against the 160 KB float64 K row; the bound is HBM (list reads +
// K writes) beside the LDS adds (one ds_add per entry).  Column blocks (kmg_gram_device_cols)
// build the lists over a block's sequences and stream them for every row.
#include "kmg_rowacc.h"

namespace kmg {

namespace {
__device__ __forceinline__ int nb_neighbours(int k) { return 1 + 3 * k + 9 * k * (k - 1) / 2; }

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

// LDS written by some lanes of the wave, read by others next: compiler and memory order at
// wave scope (a wave's LDS instructions execute in order)
__device__ __forceinline__ void nb_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// dummy column of list position pp: NB_DUMMIES LDS words past the accumulator, spread by
// position (16: the Gram kernel's LDS is counted to the word, two workgroups a CU)
constexpr int NB_DUMMIES = 16;
__device__ __forceinline__ uint16_t nb_dummy(uint32_t pad_col, uint32_t pp) {
  return (uint16_t)(pad_col + (pp & (uint32_t)(NB_DUMMIES - 1)));
}
}  // namespace

// per (chunk, k-mer): 16-bit pieces of its neighbourhood list and the segment ends (pieces)
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

// ------------------------------------------------------------------ group tables
// The lists of the 4^S k-mers u = (prefix P, suffix s_u) that share their first k - S letters
// are built together by one workgroup.  Every Hamming <= 2 neighbour of such a u is
// (prefix w, suffix s) with ham(w, P) + ham(s, s_u) <= 2, and the 4^S bins of one prefix w
// are ADJACENT in the exact index (key order): the workgroup loads the m_S = 1 + 3(k-S) +
// 9 C(k-S, 2) ranges [w 4^S, (w + 1) 4^S) of bin offsets into LDS once (k = 9, S = 2: 211
// ranges), then every wave assembles lists: 352 runs a list in segment order, a wave prefix
// sum placing each run.
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

// copy one run of n uint16 entries to o (2-byte stores)
template <typename Src>
__device__ __forceinline__ void nb_copy_run(uint16_t *o, const Src *src, uint32_t n) {
  for (uint32_t e = 0; e < n; ++e) o[e] = src[e];
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

// the same offsets in two halves, so a group's loads can be in flight while the previous
// group's lists are assembled: nb_ranges_issue (global -> registers) and nb_ranges_store
template <int SW, int NT, int NLD>
__device__ __forceinline__ void nb_ranges_issue(const uint32_t *__restrict__ xoff, int64_t cbase,
                                                uint32_t P, const uint32_t *pm, int mr,
                                                uint32_t (&v)[NLD]) {
  const int tot = mr * (SW + 1);
#pragma unroll
  for (int t = 0; t < NLD; ++t) {
    const int w = (int)threadIdx.x + t * NT;
    v[t] = 0u;
    if (w < tot) {
      const int r = w / (SW + 1), q = w - r * (SW + 1);
      v[t] = xoff[cbase + (int64_t)(P ^ pm[r]) * SW + q];
    }
  }
}
template <int SW, int NT, int NLD>
__device__ __forceinline__ void nb_ranges_store(int mr, const uint32_t (&v)[NLD], uint32_t *roff) {
  const int tot = mr * (SW + 1);
#pragma unroll
  for (int t = 0; t < NLD; ++t) {
    const int w = (int)threadIdx.x + t * NT;
    if (w < tot) roff[w] = v[t];
  }
}

// ------------------------------------------------------------------ lane-per-run list copy
// One wave builds list b (16-bit pieces, all three segments) of a group whose range offsets
// are in LDS: the 352 runs in segment order, a wave prefix sum placing each run, lane-per-run
// 2-byte copies straight from the index (L2 / the Infinity Cache; an LDS range image measured
// slower, profiles/r04_nb_fill.jsonl r04o), the dummy tail of each segment.
__device__ __forceinline__ void nb_list_lane_per_run(int k, int su, const uint32_t *rt,
                                                     const uint32_t *roff, const uint16_t *xent,
                                                     uint32_t tot, uint2 sg, uint16_t *dst,
                                                     uint32_t pad_col) {
  constexpr int SW = 16;
  const int lane = threadIdx.x & 63;
  const int nbn = nb_neighbours(k), t2 = 1 + 3 * k;  // (t2 < 64 for k <= 21)
  uint32_t carry = 0, n0 = 0, pre2 = 0;
  for (int j0 = 0; j0 < nbn; j0 += 64) {
    const int j = j0 + lane;
    uint32_t cnt = 0, srcp = 0, h = 2;
    if (j < nbn) {
      const uint32_t d = rt[j];
      const uint32_t *ro = roff + (d & 0xFFFFu) * (SW + 1);
      const uint32_t sidx = (uint32_t)su ^ ((d >> 16) & 0xFFu);
      h = d >> 24;
      srcp = ro[sidx];
      cnt = ro[sidx + 1] - srcp;
    }
    const uint32_t inc = nb_wave_incl_scan_dpp(cnt);
    const uint32_t pos = carry + inc - cnt;
    if (j0 == 0) {
      n0 = (uint32_t)__builtin_amdgcn_readlane((int)cnt, 0);
      pre2 = (uint32_t)__builtin_amdgcn_readlane((int)pos, t2 & 63);
    }
    carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    const uint32_t dpos = (h == 0 ? 0u : h == 1 ? sg.x * 8u - n0 : sg.y * 8u - pre2) + pos;
    nb_copy_run(dst + dpos, xent + srcp, cnt);
  }
  const uint32_t total = carry;
  // dummy columns after each segment, spread over 64 LDS words of the Gram kernel
  if (lane < 24) {
    const int sgi = lane >> 3, e = lane & 7;
    const uint32_t segb = sgi == 0 ? 0u : sgi == 1 ? sg.x * 8u : sg.y * 8u;
    const uint32_t segn = sgi == 0 ? n0 : sgi == 1 ? pre2 - n0 : total - pre2;
    const uint32_t segend = sgi == 0 ? sg.x * 8u : sgi == 1 ? sg.y * 8u : tot * 8u;
    const uint32_t pp = segb + segn + (uint32_t)e;
    if (pp < segend) dst[pp] = nb_dummy(pad_col, pp);
  }
}

// ------------------------------------------------------------------ sorted (packed) fill
// One 1024-thread workgroup per group of 16 lists (S = 2), one wave a list, the list's
// segment 2 counting-sorted in a per-wave LDS buffer:
//  1. the 352 runs in segment order (wave prefix sums, 64 runs a step, lane j run j);
//     segments 0 and 1 are copied from the exact index into the table (16-bit pieces);
//     segment 2's runs into the buffer, each entry also counted in a histogram of 64-column
//     buckets -- a run read as two whole 16-byte pieces of the index (texture-address work
//     is per load instruction: 2 a lane instead of one per entry) and shifted into place by
//     register selects;
//  2. the histogram's exclusive scan -> bucket starts;
//  3. the buffer into registers (ds_read_b64, 4 entries a lane), then every entry to slot
//     p + p / 15 of its bucket position p (ds_add_rtn on the bucket start): the segment in
//     column >> 6 order, as runs of 15 entries in 16-slot (32-byte) rows;
//  4. nb_pack_seg2: a row of 15 (two ds_read_b128) spanning <= 254 columns becomes a packed
//     piece, else its entries go to the 16-bit part.
// ~4.5 LDS operations a segment-2 entry (7 in round 5's first form, 1.8 ms at N=20000).
// Segment 2 past the buffer (cap2 entries, from the LDS left over) stays 16-bit.
constexpr int NBS_RW = 14;                 // ds_read_b64 registers (4 entries each) a lane
constexpr int NBS_MAXCAP = 256 * NBS_RW;   // 3584 entries a wave sorts
constexpr int NBS_BSH = 6;                 // bucket = column >> 6
constexpr int NBS_MAXBK = 512;             // buckets a list's sort handles (chunks <= 32768)

__host__ __device__ inline int nbs_table_words(int k) {
  const int kp = k - 2, mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;
  const int nbn = 1 + 3 * k + 9 * k * (k - 1) / 2;
  return (nbn + mr + mr * 17 + 3) & ~3;
}
// the staged fill's tables: nbs_table_words + a second range-offset buffer
__host__ __device__ inline int nb_staged_table_words(int k) {
  const int kp = k - 2, mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;
  return (nbs_table_words(k) + mr * 17 + 3) & ~3;
}
// per wave: the histogram (nbk words, 16-byte aligned), segments 0 + 1 (NBS_S01 words), 64
// trash words, the buffer (cap2 entries in 16-slot rows of 15)
constexpr int NBS_S01 = 256;
__host__ __device__ inline int nbs_wave_words(int nbk, int cap2) {
  return ((nbk + 3) & ~3) + NBS_S01 + 64 + ((cap2 + 14) / 15) * 8;
}

// segment 2 (n2 entries, column >> 6 order, runs of 15 in 16-slot rows at sb, 16-byte
// aligned) -> packed pieces + 16-bit spills of the list at dst (16-bit part from piece s1);
// two passes (count the spills, then write), so the packed start n16 is known before any
// piece is written; returns (n16, packed pieces)
__device__ __forceinline__ uint2 nb_pack_seg2(const uint16_t *sb, uint32_t n2, uint16_t *dst,
                                              uint32_t s1, uint32_t pad_col) {
  const int lane = threadIdx.x & 63;
  const uint64_t ltmask = (1ull << lane) - 1ull;
  const uint32_t nc = n2 / 15u;
  // row cc's 16 slots as 8 words (slot 15 unused) and its minimum / maximum column, by
  // packed 16-bit min / max (v_pk_min_u16 / v_pk_max_u16: 8 + 2 a row instead of 28)
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  auto load_row = [&](uint32_t cc, uint32_t *w, uint32_t &mn, uint32_t &mx) {
    const uint4 a = *(const uint4 *)(sb + 16u * cc), b = *(const uint4 *)(sb + 16u * cc + 8u);
    w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    us2 lo = __builtin_bit_cast(us2, w[7] | 0xFFFF0000u), hi = __builtin_bit_cast(us2, w[7] & 0xFFFFu);
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      lo = __builtin_elementwise_min(lo, __builtin_bit_cast(us2, w[q]));
      hi = __builtin_elementwise_max(hi, __builtin_bit_cast(us2, w[q]));
    }
    mn = min((uint32_t)lo.x, (uint32_t)lo.y);
    mx = max((uint32_t)hi.x, (uint32_t)hi.y);
  };
  uint32_t nfail = 0;
  for (uint32_t c0 = 0; c0 < nc; c0 += 64u) {
    const uint32_t cc = c0 + (uint32_t)lane;
    bool bad = false;
    if (cc < nc) {
      uint32_t w[8], mn, mx;
      load_row(cc, w, mn, mx);
      bad = mx - mn > 254u;
    }
    nfail += (uint32_t)__popcll(__ballot(bad));
  }
  const uint32_t nt = n2 - 15u * nc;               // the last entries, past the runs of 15
  const uint32_t nleft = 15u * nfail + nt;         // entries of the 16-bit part
  const uint32_t l16 = (nleft + 7u) >> 3;
  const uint32_t n16 = s1 + l16;
  uint16_t *ldst = dst + s1 * 8u;
  uint4 *pdst = (uint4 *)(dst + n16 * 8u);
  uint32_t okc = 0, fc = 0;
  for (uint32_t c0 = 0; c0 < nc; c0 += 64u) {
    const uint32_t cc = c0 + (uint32_t)lane;
    const bool act = cc < nc;
    uint32_t v[15];
    uint32_t mn = 0xFFFFu, mx = 0u;
    if (act) {
      uint32_t w[8];
      load_row(cc, w, mn, mx);
#pragma unroll
      for (int e = 0; e < 15; ++e) v[e] = (e & 1) ? (w[e >> 1] >> 16) : (w[e >> 1] & 0xFFFFu);
    }
    const bool ok = act && mx - mn <= 254u;
    const uint64_t om = __ballot(ok), fm = __ballot(act && !ok);
    if (ok) {
      // the minimum to slot 0: its first occurrence takes v[0]'s value
      bool done = v[0] == mn;
#pragma unroll
      for (int e = 1; e < 15; ++e) {
        const bool sw = !done && v[e] == mn;
        v[e] = sw ? v[0] : v[e];
        done = done || sw;
      }
      uint32_t o[15];
#pragma unroll
      for (int e = 1; e < 15; ++e) o[e] = v[e] - mn;
      pdst[okc + (uint32_t)__popcll(om & ltmask)] =
          make_uint4(mn | (o[1] << 16) | (o[2] << 24), o[3] | (o[4] << 8) | (o[5] << 16) | (o[6] << 24),
                     o[7] | (o[8] << 8) | (o[9] << 16) | (o[10] << 24),
                     o[11] | (o[12] << 8) | (o[13] << 16) | (o[14] << 24));
    } else if (act) {
      const uint32_t l0 = 15u * (fc + (uint32_t)__popcll(fm & ltmask));
#pragma unroll
      for (int e = 0; e < 15; ++e) ldst[l0 + e] = (uint16_t)v[e];
    }
    okc += (uint32_t)__popcll(om);
    fc += (uint32_t)__popcll(fm);
  }
  // the last nt entries (row nc of the buffer), then the dummy columns of the last 16-bit piece
  if ((uint32_t)lane < nt) ldst[15u * nfail + lane] = sb[16u * nc + lane];
  {
    const uint32_t pp = nleft + (uint32_t)lane;
    if (lane < 8 && pp < l16 * 8u) ldst[pp] = nb_dummy(pad_col, s1 * 8u + pp);
  }
  return make_uint2(n16, nc - nfail);
}

typedef uint32_t nb_u32x4 __attribute__((ext_vector_type(4), aligned(4)));

struct NbStaged {
  uint32_t *dst;    // LDS words the run's destination entries are counted from
  uint32_t w[12];   // raw index words from base
  uint32_t dpos;    // destination entry
  uint32_t sh;      // source entry parity vs destination (0 / 1)
  uint32_t cm;      // entries moved through the words (the rest: 2-byte copies)
  uint32_t cnt, srcp;
};

__device__ __forceinline__ void nb_staged_load(NbStaged &r, const uint16_t *__restrict__ xent,
                                               uint32_t srcp, uint32_t cnt, uint32_t *dst,
                                               uint32_t dpos) {
  r.dst = dst;
  r.dpos = dpos;
  r.cnt = cnt;
  r.srcp = srcp;
  const uint32_t odd = dpos & 1u;
  r.cm = 0;
  r.sh = 0;
#pragma unroll
  for (int q = 0; q < 12; ++q) r.w[q] = 0u;
  if (cnt == 0 || srcp < odd) return;  // (srcp < odd: the index's first entry at an odd slot)
  const uint32_t s0 = srcp - odd;      // source entry of the destination word boundary
  const uint32_t sh = s0 & 1u, base = s0 - sh;
  const uint32_t nq = 12u - sh;        // whole shifted words the 3 loads hold
  const uint32_t cm = min(cnt, 2u * nq - odd);
  const uint32_t end = sh + odd + cm;  // raw halfwords used
  const nb_u32x4 *pp = (const nb_u32x4 *)(xent + base);
  const nb_u32x4 z = {0u, 0u, 0u, 0u};
  const nb_u32x4 p0 = pp[0];
  const nb_u32x4 p1 = end > 8u ? pp[1] : z;
  const nb_u32x4 p2 = end > 16u ? pp[2] : z;
  r.w[0] = p0.x; r.w[1] = p0.y; r.w[2] = p0.z; r.w[3] = p0.w;
  r.w[4] = p1.x; r.w[5] = p1.y; r.w[6] = p1.z; r.w[7] = p1.w;
  r.w[8] = p2.x; r.w[9] = p2.y; r.w[10] = p2.z; r.w[11] = p2.w;
  r.sh = sh;
  r.cm = cm;
}

__device__ __forceinline__ void nb_staged_write(const NbStaged &r, const uint16_t *__restrict__ xent,
                                                uint32_t *trash) {
  const uint32_t odd = r.dpos & 1u, wd = r.dpos >> 1, end = odd + r.cm;  // end: halfwords
  uint32_t *sb32 = r.dst;
  uint16_t *sb16 = (uint16_t *)sb32;
  uint32_t o[12];
#pragma unroll
  for (int q = 0; q < 12; ++q)
    o[q] = r.sh ? __builtin_amdgcn_alignbyte(q + 1 < 12 ? r.w[q + 1] : 0u, r.w[q], 2) : r.w[q];
#pragma unroll
  for (int q = 0; q < 12; ++q) {
    const bool full = (uint32_t)q >= odd && 2u * (uint32_t)q + 2u <= end;
    *(full ? sb32 + wd + (uint32_t)q : trash) = o[q];
  }
  // the two half words: the head (odd destination start) and the tail (odd end)
  const bool head = odd && r.cm > 0;
  *(head ? sb16 + r.dpos : (uint16_t *)trash) = (uint16_t)(o[0] >> 16);
  const uint32_t qt = (end - 1u) >> 1;
  uint32_t tv = o[0];
#pragma unroll
  for (int q = 1; q < 12; ++q) tv = qt == (uint32_t)q ? o[q] : tv;
  const bool tail = (end & 1u) && r.cm > 0;
  *(tail ? sb16 + 2u * wd + end - 1u : (uint16_t *)trash) = (uint16_t)tv;
  // the rest of a long run (or a run the words cannot start): 2-byte copies
  for (uint32_t e = r.cm; e < r.cnt; ++e) sb16[r.dpos + e] = xent[r.srcp + e];
}

template <int K>
__global__ __launch_bounds__(1024) void nb_fill_sorted_kernel(
    int64_t ngroups, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint2 *__restrict__ nbuse,
    uint16_t *__restrict__ table, uint32_t pad_col, int cap2, int nbk) {
  constexpr int S = 2, SW = 16, NT = 1024, NW = NT / 64;
  constexpr int kp = K - S;
  constexpr int mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;  // prefix ranges
  constexpr int nbn = 1 + 3 * K + 9 * K * (K - 1) / 2;
  constexpr int NIT = (nbn + 63) / 64;
  constexpr int t2 = 1 + 3 * K;  // first Hamming-2 run (< 64 for k <= 21)
  constexpr int NLD = (mr * (SW + 1) + NT - 1) / NT;
  extern __shared__ __align__(16) uint32_t fsm[];
  uint32_t *rt = fsm;                        // [nbn] run j: r | suffix xor << 16 | class << 24
  uint32_t *pm = rt + nbn;                   // [mr] prefix xor of range r
  uint32_t *roffs = pm + mr;                 // [2][mr][SW + 1] absolute index offsets
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t *hist = fsm + nb_staged_table_words(K) + wave * nbs_wave_words(nbk, cap2);  // [nbk]
  uint32_t *s01 = hist + ((nbk + 3) & ~3);   // segments 0 and 1 (NBS_S01 words)
  uint32_t *trash = s01 + NBS_S01 + lane;    // 64 words
  uint32_t *sb32 = s01 + NBS_S01 + 64;       // segment 2 (16-byte aligned)
  uint16_t *sbuf = (uint16_t *)sb32;
  const uint32_t npref = 1u << (2 * kp);
  nb_group_tables<S>(K, NT, rt, pm);
  __syncthreads();
  auto group_base = [&](int64_t gi, uint32_t &P) {
    P = (uint32_t)(gi & (int64_t)(npref - 1u));
    return (gi - P) * SW;  // chunk c's first bin: c * 4^k
  };
  uint32_t v[NLD];
  int64_t gi = blockIdx.x;
  if (gi < ngroups) {
    uint32_t P;
    const int64_t cb = group_base(gi, P);
    nb_ranges_issue<SW, NT, NLD>(xoff, cb, P, pm, mr, v);
    nb_ranges_store<SW, NT, NLD>(mr, v, roffs);
  }
  __syncthreads();
  for (int par = 0; gi < ngroups; gi += gridDim.x, par ^= 1) {
    uint32_t P;
    const int64_t cbase = group_base(gi, P);
    const uint32_t *roff = roffs + par * mr * (SW + 1);
    const int64_t gn = gi + gridDim.x;
    if (gn < ngroups) {  // the next group's range offsets: in flight during this group
      uint32_t Pn;
      const int64_t cbn = group_base(gn, Pn);
      nb_ranges_issue<SW, NT, NLD>(xoff, cbn, Pn, pm, mr, v);
    }
    for (int su = wave; su < SW; su += NW) {
      const int64_t b = cbase + (int64_t)P * SW + su;
      const uint32_t start = nboff[b], tot = nboff[b + 1] - start;
      if (tot == 0) continue;  // wave-uniform
      const uint2 sg = nbseg[b];
      uint16_t *dst = table + (size_t)start * 8u;
      // segment 2 past the buffer, or segments 0 + 1 past theirs: 16-bit lists
      if ((tot - sg.y) * 8u > (uint32_t)cap2 || sg.y * 8u > 2u * NBS_S01) {
        nb_list_lane_per_run(K, su, rt, roff, xent, tot, sg, dst, pad_col);
        if (lane == 0) nbuse[b] = make_uint2(tot, 0u);
        continue;
      }
      for (int q = lane; q < nbk; q += 64) hist[q] = 0u;
      // ---- 1. runs: segments 0 / 1 to s01 at their list positions, segment 2 to the buffer
      uint32_t carry = 0, n0 = 0, pre2 = 0;
      auto stage = [&](int it, NbStaged &r) {
        const int j = it * 64 + lane;
        uint32_t cnt = 0, srcp = 0, h = 2;
        if (j < nbn) {
          const uint32_t d = rt[j];
          const uint32_t *ro = roff + (d & 0xFFFFu) * (SW + 1);
          const uint32_t sidx = (uint32_t)su ^ ((d >> 16) & 0xFFu);
          h = d >> 24;
          srcp = ro[sidx];
          cnt = ro[sidx + 1] - srcp;
        }
        const uint32_t inc = nb_wave_incl_scan_dpp(cnt);
        const uint32_t pos = carry + inc - cnt;
        if (it == 0) {
          n0 = (uint32_t)__builtin_amdgcn_readlane((int)cnt, 0);
          pre2 = (uint32_t)__builtin_amdgcn_readlane((int)pos, t2 & 63);
        }
        carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (h < 2) nb_staged_load(r, xent, srcp, cnt, s01, (h == 0 ? 0u : sg.x * 8u - n0) + pos);
        else nb_staged_load(r, xent, srcp, cnt, sb32, pos - pre2);
      };
      NbStaged cur, nxt;
      stage(0, cur);
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        if (it + 1 < NIT) stage(it + 1, nxt);
        nb_staged_write(cur, xent, trash);
        if (it + 1 < NIT) cur = nxt;
      }
      const uint32_t n2 = carry - pre2;
      // dummy columns after segments 0 and 1
      if (lane < 16) {
        const int sgi = lane >> 3, e = lane & 7;
        const uint32_t segb = sgi == 0 ? 0u : sg.x * 8u;
        const uint32_t segn = sgi == 0 ? n0 : pre2 - n0;
        const uint32_t segend = sgi == 0 ? sg.x * 8u : sg.y * 8u;
        const uint32_t pp = segb + segn + (uint32_t)e;
        if (pp < segend) ((uint16_t *)s01)[pp] = nb_dummy(pad_col, pp);
      }
      nb_wave_sync();
      // segments 0 and 1 out (16-byte stores); segment 2 into registers + its histogram
      if ((uint32_t)lane < sg.y) ((uint4 *)dst)[lane] = ((const uint4 *)s01)[lane];
      for (uint32_t q = 64u + (uint32_t)lane; q < sg.y; q += 64u) ((uint4 *)dst)[q] = ((const uint4 *)s01)[q];
      uint2 rv[NBS_RW];
#pragma unroll
      for (int r = 0; r < NBS_RW; ++r) {
        const uint32_t e = 256u * (uint32_t)r + 4u * (uint32_t)lane;
        rv[r] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        if (e < n2) {
          rv[r] = *(const uint2 *)(sbuf + e);
          // entries past n2 in the last read: no entry (0xFFFF; columns < 65408)
          if (e + 1 >= n2) rv[r].x |= 0xFFFF0000u;
          if (e + 2 >= n2) rv[r].y |= 0x0000FFFFu;
          if (e + 3 >= n2) rv[r].y |= 0xFFFF0000u;
          const uint32_t c4[4] = {rv[r].x & 0xFFFFu, rv[r].x >> 16, rv[r].y & 0xFFFFu, rv[r].y >> 16};
#pragma unroll
          for (int hh = 0; hh < 4; ++hh)
            if (c4[hh] != 0xFFFFu) atomicAdd(&hist[c4[hh] >> NBS_BSH], 1u);
        }
      }
      nb_wave_sync();
      // ---- 2. bucket starts
      {  // rows of 64 buckets: every read issued first, then one wave scan a row
        constexpr int NR = NBS_MAXBK / 64;
        uint32_t hv[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r) hv[r] = (r * 64 + lane < nbk) ? hist[r * 64 + lane] : 0u;
        uint32_t carry = 0;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          if (r * 64 < nbk) {  // wave-uniform
            const uint32_t inc = nb_wave_incl_scan_dpp(hv[r]);
            if (r * 64 + lane < nbk) hist[r * 64 + lane] = carry + inc - hv[r];
            carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
          }
        }
      }
      nb_wave_sync();
      // ---- 3. counting sort from the registers: entry -> slot p + p / 15 of its position p
#pragma unroll
      for (int r = 0; r < NBS_RW; ++r) {
        if (256u * (uint32_t)r < n2) {  // wave-uniform
          const uint32_t c4[4] = {rv[r].x & 0xFFFFu, rv[r].x >> 16, rv[r].y & 0xFFFFu, rv[r].y >> 16};
#pragma unroll
          for (int hh = 0; hh < 4; ++hh) {
            if (c4[hh] != 0xFFFFu) {
              const uint32_t p = atomicAdd(&hist[c4[hh] >> NBS_BSH], 1u);
              sbuf[p + p / 15u] = (uint16_t)c4[hh];
            }
          }
        }
      }
      nb_wave_sync();
      // ---- 4. pack
      const uint2 us = nb_pack_seg2(sbuf, n2, dst, sg.y, pad_col);
      if (lane == 0) nbuse[b] = us;
      nb_wave_sync();  // the next list reuses the histogram and the buffers
    }
    if (gn < ngroups) nb_ranges_store<SW, NT, NLD>(mr, v, roffs + (par ^ 1) * mr * (SW + 1));
    __syncthreads();  // the next group reads the other range buffer
  }
}


// ------------------------------------------------------------------ staged 16-bit fill
// The 16-bit lists through LDS: one wave a list assembles the whole list (three segments,
// dummy tails) in a per-wave LDS buffer, then writes it with 16-byte stores (1 KB a wave
// instruction).  Lane j moves run j: three dword-aligned 16-byte loads of the index (the
// index is 2-byte entries; a dwordx4 load needs 4-byte alignment only) starting at the entry
// that lands on a destination word boundary, a 2-byte register shift when source and
// destination parities differ, then 32-bit LDS writes of the words whose halves are both the
// run's and 16-bit writes at its two ends -- ~9 LDS writes and 3 texture-address operations a
// run of ~7 entries, against 2 x 7 2-byte global operations for the lane-per-run copies
// (~25 TA cycles an instruction: the grouped fill is TA-bound, profiles/r04t_pmc_fill.txt).
// Writes that a lane does not need go to its own trash word (no exec-mask branching).  The
// runs of iteration i + 1 are loaded before iteration i's writes.  Lists past the buffer take
// the lane-per-run copies.
template <int K, int NT>
__global__ __launch_bounds__(NT) void nb_fill_staged_kernel(
    int64_t ngroups, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint2 *__restrict__ nbuse,
    uint16_t *__restrict__ table, uint32_t pad_col, int cap16) {
  constexpr int S = 2, SW = 16, NW = NT / 64;
  constexpr int kp = K - S;
  constexpr int mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;  // prefix ranges
  constexpr int nbn = 1 + 3 * K + 9 * K * (K - 1) / 2;
  constexpr int NIT = (nbn + 63) / 64;
  constexpr int t2 = 1 + 3 * K;
  extern __shared__ __align__(16) uint32_t fsm[];
  constexpr int NLD = (mr * (SW + 1) + NT - 1) / NT;
  uint32_t *rt = fsm;
  uint32_t *pm = rt + nbn;
  uint32_t *roffs = pm + mr;  // [2][mr][SW + 1]: this group's and the next one's
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t *sb32 = fsm + nb_staged_table_words(K) + wave * (cap16 / 2);  // 16-byte aligned
  uint32_t *trash = sb32 + cap16 / 2 - 64 + lane;                  // the buffer's last 64 words
  const uint32_t lcap = (uint32_t)cap16 - 128u;                    // entries a list may use
  const uint32_t npref = 1u << (2 * kp);
  nb_group_tables<S>(K, NT, rt, pm);
  __syncthreads();
  auto group_base = [&](int64_t gi, uint32_t &P) {
    P = (uint32_t)(gi & (int64_t)(npref - 1u));
    return (gi - P) * SW;
  };
  uint32_t v[NLD];
  int64_t gi = blockIdx.x;
  if (gi < ngroups) {
    uint32_t P;
    const int64_t cb = group_base(gi, P);
    nb_ranges_issue<SW, NT, NLD>(xoff, cb, P, pm, mr, v);
    nb_ranges_store<SW, NT, NLD>(mr, v, roffs);
  }
  __syncthreads();
  for (int par = 0; gi < ngroups; gi += gridDim.x, par ^= 1) {
    uint32_t P;
    const int64_t cbase = group_base(gi, P);
    const uint32_t *roff = roffs + par * mr * (SW + 1);
    const int64_t gn = gi + gridDim.x;
    if (gn < ngroups) {  // the next group's range offsets: in flight during this group
      uint32_t Pn;
      const int64_t cbn = group_base(gn, Pn);
      nb_ranges_issue<SW, NT, NLD>(xoff, cbn, Pn, pm, mr, v);
    }
    for (int su = wave; su < SW; su += NW) {
      const int64_t b = cbase + (int64_t)P * SW + su;
      const uint32_t start = nboff[b], tot = nboff[b + 1] - start;
      if (tot == 0) continue;  // wave-uniform
      const uint2 sg = nbseg[b];
      uint16_t *dst = table + (size_t)start * 8u;
      if (tot * 8u > lcap) {
        nb_list_lane_per_run(K, su, rt, roff, xent, tot, sg, dst, pad_col);
        if (lane == 0) nbuse[b] = make_uint2(tot, 0u);
        continue;
      }
      uint32_t carry = 0, n0 = 0, pre2 = 0;
      auto stage = [&](int it, NbStaged &r) {
        const int j = it * 64 + lane;
        uint32_t cnt = 0, srcp = 0, h = 2;
        if (j < nbn) {
          const uint32_t d = rt[j];
          const uint32_t *ro = roff + (d & 0xFFFFu) * (SW + 1);
          const uint32_t sidx = (uint32_t)su ^ ((d >> 16) & 0xFFu);
          h = d >> 24;
          srcp = ro[sidx];
          cnt = ro[sidx + 1] - srcp;
        }
        const uint32_t inc = nb_wave_incl_scan_dpp(cnt);
        const uint32_t pos = carry + inc - cnt;
        if (it == 0) {
          n0 = (uint32_t)__builtin_amdgcn_readlane((int)cnt, 0);
          pre2 = (uint32_t)__builtin_amdgcn_readlane((int)pos, t2 & 63);
        }
        carry += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        const uint32_t dpos = (h == 0 ? 0u : h == 1 ? sg.x * 8u - n0 : sg.y * 8u - pre2) + pos;
        nb_staged_load(r, xent, srcp, cnt, sb32, dpos);
      };
      NbStaged cur, nxt;
      stage(0, cur);
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        if (it + 1 < NIT) stage(it + 1, nxt);
        nb_staged_write(cur, xent, trash);
        if (it + 1 < NIT) cur = nxt;
      }
      const uint32_t total = carry;
      if (lane < 24) {  // dummy columns after each segment
        const int sgi = lane >> 3, e = lane & 7;
        const uint32_t segb = sgi == 0 ? 0u : sgi == 1 ? sg.x * 8u : sg.y * 8u;
        const uint32_t segn = sgi == 0 ? n0 : sgi == 1 ? pre2 - n0 : total - pre2;
        const uint32_t segend = sgi == 0 ? sg.x * 8u : sgi == 1 ? sg.y * 8u : tot * 8u;
        const uint32_t pp = segb + segn + (uint32_t)e;
        if (pp < segend) ((uint16_t *)sb32)[pp] = nb_dummy(pad_col, pp);
      }
      nb_wave_sync();
      for (uint32_t q = (uint32_t)lane; q < tot; q += 64u) ((uint4 *)dst)[q] = ((const uint4 *)sb32)[q];
      if (lane == 0) nbuse[b] = make_uint2(tot, 0u);
      nb_wave_sync();  // the next list reuses the buffer
    }
    if (gn < ngroups) nb_ranges_store<SW, NT, NLD>(mr, v, roffs + (par ^ 1) * mr * (SW + 1));
    __syncthreads();
  }
}

// ------------------------------------------------------------------ 16-bit grouped fill
// One workgroup per group of 16 lists, one wave a list (nb_list_lane_per_run).
__global__ __launch_bounds__(1024) void nb_fill_grouped_kernel(
    int k, int64_t ngroups, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint2 *__restrict__ nbuse,
    uint16_t *__restrict__ table, uint32_t pad_col) {
  constexpr int S = 2, SW = 16, NT = 1024, NW = NT / 64;
  extern __shared__ __align__(16) uint32_t fsm[];
  const int kp = k - S;
  const int mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;  // prefix ranges
  const int nbn = nb_neighbours(k);
  uint32_t *rt = fsm;
  uint32_t *pm = rt + nbn;
  uint32_t *roff = pm + mr;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t npref = 1u << (2 * kp);
  nb_group_tables<S>(k, NT, rt, pm);
  __syncthreads();
  for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const uint32_t P = (uint32_t)(gi & (int64_t)(npref - 1u));
    const int64_t cbase = (gi - P) * SW;
    if (nboff[gi * SW + SW] == nboff[gi * SW]) continue;
    nb_load_range_offsets<SW, NT>(xoff, cbase, P, pm, mr, roff);
    __syncthreads();
    for (int su = wave; su < SW; su += NW) {
      const int64_t b = cbase + (int64_t)P * SW + su;
      const uint32_t start = nboff[b], tot = nboff[b + 1] - start;
      if (tot == 0) continue;  // wave-uniform
      nb_list_lane_per_run(k, su, rt, roff, xent, tot, nbseg[b], table + (size_t)start * 8u, pad_col);
      if (lane == 0) nbuse[b] = make_uint2(tot, 0u);
    }
    __syncthreads();
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
__global__ __launch_bounds__(1024) void nb_fill_pieces_kernel(
    int k, int64_t ngroups, const uint32_t *__restrict__ xoff, const uint16_t *__restrict__ xent,
    const uint32_t *__restrict__ nboff, const uint2 *__restrict__ nbseg, uint2 *__restrict__ nbuse,
    uint16_t *__restrict__ table, uint32_t pad_col, int cap) {
  constexpr int S = 2, SW = 16, NT = 1024, NW = NT / 64;
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
  const uint64_t ltmask = (1ull << lane) - 1ull;
  uint16_t *re = tabs + wave * tw;   // [nbn + 1] destination end of non-empty run idx
  uint16_t *rsd = re + nbn + 1;      // [nbn + 1] image offset - destination start
  uint16_t *pst = rsd + nbn + 1;     // [NBP_MAXP] first run reaching piece p
  for (int64_t gi = blockIdx.x; gi < ngroups; gi += gridDim.x) {
    const uint32_t P = (uint32_t)(gi & (int64_t)(npref - 1u));
    const int64_t cbase = (gi - P) * SW;
    if (nboff[gi * SW + SW] == nboff[gi * SW]) continue;  // uniform
    // ---- 1. ranges: offsets, image positions (n + 14 words each: 8-aligned + source phase)
    nb_load_range_offsets<SW, NT>(xoff, cbase, P, pm, mr, roff);
    __syncthreads();
    uint32_t myn = 0;
    for (int r = threadIdx.x * rpt; r < min(mr, (int)(threadIdx.x + 1) * rpt); ++r)
      myn += roff[r * (SW + 1) + SW] - roff[r * (SW + 1)] + 14u;
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
        const uint32_t a = roff[r * (SW + 1)];
        rbase[r] = ((run + 7u) & ~7u) + (a & 7u);
        run += roff[r * (SW + 1) + SW] - a + 14u;
      }
      if (threadIdx.x == 0) rbase[mr] = total;
      __syncthreads();
    }
    const bool staged = rbase[mr] <= (uint32_t)cap;
    // ---- 2. the image: whole 16-byte pieces of each range, one wave a range
    if (staged) {
      for (int r = wave; r < mr; r += NW) {
        const uint32_t a = roff[r * (SW + 1)], n = roff[r * (SW + 1) + SW] - a;
        if (n == 0) continue;
        const uint32_t fp = a >> 3, lp = (a + n + 7u) >> 3;
        uint16_t *d0 = img + (rbase[r] - (a & 7u));
        for (uint32_t pc = fp + (uint32_t)lane; pc < lp; pc += 64u)
          *(uint4 *)(d0 + 8u * (pc - fp)) = ((const uint4 *)xent)[pc];
      }
    }
    __syncthreads();
    // ---- 3. the group's 16 lists, one wave a list
    for (int su = wave; su < SW; su += NW) {
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
          si = rbase[r] + (a0 - ro[0]);
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
          nb_copy_run(dst + dpos, xent + a0, cnt);
        }
      }
      const uint32_t total = carry;
      if (pieces) {
        if (lane == 0) {
          re[nzc] = (uint16_t)(tot * 8u);  // sentinel: past every entry
          rsd[nzc] = 0;
        }
        nb_wave_sync();
        for (uint32_t idx = (uint32_t)lane; idx <= nzc; idx += 64u) {
          const uint32_t lo = idx ? re[idx - 1] : 0u, hi = re[idx];
          for (uint32_t p = (lo + 7u) >> 3; p < ((hi + 7u) >> 3); ++p) pst[p] = (uint16_t)idx;
        }
        nb_wave_sync();
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
                v = nb_dummy(pad_col, d);
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
        nb_wave_sync();  // the next list overwrites the tables
      } else if (lane < 24) {
        // dummy columns after each segment, spread over 64 LDS words of the Gram kernel
        const int sgi = lane >> 3, e = lane & 7;
        const uint32_t segb = sgi == 0 ? 0u : sgi == 1 ? sg.x * 8u : sg.y * 8u;
        const uint32_t segn = sgi == 0 ? n0 : sgi == 1 ? pre2 - n0 : total - pre2;
        const uint32_t segend = sgi == 0 ? sg.x * 8u : sgi == 1 ? sg.y * 8u : tot * 8u;
        const uint32_t pp = segb + segn + (uint32_t)e;
        if (pp < segend) dst[pp] = nb_dummy(pad_col, pp);
      }
      if (lane == 0) nbuse[b] = make_uint2(tot, 0u);
    }
    __syncthreads();  // the next group overwrites the image
  }
}

// ------------------------------------------------------------------ Gram
// One workgroup per (row i, column chunk c) -- an ITEM of the row-accumulator grid
// (rowacc_block: chunk-major, upper block triangle for a full square K) -- accumulating
// the row over the chunk in an int32 LDS accumulator, then streaming it out through the
// fused normalize_K epilogue (emit_row).  The row's window table -- per window (list start,
// 16-bit pieces, segment ends, packed pieces) and two prefix sums -- splits the row's
// pieces evenly over the 16 waves: first the 16-bit pieces (8 columns, weight by segment),
// then the packed ones (15 columns, weight w2), NB_UNROLL 16-byte loads a lane a batch, one
// ds_add a column.
// TWO workgroups a CU: their table build, epilogue and streaming overlap.  At a 20000-column
// chunk (configs 3 and 5) the accumulator alone is 80000 B of the 81920 B each may hold, so
// the table is kept to 4 P + 2 words (segment ends as two halfwords, 16 dummy columns) --
// the round-4 measurement of the same kernel with one workgroup a CU (a double-buffered
// table, 84.9 KB) was 22 % slower (2.60 vs 2.13 ms, N=20000, profiles/r05g_*: half the
// resident waves); a persistent form (a wave building the next row's table) and two load
// batches in flight a wave measured slower still (profiles/r05f_*).
namespace {
// descriptor words of one row: wst[P] wc16[P+1] wseg[P] wcp[P+1] srec[ldp]
__host__ __device__ inline int nb_desc_words(int P, int64_t ldp) { return 4 * P + 2 + (int)ldp; }

// the segment ends of a list as halfwords (s0 | s1 << 16); 0xFFFFFFFF when s1 >= 0xFFFF
// (lists of more than ~520000 Hamming <= 1 entries in one chunk): the stream re-reads them
__device__ __forceinline__ uint32_t nb_seg_word(uint2 sg) {
  return sg.y < 0xFFFFu ? (sg.x | (sg.y << 16)) : 0xFFFFFFFFu;
}

// one wave: inclusive prefix of wc[1 .. P] (wc[0] = 0)
__device__ __forceinline__ void nb_wave_prefix(uint32_t *wc, int P) {
  const int lane = threadIdx.x & 63;
  const int per = (P + 63) >> 6, lo = lane * per, hi = min(P, lo + per);
  uint32_t s = 0;
  for (int a = lo; a < hi; ++a) s += wc[a + 1];
  uint32_t run = nb_wave_incl_scan_dpp(s) - s;
  for (int a = lo; a < hi; ++a) {
    run += wc[a + 1];
    wc[a + 1] = run;
  }
  if (lane == 0) wc[0] = 0;
}

// the window of piece q: the last a with wc[a] <= q
__device__ __forceinline__ int nb_find_window(const uint32_t *wc, int P, uint32_t q) {
  int lo = 0, hi = P - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (wc[mid] <= q) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
}  // namespace

template <int K, int NB_UNROLL>
__global__ __launch_bounds__(1024) void gram_nb_kernel(IndexGeom g, Packed pk,
                                                       const uint32_t *__restrict__ nboff,
                                                       const uint2 *__restrict__ nbseg,
                                                       const uint2 *__restrict__ nbuse,
                                                       const uint4 *__restrict__ table,
                                                       int64_t row0, int64_t rows, int w0, int w1,
                                                       int w2, OutSpec o) {
  extern __shared__ __align__(16) uint32_t smem[];
  int c;
  int64_t il;
  rowacc_block(g, o, row0, rows, c, il);
  const int64_t i = row0 + il;
  const int64_t col0 = (int64_t)c * g.chunk;
  const int cw = (int)min((int64_t)g.chunk, g.n - col0);
  if (col0 + cw <= o.col_lo) return;  // the whole chunk lies below the written columns
  const int accw = ((g.chunk + 3) >> 2) << 2;
  const int accn = accw + NB_DUMMIES;  // counters + the dummy columns
  const int P = g.pmax;
  uint32_t *wst = smem + accn;        // [P] list start of window a (pieces)
  uint32_t *wc16 = wst + P;           // [P + 1] 16-bit pieces of windows < a
  uint32_t *wseg = wc16 + P + 1;      // [P] segment ends (nb_seg_word)
  uint32_t *wcp = wseg + P;           // [P + 1] packed pieces of windows < a
  uint32_t *srec = wcp + P + 1;       // packed row record
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  stage_record(pk, i, srec);
  __syncthreads();
  const uint32_t cbase = (uint32_t)c << (2 * K);
  for (int a = threadIdx.x; a < P; a += blockDim.x) {
    const uint32_t u = pk_window(srec, pk.cw, a, K);
    uint32_t st = 0, n16 = 0, sw = 0, np = 0;
    if (u != KMG_INVALID) {
      const uint32_t b = cbase + u;
      st = nboff[b];
      const uint32_t en = nboff[b + 1];
      const uint2 sg = nbseg[b], us = nbuse[b];  // (nbuse is stale for an empty list)
      if (en != st) {
        sw = nb_seg_word(sg);
        n16 = us.x;
        np = us.y;
      }
    }
    wst[a] = st;
    wc16[a + 1] = n16;
    wseg[a] = sw;
    wcp[a + 1] = np;
  }
  {
    uint4 *acc4 = (uint4 *)smem;
    for (int w = threadIdx.x; w < (accn >> 2); w += blockDim.x) acc4[w] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  if (wave == 0) nb_wave_prefix(wc16, P);
  if (wave == 1) nb_wave_prefix(wcp, P);
  __syncthreads();
  int32_t *acc = (int32_t *)smem;
  char *accb = (char *)smem;
  // ---- 16-bit pieces: segment 0 (w0), segment 1 (w1), the 16-bit part of segment 2 (w2)
  {
    const uint32_t T = wc16[P];
    const uint32_t qb = (uint32_t)(((uint64_t)T * wave) / nw), qe = (uint32_t)(((uint64_t)T * (wave + 1)) / nw);
    uint32_t q = qb + lane;
    int a = q < qe ? nb_find_window(wc16, P, q) : 0;
    uint32_t abeg = wc16[a], aend = wc16[a + 1], ast = wst[a], as0 = 0, as1 = 0;
    auto segs = [&]() {
      const uint32_t sw = wseg[a];
      if (sw != 0xFFFFFFFFu) {
        as0 = sw & 0xFFFFu;
        as1 = sw >> 16;
      } else {  // ends past 16 bits: from the table of segment ends
        const uint2 sg = nbseg[cbase + pk_window(srec, pk.cw, a, K)];
        as0 = sg.x;
        as1 = sg.y;
      }
    };
    segs();
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
            aend = wc16[a + 1];
            ast = wst[a];
            segs();
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
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            atomicAdd(&acc[x[h] & 0xFFFFu], wt[t]);
            atomicAdd(&acc[x[h] >> 16], wt[t]);
          }
        }
      }
    }
  }
  // ---- packed pieces of segment 2: column c0 (low half of word 0) + 14 byte offsets
  {
    const uint32_t T = wcp[P];
    const uint32_t qb = (uint32_t)(((uint64_t)T * wave) / nw), qe = (uint32_t)(((uint64_t)T * (wave + 1)) / nw);
    uint32_t q = qb + lane;
    int a = q < qe ? nb_find_window(wcp, P, q) : 0;
    uint32_t abeg = wcp[a], aend = wcp[a + 1], ast = wst[a] + (wc16[a + 1] - wc16[a]);
    for (; q < qe; q += 64 * NB_UNROLL) {
      uint4 v[NB_UNROLL];
      bool ok[NB_UNROLL];
#pragma unroll
      for (int t = 0; t < NB_UNROLL; ++t) {
        const uint32_t qq = q + 64u * t;
        ok[t] = qq < qe;
        if (ok[t]) {
          while (qq >= aend) {
            ++a;
            abeg = aend;
            aend = wcp[a + 1];
            ast = wst[a] + (wc16[a + 1] - wc16[a]);
          }
          v[t] = table[(uint64_t)ast + (qq - abeg)];
        }
      }
#pragma unroll
      for (int t = 0; t < NB_UNROLL; ++t) {
        if (ok[t]) {
          // byte addresses: 4 (c0 + o) = 4 c0 + ((word >> (8 b - 2)) & 0x3FC) for byte b
          const uint32_t b4 = (v[t].x & 0xFFFFu) << 2;
          atomicAdd((int *)(accb + b4), w2);
          atomicAdd((int *)(accb + b4 + ((v[t].x >> 14) & 0x3FCu)), w2);
          atomicAdd((int *)(accb + b4 + ((v[t].x >> 22) & 0x3FCu)), w2);
          const uint32_t y[3] = {v[t].y, v[t].z, v[t].w};
#pragma unroll
          for (int h = 0; h < 3; ++h) {
            atomicAdd((int *)(accb + b4 + ((y[h] << 2) & 0x3FCu)), w2);
            atomicAdd((int *)(accb + b4 + ((y[h] >> 6) & 0x3FCu)), w2);
            atomicAdd((int *)(accb + b4 + ((y[h] >> 14) & 0x3FCu)), w2);
            atomicAdd((int *)(accb + b4 + ((y[h] >> 22) & 0x3FCu)), w2);
          }
        }
      }
    }
  }
  __syncthreads();
  const bool norm = o.normalize && o.diagv[0] != 1.0;
  emit_row<true>(o, il, i, col0, cw, acc, norm);
}


// KMG_CHECK=1: the list metadata gram_nb_kernel trusts without a bound, validated after every
// fill.  For each list: start <= end <= the table's pieces; non-empty: segment ends s0 <= s1
// <= n16 (segments 0 / 1 lie in the 16-bit part) and n16 + np <= the list's span (the packed
// pieces end inside it; the sorted fill shrinks a list, never grows it).  A violation sets
// bit 0 of *flag (a vector-memory atomic) and records the first offending list in flag[1].
__global__ __launch_bounds__(256) void nb_check_kernel(int64_t nbins, const uint32_t *__restrict__ nboff,
                                                       const uint2 *__restrict__ nbseg,
                                                       const uint2 *__restrict__ nbuse,
                                                       uint64_t table_pieces, uint32_t *flag) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nbins) return;
  const uint32_t st = nboff[b], en = nboff[b + 1];
  bool bad = en < st || (uint64_t)en > table_pieces;
  if (!bad && en != st) {
    const uint2 sg = nbseg[b], us = nbuse[b];
    bad = sg.x > sg.y || sg.y > us.x || (uint64_t)us.x + us.y > (uint64_t)(en - st);
  }
  if (bad) {
    atomicOr(flag, 1u);
    atomicMin(flag + 1, (uint32_t)min<int64_t>(b, 0xFFFFFFFFLL));
  }
}

// ------------------------------------------------------------------ host side
hipError_t launch_nb_check(int64_t nbins, const uint32_t *nboff, const uint2 *nbseg,
                           const uint2 *nbuse, uint64_t table_pieces, uint32_t *flag,
                           hipStream_t s) {
  if (nbins <= 0) return hipSuccess;
  hipLaunchKernelGGL(nb_check_kernel, dim3((unsigned)((nbins + 255) / 256)), dim3(256), 0, s, nbins,
                     nboff, nbseg, nbuse, table_pieces, flag);
  return hipGetLastError();
}

int64_t nb_list_entries_bound(int k, int64_t occurrences, int64_t nbins) {
  // every occurrence sits in the lists of its 1 + 3k + 9k(k-1)/2 neighbours; a non-empty list
  // pads each of its three segments by at most 7 entries
  const int64_t e = (int64_t)(1 + 3 * k + 9 * k * (k - 1) / 2) * occurrences;
  return e + 21 * std::min(nbins, e);
}

size_t nb_gram_lds(const IndexGeom &g, const Packed &pk) {
  const int accw = ((g.chunk + 3) >> 2) << 2;
  return (size_t)(accw + NB_DUMMIES + nb_desc_words(g.pmax, pk.ldp)) * 4;
}

// Hamming-2 entries of a list per column of the chunk (chunk x P / 4^k occurrences of a
// k-mer, 9 k (k-1) / 2 neighbours)
static double nb_seg2_density(int k, int pmax) {
  return 4.5 * k * (k - 1) * (double)pmax / (double)(1ull << (2 * k));
}

int nb_sorted_cap(int k, int pmax, int chunk) {
  if (k < 4 || k > 12) return 0;
  const double dens = nb_seg2_density(k, pmax);
  // 15 entries must span <= 254 columns: at ~12 columns between entries (14 x 12 = 168) the
  // runs still fit; k = 10 (28 columns) would spill nearly every run
  if (dens < 1.0 / 12.0) return 0;
  const int nbk = (chunk + (1 << NBS_BSH) - 1) >> NBS_BSH;
  if (nbk > NBS_MAXBK) return 0;
  const int64_t per_wave = (160 * 1024 / 4 - nb_staged_table_words(k)) / 16;  // words, 16 waves
  // buffer words a wave: 8 a row of 15 entries
  const int64_t rows = (per_wave - ((nbk + 3) & ~3) - NBS_S01 - 64) / 8;
  int64_t cap = std::min<int64_t>(rows * 15, NBS_MAXCAP);
  // the buffer holds segment 2 of a list of the mean + 10 % (a sum of ~320 runs: sizes stay
  // within a few % of the mean; a longer list stays 16-bit)
  if (cap <= 0 || (double)cap < 1.1 * dens * chunk + 64) return 0;
  return (int)(cap & ~7LL);
}

int nb_sorted_max_chunk(int k, int pmax) {
  const double dens = nb_seg2_density(k, pmax);
  if (k < 4 || k > 12 || dens < 1.0 / 12.0) return 0;
  int lo = 8, hi = 65536 - 128;
  if (!nb_sorted_cap(k, pmax, lo)) return 0;
  while (lo < hi) {  // nb_sorted_cap is non-zero on a prefix of chunk sizes
    const int mid = (lo + hi + 1) / 2;
    if (nb_sorted_cap(k, pmax, mid)) lo = mid;
    else hi = mid - 1;
  }
  return lo & ~7;
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
                          const uint32_t *nboff, const uint2 *nbseg, uint2 *nbuse,
                          uint16_t *table, hipStream_t s, int form, int fill_threads) {
  const int64_t nbins = g.nbins();
  if (g.copies != 1 || g.k < 4 || g.k > 12) return hipErrorInvalidValue;
  const uint32_t pad_col = (uint32_t)(((g.chunk + 3) >> 2) << 2);
  const double mean = (double)g.chunk * g.pmax / (double)g.nkeys;  // occurrences of a k-mer
  const int64_t ngroups = nbins / 16;
  const int cap = nb_sorted_cap(g.k, g.pmax, g.chunk);
  if ((form == 0 || form == 1) && cap > 0) {
    // sorted fill, packed segment 2 (the Gram reads ~0.6x the bytes of 16-bit lists)
    const int nbk = (g.chunk + (1 << NBS_BSH) - 1) >> NBS_BSH;
    const size_t lds = 4 * ((size_t)nb_staged_table_words(g.k) + 16 * (size_t)nbs_wave_words(nbk, cap));
    if (lds > 160 * 1024 || (((uintptr_t)xent) & 3u) != 0) return hipErrorInvalidValue;
    const int64_t blocks = std::min<int64_t>(ngroups, 256);
    switch (g.k) {
#define KMG_NB_SORTED(KK)                                                                        \
  case KK:                                                                                       \
    hipLaunchKernelGGL(nb_fill_sorted_kernel<KK>, dim3((unsigned)blocks), dim3(1024), lds, s,    \
                       ngroups, xoff, xent, nboff, nbseg, nbuse, table, pad_col, cap, nbk);      \
    break;
      KMG_NB_SORTED(4) KMG_NB_SORTED(5) KMG_NB_SORTED(6) KMG_NB_SORTED(7) KMG_NB_SORTED(8)
      KMG_NB_SORTED(9) KMG_NB_SORTED(10) KMG_NB_SORTED(11) KMG_NB_SORTED(12)
#undef KMG_NB_SORTED
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (form == 1) return hipErrorInvalidValue;  // forced sorted fill where it cannot run
  if (form == 0 || form == 4 || form == 5) {
    // staged 16-bit fill: the whole list in a per-wave LDS buffer, 16-byte stores
    // (lists are sums of ~350 runs: their sizes stay within a few % of the mean; the rare
    // longer one takes the lane-per-run copies)
    // 512-thread workgroups, two a CU, each with its own groups and barriers, where a list
    // fits their smaller per-wave buffer (N=20000 fill 0.62 -> 0.60 ms, rank slab 5.50 ->
    // 5.40, profiles/r05at_fill_threads.jsonl); else 1024
    const double mean_list = (double)(1 + 3 * g.k + 9 * g.k * (g.k - 1) / 2) * mean;
    const int cap512 = ((80 * 1024 / 4 - nb_staged_table_words(g.k)) / 8 * 2) & ~7;
    const bool w512 = fill_threads == 512 && cap512 >= 1.08 * mean_list + 192;
    const int cap16 = w512 ? cap512 : ((160 * 1024 / 4 - nb_staged_table_words(g.k)) / 16 * 2) & ~7;
    if (cap16 >= 1.08 * mean_list + 192 && (((uintptr_t)xent) & 3u) == 0) {
      const size_t lds = 4 * ((size_t)nb_staged_table_words(g.k) + (w512 ? 8 : 16) * (size_t)(cap16 / 2));
      const int64_t blocks = std::min<int64_t>(ngroups, w512 ? 512 : 256);
      switch (g.k) {
#define KMG_NB_STAGED(KK)                                                                        \
  case KK:                                                                                       \
    if (w512)                                                                                    \
      hipLaunchKernelGGL((nb_fill_staged_kernel<KK, 512>), dim3((unsigned)blocks), dim3(512), lds, \
                         s, ngroups, xoff, xent, nboff, nbseg, nbuse, table, pad_col, cap16);    \
    else                                                                                         \
      hipLaunchKernelGGL((nb_fill_staged_kernel<KK, 1024>), dim3((unsigned)blocks), dim3(1024),  \
                         lds, s, ngroups, xoff, xent, nboff, nbseg, nbuse, table, pad_col, cap16); \
    break;
        KMG_NB_STAGED(4) KMG_NB_STAGED(5) KMG_NB_STAGED(6) KMG_NB_STAGED(7) KMG_NB_STAGED(8)
        KMG_NB_STAGED(9) KMG_NB_STAGED(10) KMG_NB_STAGED(11) KMG_NB_STAGED(12)
#undef KMG_NB_STAGED
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    if (form == 4) return hipErrorInvalidValue;
  }
  // 16-bit lists.  The piece-assembled fill where a list's runs are long enough for its fixed
  // cost per group (~7 us of range offsets + image loads) to pay: N=200000 rank slab (7
  // chunks of 28572 columns, 10.1 occurrences a k-mer and chunk) fill 9.1 -> 7.0 ms; at
  // N=20000 (7.1) the lane-per-run copies stay ahead, 1.25 vs 1.30 ms
  // (profiles/r04_nb_fill.jsonl r04z).  KMG_NB_FILL: 2 grouped, 3 pieces.
  const bool pieces = form == 3 || (form != 2 && mean >= 8.5);
  if (pieces && (((uintptr_t)xent) & 15u) == 0) {
    const size_t fixed = 4 * (size_t)nb_pieces_img_word(g.k, 1024);
    const size_t avail = (size_t)160 * 1024;
    const int cap = fixed < avail ? (int)std::min<size_t>((avail - fixed) / 2, 65528) & ~7 : 0;
    if (cap >= 1024) {
      const size_t lds = fixed + 2 * (size_t)cap;
      const int64_t blocks = std::min<int64_t>(ngroups, 256);
      hipLaunchKernelGGL(nb_fill_pieces_kernel, dim3((unsigned)blocks), dim3(1024), lds, s, g.k,
                         ngroups, xoff, xent, nboff, nbseg, nbuse, table, pad_col, cap);
      return hipGetLastError();
    }
  }
  const int kp = g.k - 2, mr = 1 + 3 * kp + 9 * kp * (kp - 1) / 2;
  const int nbn = 1 + 3 * g.k + 9 * g.k * (g.k - 1) / 2;
  const size_t lds = sizeof(uint32_t) * ((size_t)nbn + mr + (size_t)mr * 17);
  const int64_t blocks = std::min<int64_t>(ngroups, 256 * 16);
  hipLaunchKernelGGL(nb_fill_grouped_kernel, dim3((unsigned)blocks), dim3(1024), lds, s, g.k,
                     ngroups, xoff, xent, nboff, nbseg, nbuse, table, pad_col);
  return hipGetLastError();
}

hipError_t launch_gram_mismatch1_nb(const IndexGeom &g, const Packed &pk, const uint32_t *nboff,
                                    const uint2 *nbseg, const uint2 *nbuse, const uint4 *table,
                                    int64_t row0, int64_t row1, int w0, int w1, int w2,
                                    const OutSpec &o, hipStream_t s, int threads, int unroll) {
  const int64_t rows = row1 - row0;
  if (rows <= 0 || g.n == 0) return hipSuccess;
  if (g.k < 4 || g.k > 12 || g.copies != 1) return hipErrorNotSupported;
  if (threads != 512 && threads != 1024) return hipErrorInvalidValue;
  const int64_t nblk = rowacc_blocks(g, o, row0, rows);
  if (nblk * threads >= (1LL << 32)) return hipErrorInvalidValue;  // AQL grid size is 32-bit
  if (g.chunk + NB_DUMMIES + 63 >= 65536) return hipErrorInvalidValue;  // uint16 columns
  const size_t lds = nb_gram_lds(g, pk);
  if (lds > (threads == 512 ? 80 : 160) * 1024) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nblk);
  switch (g.k) {
#define KMG_NB(KK)                                                                              \
  case KK:                                                                                      \
    if (unroll == 4)                                                                            \
      hipLaunchKernelGGL((gram_nb_kernel<KK, 4>), grid, dim3(threads), lds, s, g, pk, nboff,   \
                         nbseg, nbuse, table, row0, rows, w0, w1, w2, o);                       \
    else                                                                                        \
      hipLaunchKernelGGL((gram_nb_kernel<KK, 8>), grid, dim3(threads), lds, s, g, pk, nboff,   \
                         nbseg, nbuse, table, row0, rows, w0, w1, w2, o);                       \
    break;
    KMG_NB(4) KMG_NB(5) KMG_NB(6) KMG_NB(7) KMG_NB(8) KMG_NB(9) KMG_NB(10) KMG_NB(11) KMG_NB(12)
#undef KMG_NB
  }
  return hipGetLastError();
}

}  // namespace kmg
