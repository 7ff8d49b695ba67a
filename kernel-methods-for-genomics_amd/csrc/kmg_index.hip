// kmg_index.hip — k-mer posting index on gfx950.
//
// Replaces the dense feature vectors of the reference:
//   get_phi_u  (kernels.py:12-25):  phi_u[b] = #{i < len(x)-k+1 : x[i:i+k] == b}
//   get_phi_km (kernels.py:161-175): phi_km[b] = #{i < 101-k+1 : ham(x[i:i+k], b) <= m}
// Instead of 4^k-wide float64 rows we keep, per k-mer key, the list of columns
// (sequences) holding it ("postings").  The Gram kernels then accumulate one row of
// K at a time in LDS (kmg_gram.hip).
//
// Layout: bins = [copy][chunk][key]; off[bin] .. off[bin+1] indexes ent[].
// ent is uint16: column inside the chunk (SP: 16 bits; MM: low 14 bits) | letter at
// the dropped position << 14 (MM).  Order inside a bin is unspecified (the Gram is
// an integer sum, so results do not depend on it).
//
// Build = two-launch MSD partition with LDS histograms, no global atomics (see
// "index build" below): per-block local sort by coarse bucket, then one block per bucket
// places its fine bins.
#include "kmg_internal.h"

namespace kmg {

__device__ __forceinline__ uint32_t letter_at(uint32_t code, int p, int k) {
  return (code >> (2 * (k - 1 - p))) & 3u;
}
__device__ __forceinline__ uint32_t drop_letter(uint32_t code, int p, int k) {
  const uint64_t c = code;
  const int lo_bits = 2 * (k - 1 - p);
  return (uint32_t)(((c >> (lo_bits + 2)) << lo_bits) | (c & ((1ull << lo_bits) - 1ull)));
}

constexpr int IDX_THREADS = 1024;  // upper bound; blocks launch g.part_threads
constexpr int FINE_THREADS = 1024;

// symbols [32 b, 32 b + 32) of sequence j -> code words 2b, 2b+1 and mask word b
__device__ __forceinline__ void pack_piece(const uint8_t *__restrict__ codes,
                                           const int32_t *__restrict__ lens, int64_t ldc,
                                           int64_t j, int b, uint32_t &c0, uint32_t &c1,
                                           uint32_t &m) {
  const int len = min(max(lens[j], 0), (int)ldc);
  const uint8_t *r = codes + j * ldc;
  c0 = 0, c1 = 0, m = 0;
#pragma unroll 8
  for (int q = 0; q < 32; ++q) {
    const int pos = 32 * b + q;
    const uint32_t v = pos < len ? (uint32_t)r[pos] : 4u;
    m |= (v > 3u ? 1u : 0u) << q;
    const uint32_t sym = v & 3u;
    if (q < 16)
      c0 |= sym << (30 - 2 * q);
    else
      c1 |= sym << (30 - 2 * (q - 16));
  }
}

// fused 2-bit packing (part_local_kernel with codes != nullptr): pack the block's
// sequences straight into LDS and publish their records for the Gram kernels
__device__ __forceinline__ int stage_rows_packing(const IndexGeom &g, const Packed &pk,
                                                  const uint8_t *__restrict__ codes,
                                                  const int32_t *__restrict__ lens, int64_t ldc,
                                                  uint32_t *srec, int64_t j0) {
  const int ns = (int)min((int64_t)g.seqs_per_block, g.n - j0);
  const int cw = pk.cw, mw = (int)pk.ldp - pk.cw;
  const int nb = max((cw + 1) / 2, mw);
  for (int t = threadIdx.x; t < ns * nb; t += blockDim.x) {
    const int s = t / nb, b = t - s * nb;
    uint32_t c0, c1, m;
    pack_piece(codes, lens, ldc, j0 + s, b, c0, c1, m);
    uint32_t *lrec = srec + s * pk.ldp;
    uint32_t *grec = const_cast<uint32_t *>(pk.w) + (j0 + s) * pk.ldp;  // the context's record buffer
    if (2 * b < cw) lrec[2 * b] = grec[2 * b] = c0;
    if (2 * b + 1 < cw) lrec[2 * b + 1] = grec[2 * b + 1] = c1;
    if (b < mw) lrec[cw + b] = grec[cw + b] = m;
  }
  __syncthreads();
  return ns;
}

// stage the packed records (Packed, kmg_internal.h) of seqs_per_block sequences in LDS;
// returns the number of staged sequences
__device__ __forceinline__ int stage_rows(const IndexGeom &g, const Packed &pk, uint32_t *srec,
                                          int64_t j0) {
  const int ns = (int)min((int64_t)g.seqs_per_block, g.n - j0);
  const int words = ns * (int)pk.ldp;
  const uint32_t *src = pk.w + j0 * pk.ldp;
  for (int t = threadIdx.x; t < words; t += blockDim.x) srec[t] = src[t];
  __syncthreads();
  return ns;
}

// visit every (bin, value) item of the staged sequences: windows a < pmax whose k symbols
// are all A/C/G/T and inside the sequence (mask bits clear; kernels.py:21-24 drops the rest)
template <typename F>
__device__ __forceinline__ void for_items(const IndexGeom &g, const Packed &pk, const uint32_t *srec,
                                          int ns, int64_t j0, F &&f) {
  const int per = g.pmax;
  for (int t = threadIdx.x; t < ns * per; t += blockDim.x) {
    const int s = t / per, a = t - s * per;
    const uint32_t c = pk_window(srec + s * pk.ldp, pk.cw, a, g.k);
    if (c == KMG_INVALID) continue;
    const int64_t j = j0 + s;
    const int ch = (int)(j / g.chunk);
    const uint32_t col = (uint32_t)(j - (int64_t)ch * g.chunk);
    if (g.copies == 1) {
      f((uint32_t)(ch * (int64_t)g.nkeys + c), col);
    } else {
      for (int p = 0; p < g.copies; ++p) {
        const uint32_t rk = (drop_letter(c, p, g.k) << 2) | letter_at(c, p, g.k);
        f((uint32_t)(((int64_t)p * g.nchunks + ch) * g.nkeys + rk), col);
      }
    }
  }
}

// block-wide exclusive scan over an LDS array of length len (in place); returns total
__device__ uint32_t lds_excl_scan(uint32_t *a, int len, uint32_t *wtmp) {
  const int nt = blockDim.x, t = threadIdx.x;
  const int per = (len + nt - 1) / nt;
  const int b0 = t * per, b1 = min(len, b0 + per);
  uint32_t s = 0;
  for (int q = b0; q < b1; ++q) s += a[q];
  // wave scan
  const int lane = t & 63, wave = t >> 6, nw = nt >> 6;
  uint32_t inc = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(inc, d, 64);
    if (lane >= d) inc += v;
  }
  if (lane == 63) wtmp[wave] = inc;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < nw; ++w) {
    if (w < wave) base += wtmp[w];
    total += wtmp[w];
  }
  uint32_t run = base + inc - s;
  for (int q = b0; q < b1; ++q) {
    const uint32_t v = a[q];
    a[q] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

// ------------------------------------------------------------------ index build
// Two launches, no device-scope atomics and no communication between the workgroups of
// a launch (an earlier atomics-based build paid one device-scope atomic per (block, coarse
// bucket) on a few hundred hot words, serialised at the memory-side atomic unit):
//  (1) part_local_kernel: block q stages its sequences, builds the LDS histogram over the
//      coarse buckets, scans it, and writes its items bucket-sorted into its own region
//      of tmp (cap items).  Counts and local starts are published bucket-major:
//      hcnt[b * nblk + q], hstart[b * nblk + q].
//  (2) part_gather_kernel: one block per coarse bucket b.  The bucket's global start is
//      sum_q hstart[b][q] (every block's items of the buckets before b) and its size is
//      sum_q hcnt[b][q]; LDS fine histogram + scan -> off[], then the items are gathered
//      from every block's segment into ent[].  Results do not depend on dispatch order.
__global__ __launch_bounds__(IDX_THREADS) void part_local_kernel(
    IndexGeom g, Packed pk, const uint8_t *__restrict__ codes, const int32_t *__restrict__ lens,
    int64_t ldc, int nblk, uint32_t cap, uint32_t *__restrict__ hcnt,
    uint32_t *__restrict__ hstart, uint32_t *__restrict__ tmp) {
  extern __shared__ __align__(16) uint32_t sm[];
  __shared__ uint32_t wtmp[IDX_THREADS / 64];
  const int nbk = (int)g.nbuckets();
  uint32_t *h = sm;
  uint32_t *srec = h + nbk;
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) h[b] = 0;
  const int q = blockIdx.x;
  const int64_t j0 = (int64_t)q * g.seqs_per_block;
  const int ns = codes ? stage_rows_packing(g, pk, codes, lens, ldc, srec, j0)
                       : stage_rows(g, pk, srec, j0);
  const int fb = g.fine_bits;
  const uint32_t fmask = (1u << fb) - 1u;
  for_items(g, pk, srec, ns, j0, [&](uint32_t bin, uint32_t) { atomicAdd(&h[bin >> fb], 1u); });
  __syncthreads();
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) hcnt[(size_t)b * nblk + q] = h[b];
  __syncthreads();
  lds_excl_scan(h, nbk, wtmp);
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) hstart[(size_t)b * nblk + q] = h[b];
  __syncthreads();
  uint32_t *out = tmp + (size_t)q * cap;
  for_items(g, pk, srec, ns, j0, [&](uint32_t bin, uint32_t val) {
    const uint32_t pos = atomicAdd(&h[bin >> fb], 1u);
    out[pos] = ((bin & fmask) << 16) | val;
  });
}

__global__ __launch_bounds__(FINE_THREADS) void part_gather_kernel(
    IndexGeom g, int nblk, uint32_t cap, const uint32_t *__restrict__ hcnt,
    const uint32_t *__restrict__ hstart, const uint32_t *__restrict__ tmp,
    uint32_t *__restrict__ off, uint16_t *__restrict__ ent) {
  extern __shared__ __align__(16) uint32_t sm[];
  __shared__ uint32_t wtmp[FINE_THREADS / 64];
  __shared__ uint32_t red[2][FINE_THREADS / 64];
  const int fb = g.fine_bits, nf = 1 << fb;
  const int b = blockIdx.x;
  uint32_t *fh = sm;           // nf fine counters
  uint32_t *cnt = fh + nf;     // nblk: items of block q in bucket b
  uint32_t *src = cnt + nblk;  // nblk: where they start inside block q's region
  for (int f = threadIdx.x; f < nf; f += blockDim.x) fh[f] = 0;
  uint32_t s_cnt = 0, s_start = 0;
  const uint32_t *cb = hcnt + (size_t)b * nblk, *sb = hstart + (size_t)b * nblk;
  for (int q = threadIdx.x; q < nblk; q += blockDim.x) {
    const uint32_t c = cb[q], st = sb[q];
    cnt[q] = c;
    src[q] = st;
    s_cnt += c;
    s_start += st;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    s_cnt += __shfl_xor(s_cnt, d, 64);
    s_start += __shfl_xor(s_start, d, 64);
  }
  if (lane == 0) {
    red[0][wave] = s_cnt;
    red[1][wave] = s_start;
  }
  __syncthreads();
  uint32_t total = 0, base = 0;  // items of bucket b; items of all buckets before b
  for (int w = 0; w < nw; ++w) {
    total += red[0][w];
    base += red[1][w];
  }
  // Few blocks (nblk <= SEGR waves' worth, e.g. 250 at N=20000): every wave loads the
  // first 64 items of all its segments at once and keeps them in registers across the
  // scan, so both passes cost one L2 round trip (the loop below pays one per SEGU
  // segments and loads every item twice).  Longer segments finish in remainder loops.
  constexpr int SEGR = 16;
  if (nblk <= SEGR * nw) {
    uint32_t it[SEGR];
#pragma unroll
    for (int u = 0; u < SEGR; ++u) {
      const int q = wave + u * nw;
      it[u] = (q < nblk && (uint32_t)lane < cnt[q]) ? tmp[(size_t)q * cap + src[q] + lane] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < SEGR; ++u)
      if (it[u] != 0xFFFFFFFFu) atomicAdd(&fh[it[u] >> 16], 1u);
    for (int q = wave; q < nblk; q += nw) {
      const uint32_t c = cnt[q];
      const uint32_t *sp = tmp + (size_t)q * cap + src[q];
      for (uint32_t x = 64 + lane; x < c; x += 64) atomicAdd(&fh[sp[x] >> 16], 1u);
    }
    __syncthreads();
    lds_excl_scan(fh, nf, wtmp);
    const int64_t nb = g.nbins();
    const int64_t bin0 = (int64_t)b << fb;
    for (int f = threadIdx.x; f < nf; f += blockDim.x) {
      const int64_t bin = bin0 + f;
      if (bin < nb) off[bin] = base + fh[f];
    }
    if (b == (int)gridDim.x - 1 && threadIdx.x == 0) off[nb] = base + total;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SEGR; ++u) {
      if (it[u] != 0xFFFFFFFFu) {
        const uint32_t pos = atomicAdd(&fh[it[u] >> 16], 1u);
        ent[base + pos] = (uint16_t)(it[u] & 0xFFFFu);
      }
    }
    for (int q = wave; q < nblk; q += nw) {
      const uint32_t c = cnt[q];
      const uint32_t *sp = tmp + (size_t)q * cap + src[q];
      for (uint32_t x = 64 + lane; x < c; x += 64) {
        const uint32_t v = sp[x];
        const uint32_t pos = atomicAdd(&fh[v >> 16], 1u);
        ent[base + pos] = (uint16_t)(v & 0xFFFFu);
      }
    }
    return;
  }
  // the segments of a bucket are short (~30 items at N=20000): a wave loads the first 64
  // items of SEGU segments before using any, so the pass is not one L2 round trip per
  // segment; longer segments finish in the remainder loop
  constexpr int SEGU = 4;
  for (int q0 = wave; q0 < nblk; q0 += SEGU * nw) {
    uint32_t it[SEGU];
#pragma unroll
    for (int u = 0; u < SEGU; ++u) {
      const int q = q0 + u * nw;
      it[u] = (q < nblk && (uint32_t)lane < cnt[q]) ? tmp[(size_t)q * cap + src[q] + lane] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < SEGU; ++u)
      if (it[u] != 0xFFFFFFFFu) atomicAdd(&fh[it[u] >> 16], 1u);
#pragma unroll
    for (int u = 0; u < SEGU; ++u) {
      const int q = q0 + u * nw;
      if (q >= nblk) break;
      const uint32_t c = cnt[q];
      const uint32_t *sp = tmp + (size_t)q * cap + src[q];
      for (uint32_t x = 64 + lane; x < c; x += 64) atomicAdd(&fh[sp[x] >> 16], 1u);
    }
  }
  __syncthreads();
  lds_excl_scan(fh, nf, wtmp);
  const int64_t nb = g.nbins();
  const int64_t bin0 = (int64_t)b << fb;
  for (int f = threadIdx.x; f < nf; f += blockDim.x) {
    const int64_t bin = bin0 + f;
    if (bin < nb) off[bin] = base + fh[f];
  }
  if (b == (int)gridDim.x - 1 && threadIdx.x == 0) off[nb] = base + total;
  __syncthreads();
  for (int q0 = wave; q0 < nblk; q0 += SEGU * nw) {
    uint32_t it[SEGU];
#pragma unroll
    for (int u = 0; u < SEGU; ++u) {
      const int q = q0 + u * nw;
      it[u] = (q < nblk && (uint32_t)lane < cnt[q]) ? tmp[(size_t)q * cap + src[q] + lane] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < SEGU; ++u) {
      if (it[u] != 0xFFFFFFFFu) {
        const uint32_t pos = atomicAdd(&fh[it[u] >> 16], 1u);
        ent[base + pos] = (uint16_t)(it[u] & 0xFFFFu);
      }
    }
#pragma unroll
    for (int u = 0; u < SEGU; ++u) {
      const int q = q0 + u * nw;
      if (q >= nblk) break;
      const uint32_t c = cnt[q];
      const uint32_t *sp = tmp + (size_t)q * cap + src[q];
      for (uint32_t x = 64 + lane; x < c; x += 64) {
        const uint32_t v = sp[x];
        const uint32_t pos = atomicAdd(&fh[v >> 16], 1u);
        ent[base + pos] = (uint16_t)(v & 0xFFFFu);
      }
    }
  }
}

// Slot layout of the rotated mismatch index (read by gram_mm1s_kernel): one 128-byte line
// per 4-bin group (copy p, chunk, key): halfwords 0..3 = e1, e2, e3, tot (letter-bin ends
// relative to the group start, group total), halfwords 4.. = the group's first
// KMG_SLOT_INLINE entries in CSR order.  A group of >= 0xFFFF entries gets tot = 0xFFFF
// and no inline entries (the kernel then reads it from the CSR).  8 threads per group,
// each writes 16 bytes of the line.  Inline positions past the group's entries hold
// sentinel columns sent_base + hash(group, position) in [sent_base, sent_base + 1024):
// gram_mm1t_kernel<SENT> adds them into a scratch tail of its LDS accumulator instead of
// testing every slot (spread over 1024 dwords so lanes of one wave rarely collide).
__global__ __launch_bounds__(256) void slot_pack_kernel(int64_t ngroups, const uint32_t *__restrict__ off,
                                                        const uint16_t *__restrict__ ent,
                                                        uint32_t sent_base,
                                                        uint4 *__restrict__ slots) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t gi = t >> 3;
  const int q = (int)(t & 7);
  if (gi >= ngroups) return;
  const uint32_t *ob = off + gi * 4;
  const uint32_t o0 = ob[0], o4 = ob[4];
  const uint32_t tot = o4 - o0;
  const bool big = tot >= 0xFFFFu;
  uint32_t hw[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int h = q * 8 + s;
    uint32_t v = 0;
    if (h < 4) {
      v = big ? (h == 3 ? 0xFFFFu : 0u) : (h == 3 ? tot : ob[h + 1] - o0);
    } else {
      const uint32_t e = (uint32_t)(h - 4);
      v = (!big && e < tot) ? (uint32_t)ent[o0 + e]
                            : sent_base + (((uint32_t)gi * 97u + (uint32_t)h * 31u) & 1023u);
    }
    hw[s] = v;
  }
  slots[t] = make_uint4(hw[0] | (hw[1] << 16), hw[2] | (hw[3] << 16), hw[4] | (hw[5] << 16),
                        hw[6] | (hw[7] << 16));
}

hipError_t launch_slot_pack(const IndexGeom &g, const uint32_t *off, const uint16_t *ent,
                            uint4 *slots, hipStream_t s) {
  static_assert(KMG_SLOT_BYTES == 128 && KMG_SLOT_INLINE == 60, "slot layout");
  if (!g.rot) return hipErrorInvalidValue;
  const int64_t ngroups = g.nbins() >> 2;
  if (ngroups == 0) return hipSuccess;
  const int64_t threads = ngroups * 8;
  if (threads >= (1LL << 32)) return hipErrorInvalidValue;  // grid x block < 2^32 work-items
  const uint32_t sent_base = (uint32_t)(((g.chunk + 3) >> 2) << 2);
  if (sent_base + 1024u > 0xFFFFu) return hipErrorInvalidValue;
  hipLaunchKernelGGL(slot_pack_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                     ngroups, off, ent, sent_base, slots);
  return hipGetLastError();
}

// ------------------------------------------------------------------ pair (drop-two) table
__device__ __forceinline__ void pair_decode(const PairGeom &pg, int64_t g, int &p, int &q,
                                            int &c, uint32_t &key) {
  key = (uint32_t)(g % pg.nkeys2);
  const int64_t pc = g / pg.nkeys2;  // pair * nchunks + chunk
  c = (int)(pc % pg.nchunks);
  const int pi = (int)(pc / pg.nchunks);
  p = pg.pq[pi] & 0xFF;
  q = pg.pq[pi] >> 8;
}

__device__ __forceinline__ uint32_t pair_lines(uint32_t n) {
  return n == 0 ? 0u : (n > 255u ? 1u : (16u + 2u * n + 127u) / 128u);
}

// one thread per 8 groups (one nibble word of a summary record); 4 threads per record
__global__ __launch_bounds__(256) void pair_count_kernel(PairGeom pg,
                                                         const uint32_t *__restrict__ xoff,
                                                         uint32_t *__restrict__ summary,
                                                         uint32_t *__restrict__ rtot) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nrec = pg.nrec();
  const bool live = t < nrec * 4;
  uint32_t word = 0, tot = 0;
  if (live) {
    const int64_t g0 = (t >> 2) * 32 + (t & 3) * 8;
    for (int r = 0; r < 8; ++r) {
      const int64_t g = g0 + r;
      if (g >= pg.ngroups()) break;
      int p, q, c;
      uint32_t key;
      pair_decode(pg, g, p, q, c, key);
      const uint32_t *xo = xoff + (size_t)c * ((size_t)pg.nkeys2 << 4);
      uint32_t n = 0;
      for (uint32_t b = 0; b < 16; ++b) {
        const uint32_t z = pair_insert(key, pg.k, p, q, b >> 2, b & 3u);
        n += xo[z + 1] - xo[z];
      }
      const uint32_t nl = pair_lines(n);
      word |= nl << (4 * r);
      tot += nl;
    }
    summary[(t >> 2) * 8 + 1 + (t & 3)] = word;
  }
  // record total over its 4 threads (adjacent lanes)
  tot += __shfl_xor(tot, 1, 64);
  tot += __shfl_xor(tot, 2, 64);
  if (live && (t & 3) == 0) rtot[t >> 2] = tot;
}

// 16 lanes per group (lane b = sub-bin (z_p, z_q) = (b >> 2, b & 3)), 16 groups per block:
// the group's lines are assembled in LDS (header bytes, then every bin's entries copied
// from the exact index) and written out with 16-byte stores.
constexpr int PAIR_PACK_GROUPS = 16;
constexpr int PAIR_MAX_LINES = 5;  // n <= 255: (16 + 510) / 128 -> 5 lines
__global__ __launch_bounds__(256) void pair_pack_kernel(PairGeom pg,
                                                        const uint32_t *__restrict__ xoff,
                                                        const uint16_t *__restrict__ xent,
                                                        const uint32_t *__restrict__ rbase,
                                                        uint32_t *__restrict__ summary,
                                                        uint4 *__restrict__ lines) {
  __shared__ __align__(16) uint32_t img[PAIR_PACK_GROUPS][PAIR_MAX_LINES * 32];
  const int lg = threadIdx.x >> 4, b = threadIdx.x & 15;
  const int64_t g = (int64_t)blockIdx.x * PAIR_PACK_GROUPS + lg;
  const bool live = g < pg.ngroups();
  // record base -> summary w0 (first lane of each record's first group)
  if (live && (g & 31) == 0 && b == 0) summary[(g >> 5) * 8] = rbase[g >> 5];
  // header words 0; every other halfword h a dummy column acc_words + (h & 63) (64 LDS words
  // past the Gram kernel's accumulator, one per lane: conflict-free no-op adds)
  const uint32_t dcol = (uint32_t)(((pg.chunk + 3) >> 2) << 2);
  for (int w = b; w < PAIR_MAX_LINES * 32; w += 16)
    img[lg][w] = w < 4 ? 0u : (dcol + ((2u * w) & 63u)) | ((dcol + ((2u * w + 1u) & 63u)) << 16);
  uint32_t s0 = 0, cnt = 0, key = 0;
  int p = 0, q = 1, c = 0;
  if (live) {
    pair_decode(pg, g, p, q, c, key);
    const uint32_t z = pair_insert(key, pg.k, p, q, (uint32_t)b >> 2, (uint32_t)b & 3u);
    const uint32_t *xo = xoff + (size_t)c * ((size_t)pg.nkeys2 << 4);
    s0 = xo[z];
    cnt = xo[z + 1] - s0;
  }
  // inclusive scan of the 16 bin counts
  uint32_t end = cnt;
#pragma unroll
  for (int d = 1; d < 16; d <<= 1) {
    const uint32_t v = __shfl_up(end, d, 16);
    if (b >= d) end += v;
  }
  const uint32_t n = __shfl(end, 15, 16);
  // base line of this group: record base + line counts of the record's earlier groups
  uint32_t base = 0;
  if (live) {
    const int64_t rec = g >> 5;
    const int r = (int)(g & 31);
    base = rbase[rec];
    for (int j = 0; j < r; ++j) base += (summary[rec * 8 + 1 + (j >> 3)] >> (4 * (j & 7))) & 15u;
  }
  __syncthreads();
  const uint32_t nl = pair_lines(n);
  uint8_t *im = (uint8_t *)img[lg];
  if (live && n > 0) {
    if (n > 255u) {  // wide marker: byte 14 = 0xFF, byte 15 = 0
      if (b == 14) im[14] = 0xFF;
    } else {
      im[b] = (uint8_t)end;
      uint16_t *dst = (uint16_t *)(im + 16) + (end - cnt);
      for (uint32_t e = 0; e < cnt; ++e) dst[e] = xent[s0 + e];
    }
  }
  __syncthreads();
  if (live)
    for (uint32_t w = b; w < nl * 8; w += 16)
      lines[(size_t)base * 8 + w] = ((const uint4 *)img[lg])[w];
}

hipError_t launch_pair_count(const PairGeom &pg, const uint32_t *xoff, uint32_t *summary,
                             uint32_t *rtot, hipStream_t s) {
  const int64_t threads = pg.nrec() * 4;
  if (threads == 0) return hipSuccess;
  if (threads >= (1LL << 32)) return hipErrorInvalidValue;  // grid x block < 2^32 work-items
  hipLaunchKernelGGL(pair_count_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                     pg, xoff, summary, rtot);
  return hipGetLastError();
}

hipError_t launch_pair_pack(const PairGeom &pg, const uint32_t *xoff, const uint16_t *xent,
                            const uint32_t *rbase, uint32_t *summary, uint4 *lines,
                            hipStream_t s) {
  const int64_t blocks = (pg.ngroups() + PAIR_PACK_GROUPS - 1) / PAIR_PACK_GROUPS;
  if (blocks == 0) return hipSuccess;
  if (blocks * 256 >= (1LL << 32)) return hipErrorInvalidValue;  // < 2^32 work-items
  if ((((int64_t)pg.chunk + 3) >> 2 << 2) + 64 > 65536) return hipErrorInvalidValue;  // dummies
  hipLaunchKernelGGL(pair_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, pg, xoff, xent,
                     rbase, summary, lines);
  return hipGetLastError();
}

// plain k-mer extraction (Hamming formulation)
__global__ __launch_bounds__(256) void extract_kernel(IndexGeom g, Packed pk,
                                                      uint32_t *__restrict__ kmers) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= g.n * g.pmax) return;
  const int64_t j = t / g.pmax;
  const int a = (int)(t - j * g.pmax);
  kmers[t] = pk_window(pk.w + j * pk.ldp, pk.cw, a, g.k);
}

// ------------------------------------------------------------------ 2-bit packing
// one thread per (sequence, 32-symbol block): 2 code words + 1 mask word of the record
__global__ __launch_bounds__(256) void pack_kernel(const uint8_t *__restrict__ codes,
                                                   const int32_t *__restrict__ lens, int64_t n,
                                                   int64_t ldc, int cw, int mw, int nb,
                                                   uint32_t *__restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * nb) return;
  const int64_t j = t / nb;
  const int b = (int)(t - j * nb);
  uint32_t c0, c1, m;
  pack_piece(codes, lens, ldc, j, b, c0, c1, m);
  uint32_t *rec = out + j * (int64_t)(cw + mw);
  if (2 * b < cw) rec[2 * b] = c0;
  if (2 * b + 1 < cw) rec[2 * b + 1] = c1;
  if (b < mw) rec[cw + b] = m;
}

hipError_t launch_pack(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc,
                       int window, uint32_t *packed, hipStream_t s) {
  (void)window;
  if (n == 0) return hipSuccess;
  const int cw = packed_cw(ldc), mw = packed_mw(ldc);
  const int nb = max((cw + 1) / 2, mw);
  const int64_t threads = n * nb;
  hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, codes,
                     lens, n, ldc, cw, mw, nb, packed);
  return hipGetLastError();
}

// ------------------------------------------------------------------ scan (bucket counts)
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t &excl, uint32_t *tmp) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t inc = wave_incl_scan(v);
  if (lane == 63) tmp[wave] = inc;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < nw; ++w) {
    const uint32_t s = tmp[w];
    if (w < wave) base += s;
    total += s;
  }
  __syncthreads();
  excl = base + inc - v;
  return total;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_tiles_kernel(const uint32_t *__restrict__ in,
                                                                  int64_t nb,
                                                                  uint32_t *__restrict__ partials) {
  __shared__ uint32_t tmp[SCAN_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q)
    if (base + q < nb) s += in[base + q];
  uint32_t excl;
  const uint32_t total = block_excl_scan(s, excl, tmp);
  if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void scan_partials_kernel(uint32_t *__restrict__ partials,
                                                             int64_t np) {
  __shared__ uint32_t tmp[16];
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < np; b0 += blockDim.x) {
    const int64_t idx = b0 + threadIdx.x;
    const uint32_t v = idx < np ? partials[idx] : 0u;
    uint32_t excl;
    const uint32_t total = block_excl_scan(v, excl, tmp);
    if (idx < np) partials[idx] = carry + excl;
    carry += total;
  }
  if (threadIdx.x == 0) partials[np] = carry;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_finalize_kernel(
    const uint32_t *__restrict__ in, int64_t nb, const uint32_t *__restrict__ partials,
    uint32_t *__restrict__ off, uint32_t *__restrict__ cursor) {
  __shared__ uint32_t tmp[SCAN_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q) {
    v[q] = (base + q < nb) ? in[base + q] : 0u;
    s += v[q];
  }
  uint32_t excl;
  block_excl_scan(s, excl, tmp);
  uint32_t run = partials[blockIdx.x] + excl;
#pragma unroll
  for (int q = 0; q < SCAN_ITEMS; ++q) {
    if (base + q < nb) {
      off[base + q] = run;
      cursor[base + q] = run;
    }
    run += v[q];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) off[nb] = partials[gridDim.x];
}

size_t scan_partials_words(int64_t nb) { return (size_t)((nb + SCAN_TILE - 1) / SCAN_TILE) + 1; }

hipError_t launch_scan(const uint32_t *hist, uint32_t *off, uint32_t *cursor, int64_t nb,
                       uint32_t *partials, hipStream_t s) {
  const int64_t tiles = (nb + SCAN_TILE - 1) / SCAN_TILE;
  if (tiles == 0) return hipMemsetAsync(off, 0, sizeof(uint32_t), s);
  hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, s, hist, nb,
                     partials);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(1024), 0, s, partials, tiles);
  hipLaunchKernelGGL(scan_finalize_kernel, dim3((unsigned)tiles), dim3(SCAN_THREADS), 0, s, hist,
                     nb, partials, off, cursor);
  return hipGetLastError();
}

// ------------------------------------------------------------------ launchers
static size_t part_lds(const IndexGeom &g, const Packed &pk, int arrays) {
  return sizeof(uint32_t) * ((size_t)g.nbuckets() * arrays + (size_t)g.seqs_per_block * pk.ldp) + 16;
}

size_t index_gather_lds(const IndexGeom &g, int64_t nblk) {
  return sizeof(uint32_t) * (((size_t)1 << g.fine_bits) + 2 * (size_t)nblk);
}

hipError_t launch_index_local(const IndexGeom &g, const Packed &pk, const uint8_t *codes,
                              const int32_t *lens, int64_t ldc, int nblk, uint32_t cap,
                              uint32_t *hcnt, uint32_t *hstart, uint32_t *tmp, hipStream_t s) {
  if (g.n == 0 || nblk == 0) return hipSuccess;
  hipLaunchKernelGGL(part_local_kernel, dim3((unsigned)nblk), dim3(g.part_threads),
                     part_lds(g, pk, 1), s, g, pk, codes, lens, ldc, nblk, cap, hcnt, hstart, tmp);
  return hipGetLastError();
}

hipError_t launch_index_gather(const IndexGeom &g, int nblk, uint32_t cap, const uint32_t *hcnt,
                               const uint32_t *hstart, const uint32_t *tmp, uint32_t *off,
                               uint16_t *ent, hipStream_t s) {
  const int64_t nbk = g.nbuckets();
  const size_t lds = index_gather_lds(g, nblk);
  if (lds > 160 * 1024 - 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(part_gather_kernel, dim3((unsigned)nbk), dim3(FINE_THREADS), lds, s, g, nblk,
                     cap, hcnt, hstart, tmp, off, ent);
  return hipGetLastError();
}

hipError_t launch_extract(const IndexGeom &g, const Packed &pk, uint32_t *kmers, hipStream_t s) {
  const int64_t items = g.n * g.pmax;
  if (items == 0) return hipSuccess;
  const int64_t blocks = (items + 255) / 256;
  hipLaunchKernelGGL(extract_kernel, dim3((unsigned)blocks), dim3(256), 0, s, g, pk, kmers);
  return hipGetLastError();
}

}  // namespace kmg
