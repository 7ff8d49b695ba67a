// kmg_internal.h — shared declarations of the kmgram HIP library (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "kmgram.h"

#define KMG_INVALID 0xFFFFFFFFu
#define KMG_ENTRY_LETTER_SHIFT 30
#define KMG_ENTRY_SEQ_MASK 0x3FFFFFFFu
// slot layout of the rotated mismatch index: 128-byte line = 8-byte header + 60 entries
#define KMG_SLOT_BYTES 128
#define KMG_SLOT_INLINE 60
// internal output dtype (not in the ABI): raw counts as uint16, the round slabs of the
// multi-GPU upper-triangle assembly (kmg_gram_blocks), widened by tri_unpack16_kernel
#define KMG_U16 16
// ... and raw counts as uint8 with the diagonal left out (0 in the slab; the unpack takes
// K_ii from the diagonal every rank computes itself): the spectrum's off-diagonal counts
// are mostly < 256 where its diagonal (up to P^2) is not
#define KMG_U8 8

namespace kmg {

// ---------------------------------------------------------------- index build
// Posting index of k-mer occurrences, the MI355X replacement of the dense 4^k
// feature vectors phi of get_phi_u / get_phi_km (kernels.py:12-25, 161-175).
//   bins  = copies x nchunks x nkeys, laid out [copy][chunk][key]
//   off   = bin start offsets (nbins + 1 entries)
//   ent   = uint16 per occurrence: column inside its chunk (SP: 16 bits; MM: 14 bits)
//           | letter at the dropped position << 14 (mismatch index only)
struct IndexGeom {
  int k;            // k-mer length
  int window;       // 0: per-sequence length (spectrum); >0: fixed window (mismatch, 101)
  int pmax;         // k-mer slots per sequence
  int copies;       // 1 = exact k-mer keys; k = one copy per dropped position (mismatch)
  int chunk;        // columns per chunk
  int nchunks;
  uint32_t nkeys;   // keys per (copy, chunk): 4^k or 4^(k-1)
  int64_t n;
  int fine_bits;    // bins per coarse bucket = 2^fine_bits (partition pass)
  int rot;             // mismatch layout: copy p keyed by the k-mer with letter p rotated
                       // to the lowest digit (4 adjacent letter sub-lists); entry = column
  int seqs_per_block;  // partition pass: sequences per block
  int part_threads;    // partition pass: threads per block
  __host__ __device__ int64_t nbins() const { return (int64_t)copies * nchunks * (int64_t)nkeys; }
  __host__ __device__ int64_t nbuckets() const {
    return (nbins() + ((int64_t)1 << fine_bits) - 1) >> fine_bits;
  }
};

// 2-bit packed sequences (kmg_pack_kernel, kmg_index.hip).  Record of sequence j =
// w + j * ldp words:
//   words [0, cw)        symbols, 16 per word, big-endian: symbol t at bits 30 - 2 (t & 15)
//                        of word t >> 4 (so a k-mer read off the words has its first
//                        letter most significant, the base-4 order of kernels.py:37,206)
//   words [cw, cw + mw)  invalid mask: bit t & 31 of word cw + (t >> 5) is set when symbol
//                        t is not A/C/G/T (the reference drops such k-mers, kernels.py:23-24)
//                        or t >= len (padding), so a window is valid iff its k mask bits are 0
// cw = ldc / 16 + 2 and mw = ldc / 32 + 2 leave one zero word past the last symbol, so a
// window read never leaves its record.
struct Packed {
  const uint32_t *w;
  int64_t ldp;  // words per record = cw + mw
  int cw;       // code words
};
inline int packed_cw(int64_t ldc) { return (int)(ldc / 16) + 2; }
inline int packed_mw(int64_t ldc) { return (int)(ldc / 32) + 2; }

// k-mer code (k <= 16) of window a of a packed record; KMG_INVALID if it holds a masked symbol
__device__ __forceinline__ uint32_t pk_window(const uint32_t *rec, int cw, int a, int k) {
  const int i = a >> 4, sh = 2 * (a & 15);
  const uint64_t v = ((uint64_t)rec[i] << 32) | rec[i + 1];
  const uint32_t code = (uint32_t)((v << sh) >> (64 - 2 * k));
  const int j = a >> 5;
  const uint64_t m = ((((uint64_t)rec[cw + j + 1]) << 32) | rec[cw + j]) >> (a & 31);
  return (m & ((1ull << k) - 1ull)) ? KMG_INVALID : code;
}

// codes uint8 [n][ldc] (values 0..3 = ACGT, >= 4 other) + lens -> packed records
hipError_t launch_pack(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc,
                       int window, uint32_t *packed, hipStream_t s);

// exclusive scan of hist[0..nb) into off[0..nb] (off[nb] = total); cursor = off[0..nb)
hipError_t launch_scan(const uint32_t *hist, uint32_t *off, uint32_t *cursor, int64_t nb,
                       uint32_t *partials, hipStream_t s);
size_t scan_partials_words(int64_t nb);
hipError_t launch_extract(const IndexGeom &g, const Packed &pk, uint32_t *kmers, hipStream_t s);
// index build (no device-scope atomics): per-block local sort, then per-bucket gather.
// hcnt/hstart: nbuckets x nblk (bucket-major); tmp: nblk x cap items.  codes != nullptr:
// the local pass also packs the sequences into pk (launch_pack fused into the first pass).
size_t index_gather_lds(const IndexGeom &g, int64_t nblk);
hipError_t launch_index_local(const IndexGeom &g, const Packed &pk, const uint8_t *codes,
                              const int32_t *lens, int64_t ldc, int nblk, uint32_t cap,
                              uint32_t *hcnt, uint32_t *hstart, uint32_t *tmp, hipStream_t s);
hipError_t launch_index_gather(const IndexGeom &g, int nblk, uint32_t cap, const uint32_t *hcnt,
                               const uint32_t *hstart, const uint32_t *tmp, uint32_t *off,
                               uint16_t *ent, hipStream_t s);
// rotated mismatch index (rot = 1): one KMG_SLOT_BYTES line per 4-bin group
hipError_t launch_slot_pack(const IndexGeom &g, const uint32_t *off, const uint16_t *ent,
                            uint4 *slots, hipStream_t s);

// ---------------------------------------------------------------- pair (drop-two) table
// Mismatch (k, 1) through the drop-two-letters index: for every pair of positions
// p < q (npairs = k(k-1)/2, enumerated (0,1), (0,2), ..., (k-2,k-1)) and every k-mer z,
// key_pq(z) = z with letters p and q removed (k-2 letters).  Group (pair, chunk, key) holds
// every occurrence z with that key, sorted into 16 sub-bins by (z_p, z_q).
// Storage: each group is nl whole 128-byte lines at line index base(g) of `lines`:
//   16-byte header = bin ends e[0..15] as bytes (e[15] = n), then n uint16 columns;
//   nl = ceil((16 + 2n) / 128); n = 0 -> nl = 0 (no lines);
//   n > 255 -> "wide": one marker line (byte 14 = 0xFF, byte 15 = 0) and the entries are
//   read from the exact k-mer index (xoff / xent) in a slow path.
// Summary (L2-resident, 1 byte per group): per 32 groups a 32-byte record
//   w0 = base line of the record's first group, w1..w4 = nl of the 32 groups, 4 bits each.
#define KMG_PAIRS_MAX 66
struct PairGeom {
  int k;
  int npairs;
  int nchunks;
  int chunk;
  uint32_t nkeys2;                 // 4^(k-2)
  uint16_t pq[KMG_PAIRS_MAX];      // p | q << 8
  __host__ __device__ int64_t ngroups() const { return (int64_t)npairs * nchunks * nkeys2; }
  __host__ __device__ int64_t nrec() const { return (ngroups() + 31) / 32; }
};
// z with letters zp at p and zq at q inserted into the (k-2)-letter key (p < q)
__host__ __device__ __forceinline__ uint32_t pair_insert(uint32_t key, int k, int p, int q,
                                                         uint32_t zp, uint32_t zq) {
  const int lo = 2 * (k - 1 - q), mid = 2 * (q - p - 1);
  const uint32_t bottom = key & ((1u << lo) - 1u);
  const uint32_t middle = (key >> lo) & ((1u << mid) - 1u);
  const uint32_t top = (uint32_t)((uint64_t)key >> (lo + mid));
  return (((((top << 2) | zp) << mid | middle) << 2 | zq) << lo) | bottom;
}
// (k-2)-letter key of k-mer u for the pair p < q
__host__ __device__ __forceinline__ uint32_t pair_key(uint32_t u, int k, int p, int q) {
  const int lo = 2 * (k - 1 - q), mid = 2 * (q - p - 1);
  const uint32_t bottom = u & ((1u << lo) - 1u);
  const uint32_t middle = (u >> (lo + 2)) & ((1u << mid) - 1u);
  const uint32_t top = (uint32_t)((uint64_t)u >> (2 * (k - p)));
  return (((top << mid) | middle) << lo) | bottom;
}
// from the exact index (xoff over [chunk][4^k]): per-group line counts into summary
// w1..w4 and per-record line totals rtot[nrec]
hipError_t launch_pair_count(const PairGeom &pg, const uint32_t *xoff, uint32_t *summary,
                             uint32_t *rtot, hipStream_t s);
// after the exclusive scan of rtot into rbase: summary w0 = rbase, then the lines
hipError_t launch_pair_pack(const PairGeom &pg, const uint32_t *xoff, const uint16_t *xent,
                            const uint32_t *rbase, uint32_t *summary, uint4 *lines,
                            hipStream_t s);
// upper bound of the line count (no device round trip before allocating): a non-empty
// group holds >= 1 of the npairs * occurrences entries and takes <= 1 + (16 + 2n) / 128 lines
inline int64_t pair_lines_bound(const PairGeom &pg, int64_t occurrences) {
  const int64_t entries = (int64_t)pg.npairs * occurrences;
  const int64_t nonempty = pg.ngroups() < entries ? pg.ngroups() : entries;
  return nonempty + nonempty / 8 + 2 * entries / 128 + 64;
}

// ---------------------------------------------------------------- Gram kernels
struct OutSpec {
  void *out;         // points at row row0
  int64_t ld;        // elements
  int32_t dtype;     // KMG_I32 / KMG_F32 / KMG_F64
  int normalize;     // fused normalize_K epilogue
  const double *diagv;  // raw diagonal (normalize)
  const double *dsq;    // sqrt(raw diagonal) (normalize)
  int64_t col_lo = 0;   // columns < col_lo are not written (upper-triangle multi-GPU
                        // builds; kernels that honour it: spectrum, mismatch slots / pairs)
  int64_t col_seq0 = 0; // sequence of output column 0 (column blocks, kmg_gram_device_cols):
                        // the diagonal and the normalisation's K_jj are taken at col_seq0 + j
  int tri = 0;          // full square K (rows [0, n)): the mismatch posting-list kernels
                        // compute only the column chunks that reach column i of row i
                        // (rowacc_block); the caller mirrors the rest (launch_mirror_chunks)
  uint32_t *ovf = nullptr;  // dtype KMG_U16 / KMG_U8: set to 1 when a count exceeds 65535
                            // / an off-diagonal count exceeds 255 (the stored value is then
                            // clipped and the caller redoes the build with wider slabs)
  // dtype KMG_U8 with an escape list: an off-diagonal count >= 255 is stored as the escape
  // byte 255 and appended as (row, column, count, 0) to esc[*esc_n] (esc_n counts every
  // attempt; past esc_cap the overflow flag is raised instead)
  uint4 *esc = nullptr;
  uint32_t *esc_n = nullptr;
  uint32_t esc_cap = 0;
};

// uint8 round-slab byte of the off-diagonal count x at (row i, column col)
__device__ __forceinline__ uint32_t u8_slab_entry(const OutSpec &o, int64_t i, int64_t col,
                                                  uint32_t x, bool &big) {
  if (x < 255u) return x;
  if (o.esc) {
    const uint32_t k = atomicAdd(o.esc_n, 1u);
    if (k < o.esc_cap) {
      o.esc[k] = make_uint4((uint32_t)i, (uint32_t)col, x, 0u);
      return 255u;
    }
  }
  big = true;
  return 255u;
}

// multi-GPU upper-triangle assembly (kmg_gram_blocks): round slab S (R rows x w = n - c0
// columns, row-major: rows c0 .. c0 + R of K restricted to columns >= c0) -> K's rows
// c0 + y at columns >= c0, and the lower-triangle mirror K[c0 + j][c0 + y] = S[y][j] for
// j >= R; one LDS-tiled pass over S (esz = 4 or 8 bytes)
hipError_t launch_tri_unpack(const void *S, int64_t w, int64_t R, int64_t c0, int64_t n, void *K,
                             int64_t ld, int esz, hipStream_t s);
// the same from a uint16 slab of raw counts into K of dtype dt (int32 / float32 / float64),
// normalize_K applied on the way when `normalize` and diagv[0] != 1 (the fused epilogue's
// formula, bit for bit)
hipError_t launch_mirror_chunks(void *K, int64_t ld, int64_t n, int chunk, int esz,
                                hipStream_t s);
// column-block assembly (kmg_gram_blocks gather 5 / 6): K[j][i] = M[i][j] for the column block
// M (rows x w, row stride ldm) into w rows of K (row stride ldk), 64 x 64 LDS tiles, 16 bytes
// a lane both ways (esz = 4 or 8 bytes)
hipError_t launch_transpose(const void *M, int64_t ldm, int64_t rows, int64_t w, void *K,
                            int64_t ldk, int esz, hipStream_t s);
hipError_t launch_tri_unpack16(const uint16_t *S, int64_t w, int64_t R, int64_t c0, int64_t n,
                               void *K, int64_t ld, int dt, int normalize, const double *diagv,
                               const double *dsq, hipStream_t s);
// uint8 slab (diagonal left out): K_ii = diagv[i] (raw), normalised 1
hipError_t launch_tri_unpack8(const uint8_t *S, int64_t w, int64_t R, int64_t c0, int64_t n,
                              void *K, int64_t ld, int dt, int normalize, const double *diagv,
                              const double *dsq, hipStream_t s);
// escapes of uint8 slabs: nsets lists of stride entries, list s holding counts[s] entries
// (row, column, count, 0); writes K[row][col] and K[col][row] as the unpack would have
hipError_t launch_tri_patch8(const uint4 *esc, const uint32_t *counts, int nsets, int64_t stride,
                             int64_t max_count, void *K, int64_t ld, int dt, int normalize,
                             const double *diagv, const double *dsq, hipStream_t s);
hipError_t launch_gram_spectrum(const IndexGeom &g, const Packed &pk, const uint32_t *off,
                                const uint16_t *ent, int64_t row0, int64_t row1, const OutSpec &o,
                                hipStream_t s, int store = 0, int order = 0, int rows_per = 0);
// mismatch (k,1), 8 <= k <= 12, on the slot layout (one line per list)
hipError_t launch_gram_mismatch1_slots(const IndexGeom &g, const Packed &pk, const uint4 *slots,
                                       const uint32_t *off, const uint16_t *ent, int64_t row0,
                                       int64_t row1, int w0, int w1, int w2, const OutSpec &o,
                                       hipStream_t s);
// mismatch (k,1), 3 <= k <= 12, on the pair (drop-two) table; xoff / xent = exact index
hipError_t launch_gram_mismatch1_pairs(const PairGeom &pg, const IndexGeom &g, const Packed &pk,
                                       const uint32_t *summary, const uint4 *lines,
                                       int64_t nlines, const uint32_t *xoff, const uint16_t *xent,
                                       int64_t row0, int64_t row1, int w0, int w1, int w2,
                                       const OutSpec &o, hipStream_t s);
// mismatch (k, 1), 4 <= k <= 12, through neighbourhood lists (kmg_nbhd.hip): from the exact
// index (xoff / xent over [chunk][4^k]) every (chunk, k-mer)'s list of the column windows at
// Hamming distance 0 | 1 | 2 (3 segments; segment 2 packed where the sorted fill runs);
// hist / nboff / cursor nbins + 1 words, nbseg / nbuse nbins, table
// nb_list_entries_bound(...) uint16
int64_t nb_list_entries_bound(int k, int64_t occurrences, int64_t nbins);
size_t nb_gram_lds(const IndexGeom &g, const Packed &pk);
// entries of segment 2 the sorted fill's per-wave LDS buffer holds at this chunk (0: the
// lists stay 16-bit: k too sparse to pack, or the buffer below 1.25x the mean segment), and
// the largest chunk it runs at (0: none)
int nb_sorted_cap(int k, int pmax, int chunk);
int nb_sorted_max_chunk(int k, int pmax);
hipError_t launch_nb_count(const IndexGeom &g, const uint32_t *xoff, uint32_t *hist,
                           uint32_t *nboff, uint32_t *cursor, uint2 *nbseg, uint32_t *partials,
                           hipStream_t s);
// form: 0 auto (sorted where nb_sorted_cap > 0, else 16-bit lists), 1 sorted, 2 grouped,
// 3 pieces, 4 staged, 5 auto 16-bit (staged where a typical list fits its per-wave LDS
// buffer, else the piece-assembled fill past 8.5 occurrences a k-mer and chunk, else grouped)
hipError_t launch_nb_fill(const IndexGeom &g, const uint32_t *xoff, const uint16_t *xent,
                          const uint32_t *nboff, const uint2 *nbseg, uint2 *nbuse,
                          uint16_t *table, hipStream_t s, int form = 0, int fill_threads = 512);
hipError_t launch_gram_mismatch1_nb(const IndexGeom &g, const Packed &pk, const uint32_t *nboff,
                                    const uint2 *nbseg, const uint2 *nbuse, const uint4 *table,
                                    int64_t row0, int64_t row1, int w0, int w1, int w2,
                                    const OutSpec &o, hipStream_t s, int threads, int unroll = 8);
// KMG_CHECK: validate the filled lists' metadata (nb_check_kernel); flag[0] bit 0 set on a
// violation, flag[1] = min offending list (the caller zeroes flag[0] and sets flag[1] to ~0)
hipError_t launch_nb_check(int64_t nbins, const uint32_t *nboff, const uint2 *nbseg,
                           const uint2 *nbuse, uint64_t table_pieces, uint32_t *flag,
                           hipStream_t s);
// all-pairs Hamming formulation, any (k <= 16, m): K = sum_{a,b} w[ham(x_a, y_b)]
hipError_t launch_gram_hamming(const IndexGeom &g, const uint32_t *kmers, int64_t row0,
                               int64_t row1, const int64_t *wtab, const OutSpec &o, hipStream_t s);
// max_dist: largest Hamming distance with a non-zero weight (min(2m, k) for mismatch)
hipError_t launch_diag_hamming(const IndexGeom &g, const Packed &pk, const int64_t *wtab,
                               int max_dist, double *diagv, double *dsq, hipStream_t s);

struct SeqSpec {
  const uint8_t *codes;
  const int32_t *lens;
  int64_t n, ldc;
  int maxlen;
};

// kmg_generic.hip: per-pair fallbacks (spectrum / mismatch k > 16, WD / WDS past the
// specialised kernels' shift and length limits)
hipError_t launch_gram_sp_generic(const SeqSpec &q, int64_t row0, int64_t row1, int k, int mirror,
                                  const OutSpec &o, hipStream_t s);
hipError_t launch_sp_generic_diag(const SeqSpec &q, int k, double *diagv, double *dsq,
                                  hipStream_t s);
hipError_t launch_mm_generic_diag(const SeqSpec &q, int W, int k, const int64_t *w, int maxd,
                                  double *diagv, double *dsq, hipStream_t s);
hipError_t launch_gram_mm_generic(const SeqSpec &q, int64_t row0, int64_t row1, int W, int k,
                                  const int64_t *w, int maxd, int mirror, const OutSpec &o,
                                  hipStream_t s);
hipError_t launch_gram_wds_generic(const SeqSpec &q, int64_t row0, int64_t row1, int d, int S,
                                   int span, const double *coef_a, const double *coef_b,
                                   int wd_diag, int mirror, const OutSpec &o, hipStream_t s);

hipError_t launch_gram_wd(const SeqSpec &q, int64_t row0, int64_t row1, int d, int span,
                          const double *beta, const OutSpec &o, hipStream_t s);
hipError_t launch_gram_wd_packed(const SeqSpec &q, const Packed &pk, int64_t row0, int64_t row1,
                                 int d, int span, const double *beta, const OutSpec &o,
                                 hipStream_t s);
hipError_t launch_gram_wds(const SeqSpec &q, int64_t row0, int64_t row1, int d, int S, int span,
                           const double *beta, const double *delta, const OutSpec &o,
                           hipStream_t s);
// lpp: lanes a pair of the grouped sweep (0 auto; 16 / 32 force the wider groups);
// bmode: B_kk(x, y) of the recursion (kernels.py:322-342) instead of K_kk (grouped sweep only)
hipError_t launch_gram_ss(const SeqSpec &q, int64_t row0, int64_t row1, int kk, double lam,
                          double lam2, int mirror, const OutSpec &o, hipStream_t s, int lpp = 0,
                          int bmode = 0);
// LA kernel, intended semantics (KMG_LA_INTENDED): five-array affine-gap DP per pair
hipError_t launch_gram_la(const SeqSpec &q, int64_t row0, int64_t row1, double e, double d,
                          double beta, int smith, int mirror, const OutSpec &o, hipStream_t s,
                          int lpp = 0);
// stats[0] = max code over every row's first len symbols, stats[1] = min len (preset to 0 /
// UINT_MAX by the caller)
hipError_t launch_row_stats(const SeqSpec &q, uint32_t *stats, hipStream_t s);
hipError_t launch_gram_gappy1(const SeqSpec &q, int64_t row0, int64_t row1, int window,
                              const OutSpec &o, double *diagv, double *dsq, hipStream_t s);
hipError_t launch_fill(const OutSpec &o, int64_t rows, int64_t cols, double value, hipStream_t s);

// per-sequence feature vectors over caller-chosen k-mer columns (kmg_features.hip):
// out[r][j] for sequences row0 + r, r < rows; window 0 = every window of the row
#define KMG_FEAT_MAXW 4096
hipError_t launch_features_sym(const uint8_t *codes, const int32_t *lens, int64_t ldc, int64_t row0,
                               int64_t rows, int k, int m, int window, int bcast, const uint4 *cols,
                               int64_t ncols, double *out, int64_t ld, hipStream_t s);
hipError_t launch_features(const uint8_t *codes, const int32_t *lens, int64_t ldc, int64_t row0,
                           int64_t rows, int k, int m, int window, int binary,
                           const uint32_t *cols, int64_t ncols, double *out, int64_t ld,
                           hipStream_t s);

// gappy (k, g), intended semantics: binary (k-g)-mer presence features (kmg_dense.hip)
hipError_t launch_gappy_features(const uint8_t *codes, int64_t ldc, int64_t n, int k, int kk,
                                 int window, int dp, const uint32_t *combos, int ncomb, int8_t *F,
                                 double *diagv, double *dsq, hipStream_t s);
// dense count-vector formulation (kmg_dense.hip): int8 F [rows >= n + 128][dp], K = F F^T
// KMG_ALGO=3: int8 count rows widened to fp32 for rocblas_sgemm; the fp32 K to the output
hipError_t launch_i8_to_f32(const int8_t *F, int64_t elems, float *G, hipStream_t s);
hipError_t launch_f32_gram_out(const float *K32, int64_t n, int64_t row0, int64_t row1,
                               const OutSpec &o, hipStream_t s);
hipError_t launch_dense_features(const uint8_t *codes, const int32_t *lens, int64_t ldc, int64_t n,
                                 int k, int window, int dp, const uint32_t *masks, int nmask,
                                 int8_t *F, double *diagv, double *dsq, hipStream_t s);
hipError_t launch_gram_dense(const int8_t *F, int dp, int64_t n, int64_t row0, int64_t row1,
                             const uint32_t *order, const OutSpec &o, hipStream_t s, int bk = 64,
                             bool half = false);

// kernel-combination consumers (kmg_combine.hip): K = device array of p matrix pointers
#define KMG_COMBINE_PMAX 12
hipError_t launch_combine(const double *const *K, const double *u, int p, int degree, int64_t n,
                          int64_t ld, double *out, int64_t ld_out, hipStream_t s);
// part: n x p scratch; grad: p
hipError_t launch_nlck_grad(const double *const *K, const double *u, int p, int degree,
                            const double *alpha, int64_t n, int64_t ld, double *part,
                            double *grad, hipStream_t s);
// rmean/cmean: p x n, tmean: p, part: n x (p + p(p+1)/2), out: p + p(p+1)/2
hipError_t launch_alignf(const double *const *K, int p, const double *y, int64_t n, int64_t ld,
                         double *rmean, double *cmean, double *tmean, double *part, double *out,
                         hipStream_t s);

// dense learners on K (kmg_solve.hip): B = diag(s) K diag(s) + shift I (s may be NULL)
// (dvec may be NULL; else B[i][i] += shift + dvec[i])
hipError_t launch_shift_scale(const double *K, int64_t ldk, const double *s, double shift,
                              const double *dvec, int64_t n, double *B, int64_t ldb,
                              hipStream_t st);
// blocked Cholesky (kmg_solve.hip): one diagonal block (nb <= 128) factorised in place
// (column-major lower) plus its inverse Y and Y^T (ld 128); a non-positive pivot sets *info
// (1-based column j0 + j + 1); returns at once if *info != 0
hipError_t launch_chol_diag(double *A, int64_t lda, int nb, int j0, int *info, double *Y, double *YT,
                            hipStream_t st);
// dynamic LDS of one launch_chol_diag workgroup (its inverse: ~133 KB, gfx950's 160 KB LDS)
size_t chol_diag_lds_bytes();
// one block step of the substitution sweeps (forward: M = Y, back: M = Y^T)
hipError_t launch_tri_sweep(const double *L, int64_t n, const double *M, int64_t j0, int jb, int back,
                            double *src, double *dst, hipStream_t st);
// *flag |= 1 when K is not exactly symmetric (flag must be zeroed before)
hipError_t launch_asymmetry(const double *K, int64_t ld, int64_t n, int *flag, hipStream_t st);
// KLR IRLS step: s = sqrt(sig(m) sig(-m)), rhs = s * (m + y / sig(-y m))
hipError_t launch_irls(const double *m, const double *y, int64_t n, double *s, double *rhs,
                       hipStream_t st);
// alpha = s * x, out[0] = ||alpha - prev||^2
hipError_t launch_scale_diff(const double *s, const double *x, const double *prev, int64_t n,
                             double *alpha, double *out, hipStream_t st);

// C-SVM dual QP interior point (kmg_solve.hip): vec = 11 x n doubles, sc >= 8 doubles.
// phase 0 init, 1 v = y o x, 2 residual/D/predictor rhs (sc = mu, ||rd||_inf, obj),
// 3 affine step + corrector rhs, 4 corrector step + update, 5 alpha = y o x
#define KMG_SVM_NVEC 11
#define KMG_SVM_V 8   // vector index of v (GEMV input)
#define KMG_SVM_U 9   // vector index of u (GEMV output)
#define KMG_SVM_RHS 10
hipError_t launch_svm(int phase, const double *y, int64_t n, double C, double *vec, double *sc,
                      double *alpha, hipStream_t st);

// host-matrix helpers (normalize_K / center_K)
hipError_t launch_normalize_dense(double *K, int64_t n, int64_t ld, hipStream_t s);
hipError_t launch_center_dense(const double *K, int64_t ldk, double *out, int64_t ld_out,
                               int64_t n, double *rowmean, double *colmean, double *tot,
                               hipStream_t s);

}  // namespace kmg
