// kmg_api.cpp — C ABI of libkmgram.so (include/kmgram.h): context, device workspace,
// parameter validation, dispatch to the HIP kernels, and the RCCL row all-gather.
//
// Reference entry points replaced (afiliot/Kernel-Methods-For-Genomics kernels.py):
//   select_method 461-505 dispatches to
//   get_spectrum_K 28-47, get_mismatch_K 196-217, get_WD_K 84-101,
//   get_WDShifts_K 138-155, get_string_K 367-382, get_LA_K 273-302, get_gappy_K 436-455,
//   normalize_K 398-415, center_K 387-395.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "kmg_internal.h"

struct kmg_ctx;
static int blas_handle(kmg_ctx *c);  // rocBLAS / rocSOLVER handle on the context stream

using namespace kmg;

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define KMG_HIP(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      return fail(_e == hipErrorOutOfMemory ? KMG_ENOMEM : KMG_EHIP, "%s failed: %s (%s:%d)", \
                  #expr, hipGetErrorString(_e), __FILE__, __LINE__);                           \
  } while (0)

#define KMG_TRY(expr)          \
  do {                         \
    int _r = (expr);           \
    if (_r != KMG_OK) return _r; \
  } while (0)

struct DevBuf {
  void *p = nullptr;
  size_t bytes = 0;
  int ensure(size_t want) {
    if (want <= bytes) return KMG_OK;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      bytes = 0;
    }
    size_t alloc = want < 256 ? 256 : want;
    hipError_t e = hipMalloc(&p, alloc);
    if (e != hipSuccess) {
      p = nullptr;
      return fail(KMG_ENOMEM, "hipMalloc(%zu) failed: %s", alloc, hipGetErrorString(e));
    }
    bytes = alloc;
    return KMG_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  template <typename T>
  T *as() const {
    return (T *)p;
  }
};

// "pack" = 2-bit packing of the input, "slots" = slot layout of the mismatch index,
// "lists" = neighbourhood-list sizes and starts, "nbfill" = the neighbourhood lists
// themselves, "gather" = the RCCL row all-gather (kmg_allgather_rows)
const char *kStageNames[] = {"count",   "scan",     "place", "fine",    "diag",
                             "gram",    "extract",  "pack",  "features", "combine",
                             "solve",   "slots",    "memset", "gather", "unpack",
                             "mirror",  "lists",    "nbfill"};
constexpr int kNumStages = 18;
enum {
  ST_COUNT, ST_SCAN, ST_PLACE, ST_FINE, ST_DIAG, ST_GRAM, ST_EXTRACT, ST_PACK, ST_FEATURES,
  ST_COMBINE, ST_SOLVE, ST_SLOTS, ST_MEMSET, ST_GATHER, ST_UNPACK, ST_MIRROR, ST_LISTS,
  ST_NBFILL
};

// Tuning knobs: read from the environment once per context (kmg_create) and again only on
// kmg_reload_tuning, never per launch.
struct Tuning {
  int sp_chunk = 24576;     // KMG_SP_CHUNK: columns per chunk, spectrum index
  int mm_chunk = 20480;     // KMG_MM_CHUNK: columns per chunk, mismatch index (upper bound)
  int mm_form = 0;          // KMG_MM_FORM: 0 auto, 1 drop-one slot table, 2 drop-two pair table,
                            // 4 neighbourhood lists (kmg_nbhd.hip); (3, round 3's pair lines,
                            // was removed in round 5: measured slower than the lists at k = 9)
  int nb_threads = 0;       // KMG_NB_THREADS: neighbourhood-list Gram workgroup, 512 / 1024
                            // (0 auto: 512 for a column block -- three workgroups a CU over its
                            // narrower chunks: config-5 1/8 share raw 19.0 -> 18.0 ms, float64
                            // 25.3 -> 24.9, N=20000 7000 columns 1.62 -> 1.51; 1024 otherwise,
                            // two a CU at 20000 columns; profiles/r06n_colblock_threads2.jsonl)
  int nb_lds512 = 0;        // KMG_NB_LDS512: KB of LDS a 512-thread NB Gram workgroup may take
                            // when sizing chunks (0 auto: 53, three a CU, for a column block;
                            // 40, four a CU, otherwise)
  int nb_unroll = 0;        // KMG_NB_UNROLL: 16-byte pieces in flight a lane, NB Gram (4 / 8;
                            // 0 auto: 8, or 4 for an upper-block-triangle build or packed
                            // lists -- profiles/r04x2_nb_unroll_ab.jsonl; column block N=200000
                            // x 25000 Gram 23.6 -> 22.3 ms, profiles/r05x_colblock.jsonl)
  int nb_fill = 0;          // KMG_NB_FILL: list fill, 0 auto (sorted + packed segment 2 where a
                            // list is read >= nb_pack_reads times and nb_sorted_cap allows;
                            // else staged 16-bit lists), 1 sorted, 2 grouped lane-per-run,
                            // 3 piece-assembled, 4 staged (launch_nb_fill)
  int nb_fill_threads = 512;  // KMG_NB_FILL_THREADS: staged fill workgroup, 512 (two a CU where
                              // a list fits their buffers) or 1024
  int nb_pack_reads = 16;   // KMG_NB_PACK_READS: reads a list must get for the packed segment 2
                            // (its sort costs ~1 ms more at N=20000, k=9; each read of the
                            // list saves ~0.9 of its 16-bit segment-2 bytes)
  int mm_tri = 1;           // KMG_MM_TRI: full square mismatch K by its upper block triangle
                            // (column chunks at or right of the row's own) + mirror, 0 off
  int esc_cap = 0;          // KMG_ESC_CAP: escape-list entries of uint8 round slabs (0: by size)
  int ss_lpp = 0;           // KMG_SS_LPP: SS grouped sweep, lanes a pair (0 auto, 16, 32)
  int la_lpp = 0;           // KMG_LA_LPP: intended-LA grouped sweep, lanes a pair (0 auto, 16, 32)
  int wd_form = 0;          // KMG_WD_FORM: 0 2-bit packed WD kernel, 1 byte-tile WD kernel
  int algo = 0;             // KMG_ALGO: 0 auto, 1 dense MFMA, 2 index / Hamming, 3 dense
                            // count vectors as an fp32 rocBLAS GEMM (configs[3]'s wording)
  int dense_kmax_sp = 5;    // KMG_DENSE_KMAX_SP: dense formulation for spectrum k <= this
  int dense_kmax_mm = 7;    // KMG_DENSE_KMAX_MM: ... and mismatch k <= this
  int idx_seqs = 0;         // KMG_IDX_SEQS: sequences per partition block (0: auto, build_index)
  int idx_buckets = 0;      // KMG_IDX_BUCKETS: coarse buckets (0: 384 spectrum / 1024 mismatch)
  int idx_threads = 1024;   // KMG_IDX_THREADS
  int poison = 0;           // KMG_POISON: fill the output with 0xA5 first (testing)
  int potrf_upper = 0;      // KMG_POTRF_UPPER: rocSOLVER upper-triangle Cholesky (implies KMG_CHOL=0)
  int chol = 1;             // KMG_CHOL: 1 blocked Cholesky + solves (chol_factor), 0 rocSOLVER potrf/potrs
  int chol_panels = 4;      // KMG_CHOL_PANELS: trailing update as this many GEMM column panels (0:
                            // one dsyrk).  KRR n=9000 19.3-19.5 -> 18.3 ms at 4 (2: 19.0, 3: 18.4,
                            // 6: 18.4, 8: 18.5; profiles/r05bo_chol_panels.json)
  int sp_store = 0;         // KMG_SP_STORE: spectrum K stores, 0 auto, 1 non-temporal, 2 plain
  int sp_order = 1;         // KMG_SP_ORDER: spectrum grid, 0 row-major, 1 chunk-major (N=100000:
                            // Gram 6.66 -> 5.85 ms, interleaved A/B profiles/r02aq_sp_order_ab.jsonl)
  int sp_rows = 0;          // KMG_SP_ROWS: spectrum rows per workgroup, 1, 2 or 4 (full-width
                            // dtypes), 0 auto: 2 for chunks <= 16384 columns (the 12500-column
                            // block: Gram 1.18 -> 0.88 ms; at 20000- and 25000-column chunks
                            // neutral or slower, profiles/r06j_rows*_ab.jsonl, r06k_*), else 1
  int sp_cb_chunk = 32768;  // KMG_SP_CB_CHUNK: spectrum column blocks this wide or narrower
                            // are one column chunk (kmg_gram_device_cols)
  int dense_sb = 0;         // KMG_DENSE_SB: dense Gram super-block edge in tiles (0: by F panel size)
  int dense_bk = 128;       // KMG_DENSE_BK: dense Gram k-stage bytes, 64 or 128 (128: half the
                            // barriers; MM k=7 N=20000 3.38 -> 3.13 ms, k=6 0.92 -> 0.87,
                            // SP k=5 0.38 -> 0.367; profiles/r02ay_dense_bk_ab.jsonl)
  int dense_half = -1;      // KMG_DENSE_HALF: dense Gram tiles over two 4-wave workgroups (BK
                            // 64), -1: when dp <= 1024 (SP k=5 N=20000 0.41 -> 0.39 ms; at
                            // dp >= 4096 BK 128 wins; profiles/r02bj_dense_epilogue_ab.jsonl)
  int check = 0;            // KMG_CHECK: 1 validate the neighbourhood lists' metadata after
                            // every fill (nb_check_kernel; one host sync a build) and fail with
                            // KMG_EINTERNAL before any Gram launch reads past a list; 2 the
                            // same after overwriting every list's piece counts (tests only)
};

int env_or(const char *name, int dflt) {
  const char *v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

void read_tuning(Tuning &t) {
  const Tuning d;
  t.sp_chunk = env_or("KMG_SP_CHUNK", d.sp_chunk);
  t.mm_chunk = env_or("KMG_MM_CHUNK", d.mm_chunk);
  t.algo = env_or("KMG_ALGO", d.algo);
  t.dense_kmax_sp = env_or("KMG_DENSE_KMAX_SP", d.dense_kmax_sp);
  t.dense_kmax_mm = env_or("KMG_DENSE_KMAX_MM", d.dense_kmax_mm);
  t.idx_seqs = env_or("KMG_IDX_SEQS", d.idx_seqs);
  t.idx_buckets = env_or("KMG_IDX_BUCKETS", d.idx_buckets);
  t.idx_threads = env_or("KMG_IDX_THREADS", d.idx_threads);
  t.poison = env_or("KMG_POISON", d.poison);
  t.potrf_upper = env_or("KMG_POTRF_UPPER", d.potrf_upper);
  t.chol = env_or("KMG_CHOL", d.chol);
  t.chol_panels = env_or("KMG_CHOL_PANELS", d.chol_panels);
  t.mm_form = env_or("KMG_MM_FORM", d.mm_form);
  t.esc_cap = env_or("KMG_ESC_CAP", d.esc_cap);
  t.mm_tri = env_or("KMG_MM_TRI", d.mm_tri);
  t.wd_form = env_or("KMG_WD_FORM", d.wd_form);
  t.ss_lpp = env_or("KMG_SS_LPP", d.ss_lpp);
  t.nb_threads = env_or("KMG_NB_THREADS", d.nb_threads);
  t.nb_lds512 = env_or("KMG_NB_LDS512", d.nb_lds512);
  if (t.nb_lds512 != 0) t.nb_lds512 = std::max(16, std::min(80, t.nb_lds512));
  t.nb_fill = env_or("KMG_NB_FILL", d.nb_fill);
  t.nb_pack_reads = env_or("KMG_NB_PACK_READS", d.nb_pack_reads);
  t.nb_fill_threads = env_or("KMG_NB_FILL_THREADS", d.nb_fill_threads);
  t.nb_unroll = env_or("KMG_NB_UNROLL", d.nb_unroll);
  if (t.nb_threads != 512 && t.nb_threads != 1024) t.nb_threads = 0;
  t.la_lpp = env_or("KMG_LA_LPP", d.la_lpp);
  t.sp_store = env_or("KMG_SP_STORE", d.sp_store);
  t.sp_order = env_or("KMG_SP_ORDER", d.sp_order);
  t.sp_rows = env_or("KMG_SP_ROWS", d.sp_rows);
  t.sp_cb_chunk = env_or("KMG_SP_CB_CHUNK", d.sp_cb_chunk);
  t.dense_sb = env_or("KMG_DENSE_SB", d.dense_sb);
  t.dense_bk = env_or("KMG_DENSE_BK", d.dense_bk);
  t.dense_half = env_or("KMG_DENSE_HALF", d.dense_half);
  t.check = env_or("KMG_CHECK", d.check);
  if (getenv("KMG_MM_CHUNK") == nullptr) t.mm_chunk = 0;  // 0: per-formulation default
}

}  // namespace

struct kmg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  DevBuf kmers, partials, tmp, off, ent, diagv, dsq, wtab;
  DevBuf hcnt, hstart;            // index build v2: per-(bucket, block) counts / local starts
  DevBuf feat, masks;             // dense formulation: int8 F, neighbour xor masks
  DevBuf feat32, k32;             // KMG_ALGO=3: fp32 F and the fp32 GEMM's K
  DevBuf dense_tiles;             // dense Gram tile order (dense_tile_order)
  int64_t dense_key[4] = {-1, -1, -1, -1};
  DevBuf slots;                   // mismatch slot layout (one 128-byte line per list)
  DevBuf gcoef;                   // generic WD/WDS kernel: beta_k, delta_s (device copies)
  DevBuf packed;                  // 2-bit packed sequence records (Packed, kmg_internal.h)
  DevBuf tri_stage, tri_scratch;  // upper-triangle multi-GPU build: round slabs, full rows
  DevBuf ovf;                     // 16-bit round slabs: count-overflow flag
  DevBuf esc, esc_all, esc_cnt;   // uint8 round slabs: escape list, all-gathered lists, counts
  uint32_t esc_cap = 0;           // entries of `esc` in use by the current build (0: none)
  int64_t cur_n = 0;              // columns of the current Gram call
  int32_t plan[6] = {-1, 0, 0, 0, 0, 0};  // last spectrum / mismatch call (kmg_last_plan)
  int32_t last_factor = 0;        // last KRR / KLR solve's factorisation (kmg_last_factorisation)
  DevBuf pr_summary, pr_rtot, pr_rbase, pr_cursor, pr_lines;  // pair (drop-two) table
  DevBuf nb_seg, nb_use, nb_lines;  // neighbourhood lists: segment ends, pieces in use, lists
  DevBuf chk;                       // KMG_CHECK: validation flag + first offending list
  DevBuf cb_scratch;                // column-block assembly: one rank's K[:, C_q] (n x block)
  Tuning tune;
  DevBuf cmb_k, cmb_ptrs, cmb_vec, cmb_out, cmb_tmp;  // combination consumers (host path)
  DevBuf sv_mat, sv_vec, sv_info;  // dense learners: factorised system, vectors, info/ipiv
  DevBuf sv_inv, sv_panel;         // blocked Cholesky: diagonal-block inverses, panel / sweep scratch
  rocblas_handle blas = nullptr;   // rocBLAS/rocSOLVER handle bound to `stream` (lazy)
  int masks_k = -1, masks_m = -1, nmask = 0;
  DevBuf h_codes, h_lens, h_out;  // host-path staging on the device
  DevBuf ft_cols;                 // kmg_features: the column k-mer codes
  DevBuf slabs;                   // kmg_gram_to_host: two device row slabs
  hipStream_t d2h_stream = nullptr;             // kmg_gram_to_host: slab copies out
  hipEvent_t ev_slab[2] = {nullptr, nullptr};   // slab Gram done / copied out
  hipEvent_t ev_out[2] = {nullptr, nullptr};
  int timing = 0;  // 0 off, 1 every stage, 2 the Gram and gather stages only
  // per-stage event pairs of every timed call since the last reset (read after a sync)
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> ev_log;
  size_t ev_used = 0;
  int last_call_first = 0;
  int64_t wtab_host[33] = {};
  bool wtab_valid = false;
  ncclComm_t comm = nullptr;
  hipStream_t comm_stream = nullptr;  // RCCL all-gathers of kmg_gram_blocks
  hipEvent_t ev_sync = nullptr;       // context stream <-> comm stream ordering
  hipEvent_t ev_tri[2] = {nullptr, nullptr};  // upper-triangle slabs released by their mirror
  hipStream_t unpack_stream = nullptr;          // upper triangle over RCCL: unpack of round t
  hipEvent_t ev_gath[2] = {nullptr, nullptr};   // overlaps the all-gather of round t + 1
  int last_wire_bytes = 0;                      // slab element bytes of the last blocks call
  hipStream_t chol_stream = nullptr;            // blocked Cholesky: next diagonal block, ahead
  hipEvent_t ev_chol[2] = {nullptr, nullptr};   // [0] its panel updated, [1] its factor done
  int nranks = 1, rank = 0;
  int lds_max = 0;  // LDS bytes a workgroup may allocate on the device (kmg_create)
};

namespace {

hipEvent_t pool_event(kmg_ctx *c) {
  if (c->ev_used == c->ev_pool.size()) {
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    c->ev_pool.push_back(e);
  }
  return c->ev_pool[c->ev_used++];
}

struct StageTimer {
  kmg_ctx *c;
  hipStream_t st;
  hipEvent_t end = nullptr;
  // events on stream s (default: the context stream)
  StageTimer(kmg_ctx *c_, int i, hipStream_t s = nullptr) : c(c_), st(s ? s : c_->stream) {
    if (c->timing == 1 ||
        (c->timing == 2 && (i == ST_GRAM || i == ST_GATHER || i == ST_MEMSET || i == ST_UNPACK ||
                            i == ST_MIRROR))) {
      hipEvent_t b = pool_event(c);
      end = pool_event(c);
      (void)hipEventRecord(b, st);
      c->ev_log.push_back({i, {b, end}});
    }
  }
  ~StageTimer() {
    if (end) (void)hipEventRecord(end, st);
  }
};

size_t dtype_size(int32_t dt) { return dt == KMG_F64 ? 8 : dt == KMG_U16 ? 2 : dt == KMG_U8 ? 1 : 4; }

int64_t pow4(int e) { return (int64_t)1 << (2 * e); }

// w_m(d): number of betas within Hamming distance m of two k-mers at distance d
// (the closed form of <Phi_x, Phi_y> for get_phi_km, kernels.py:161-175)
void mismatch_weights(int k, int m, int64_t *w) {
  auto C = [](int n, int r) -> int64_t {
    if (r < 0 || r > n) return 0;
    int64_t v = 1;
    for (int t = 1; t <= r; ++t) v = v * (n - r + t) / t;
    return v;
  };
  for (int d = 0; d <= 32; ++d) w[d] = 0;
  // two k-mers further apart than 2m share no beta within m of both: w[d > 2m] = 0
  for (int d = 0; d <= std::min(k, std::min(2 * m, 32)); ++d) {
    int64_t tot = 0;
    for (int i = 0; i <= k - d; ++i) {
      int64_t p3 = 1;
      for (int t = 0; t < i; ++t) p3 *= 3;
      for (int a = 0; a <= d; ++a)
        for (int b = 0; a + b <= d; ++b) {
          const int c = d - a - b;
          if (i + b + c > m || i + a + c > m) continue;
          int64_t multi = C(d, a) * C(d - a, b);
          tot += C(k - d, i) * p3 * multi * ((int64_t)1 << c);
        }
    }
    w[d] = tot;
  }
}

int check_params(const kmg_params *p, int64_t n, int64_t ldc, int32_t dt) {
  if (!p) return fail(KMG_EINVAL, "params is NULL");
  if (n < 0) return fail(KMG_EINVAL, "n < 0");
  if (ldc <= 0 && n > 0) return fail(KMG_EINVAL, "ldc must be > 0");
  if (dt != KMG_I32 && dt != KMG_F32 && dt != KMG_F64)
    return fail(KMG_EINVAL, "unknown out dtype %d", dt);
  return KMG_OK;
}

// ----------------------------------------------------------------- posting index
// codes != nullptr: the records in pk are packed by the index build itself (fused into the
// v2 local pass; a separate pack launch before the v1 passes)
int build_index(kmg_ctx *c, IndexGeom &g, const Packed &pk, const uint8_t *codes = nullptr,
                const int32_t *lens = nullptr, int64_t ldc = 0) {
  // coarse buckets (one fine block each), fine LDS histogram <= 2^14 bins: ~384 for the
  // spectrum index, ~1024 for the k-copy mismatch index (16.7M occurrences at N=20000,
  // where 288 buckets left the fine pass at 240 us and 576 halved it); large builds one
  // bucket per ~40000 occurrences, up to 4096 (N=200000 MM(9,1), 167M occurrences:
  // place + fine 3.95 -> 2.65 ms at 4096, profiles/r02ad_index_geometry.jsonl)
  const int64_t occ = g.n * g.pmax * std::max(1, g.copies);
  const int target_buckets =
      c->tune.idx_buckets > 0 ? c->tune.idx_buckets
                              : (int)std::max<int64_t>(g.copies > 1 ? 1024 : 384,
                                                       std::min<int64_t>(4096, occ / 40000));
  g.fine_bits = 8;
  while (g.fine_bits < 14 && (g.nbins() >> g.fine_bits) > target_buckets) ++g.fine_bits;
  // sequences per partition block: 80, or enough for at most ~256 blocks, so the gather
  // pass keeps every segment's items in registers (N=100000 spectrum: fine 125 -> 93 us;
  // N=200000 MM(9,1): place + fine 2.81 -> 2.35 ms; profiles/r02bb_index_seqs.jsonl,
  // r02be_index_seqs_mm.jsonl)
  g.seqs_per_block = c->tune.idx_seqs > 0 ? c->tune.idx_seqs
                                          : (int)std::max<int64_t>(80, (g.n + 255) / 256);
  {  // LDS: two bucket arrays + the staged packed records
    const int64_t budget = 150 * 1024 - 8 * (g.nbins() >> g.fine_bits) - 4096;
    g.seqs_per_block = (int)std::max<int64_t>(1, std::min<int64_t>(g.seqs_per_block, budget / (4 * pk.ldp)));
  }
  g.part_threads = std::min(1024, std::max(64, c->tune.idx_threads));
  const int64_t nb = g.nbins();
  const int64_t nbk = g.nbuckets();
  if (nbk > 16384) return fail(KMG_EUNSUPPORTED, "index too large (%lld bins)", (long long)nb);
  if (pk.ldp * 4 > 8192) return fail(KMG_EUNSUPPORTED, "sequences longer than 8192");
  const int64_t items = g.n * g.pmax * g.copies;
  if ((double)items >= 4294967295.0)
    return fail(KMG_EUNSUPPORTED, "too many k-mer occurrences for 32-bit offsets");
  const int64_t nblk = (g.n + g.seqs_per_block - 1) / g.seqs_per_block;
  const int64_t cap = (int64_t)g.seqs_per_block * g.pmax * g.copies;
  if (g.n == 0) return KMG_OK;
  // the partition build (two launches, no device-scope atomics): its gather pass holds one
  // fine histogram and two words per partition block in LDS
  if (index_gather_lds(g, nblk) > 150 * 1024 || nblk * cap >= ((int64_t)1 << 34))
    return fail(KMG_EUNSUPPORTED, "index build: %lld partition blocks exceed the LDS budget",
                (long long)nblk);
  KMG_TRY(c->hcnt.ensure(sizeof(uint32_t) * (size_t)(nbk * nblk)));
  KMG_TRY(c->hstart.ensure(sizeof(uint32_t) * (size_t)(nbk * nblk)));
  KMG_TRY(c->tmp.ensure(sizeof(uint32_t) * (size_t)(nblk * cap)));
  KMG_TRY(c->off.ensure(sizeof(uint32_t) * (size_t)(nb + 1)));
  KMG_TRY(c->ent.ensure(sizeof(uint16_t) * (size_t)(items + 512)));  // + pad: whole-piece reads
  {
    StageTimer t(c, ST_PLACE);
    KMG_HIP(launch_index_local(g, pk, codes, lens, ldc, (int)nblk, (uint32_t)cap,
                               c->hcnt.as<uint32_t>(), c->hstart.as<uint32_t>(),
                               c->tmp.as<uint32_t>(), c->stream));
  }
  {
    StageTimer t(c, ST_FINE);
    KMG_HIP(launch_index_gather(g, (int)nblk, (uint32_t)cap, c->hcnt.as<uint32_t>(),
                                c->hstart.as<uint32_t>(), c->tmp.as<uint32_t>(),
                                c->off.as<uint32_t>(), c->ent.as<uint16_t>(), c->stream));
  }
  return KMG_OK;
}

void choose_chunks(IndexGeom &g, int max_chunk) {
  if (g.n <= 0) {
    g.chunk = 8;
    g.nchunks = 1;
    return;
  }
  const int64_t nch = (g.n + max_chunk - 1) / max_chunk;
  int64_t ch = (g.n + nch - 1) / nch;
  ch = (ch + 7) & ~7LL;
  g.chunk = (int)ch;
  g.nchunks = (int)((g.n + ch - 1) / ch);
}

int upload_wtab(kmg_ctx *c, const int64_t *w) {
  if (c->wtab_valid && memcmp(c->wtab_host, w, sizeof(int64_t) * 33) == 0) return KMG_OK;
  KMG_TRY(c->wtab.ensure(sizeof(int64_t) * 33));
  memcpy(c->wtab_host, w, sizeof(int64_t) * 33);
  c->wtab_valid = true;
  KMG_HIP(hipMemcpyAsync(c->wtab.p, c->wtab_host, sizeof(int64_t) * 33, hipMemcpyHostToDevice,
                         c->stream));
  // pageable source: make the copy complete before the table can change
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

int diag_hamming(kmg_ctx *c, const IndexGeom &g, const Packed &pk) {
  int max_dist = 0;  // weights are zero past this Hamming distance
  for (int d = 0; d <= 32; ++d)
    if (c->wtab_host[d] != 0) max_dist = d;
  KMG_TRY(c->diagv.ensure(sizeof(double) * (size_t)(g.n > 0 ? g.n : 1)));
  KMG_TRY(c->dsq.ensure(sizeof(double) * (size_t)(g.n > 0 ? g.n : 1)));
  if (g.pmax > 4096) return fail(KMG_EUNSUPPORTED, "more than 4096 k-mers per sequence");
  StageTimer t(c, ST_DIAG);
  KMG_HIP(launch_diag_hamming(g, pk, c->wtab.as<int64_t>(), max_dist, c->diagv.as<double>(),
                              c->dsq.as<double>(), c->stream));
  return KMG_OK;
}

// Max symbol code and min length over the device-resident rows (one small kernel and a
// stream sync; only the kernels that need it call this).
int row_stats(kmg_ctx *c, const uint8_t *d_codes, const int32_t *d_lens, int64_t n, int64_t ldc,
              uint32_t &max_code, uint32_t &min_len) {
  max_code = 0;
  min_len = 0;
  if (n <= 0) return KMG_OK;
  KMG_TRY(c->ovf.ensure(4 * sizeof(uint32_t)));
  const uint32_t init[2] = {0u, 0xFFFFFFFFu};
  KMG_HIP(hipMemcpyAsync(c->ovf.p, init, sizeof(init), hipMemcpyHostToDevice, c->stream));
  SeqSpec q{d_codes, d_lens, n, ldc, 0};
  KMG_HIP(launch_row_stats(q, c->ovf.as<uint32_t>(), c->stream));
  uint32_t st[2];
  KMG_HIP(hipMemcpyAsync(st, c->ovf.p, sizeof(st), hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  max_code = st[0];
  min_len = st[1];
  return KMG_OK;
}

// ----------------------------------------------------------------- dense formulation
// xor masks of every k-mer within Hamming distance m of a k-mer (2-bit letters; a
// non-zero xor of a letter is one of the 3 other letters): sum_{t<=m} C(k,t) 3^t masks.
int64_t dense_mask_count(int k, int m) {
  int64_t tot = 0, c = 1, p3 = 1;
  for (int t = 0; t <= std::min(m, k); ++t) {
    tot += c * p3;
    c = c * (k - t) / (t + 1);
    p3 *= 3;
  }
  return tot;
}

int upload_masks(kmg_ctx *c, int k, int m) {
  if (c->masks_k == k && c->masks_m == m) return KMG_OK;
  std::vector<uint32_t> masks;
  masks.push_back(0);
  // breadth-first over Hamming weight: extend every mask of weight t by one more
  // position above its highest set position
  std::vector<std::pair<uint32_t, int>> cur = {{0u, -1}};
  for (int t = 1; t <= std::min(m, k); ++t) {
    std::vector<std::pair<uint32_t, int>> nxt;
    for (auto &e : cur)
      for (int pos = e.second + 1; pos < k; ++pos)
        for (uint32_t x = 1; x <= 3; ++x) {
          const uint32_t mk = e.first | (x << (2 * pos));
          nxt.push_back({mk, pos});
          masks.push_back(mk);
        }
    cur.swap(nxt);
  }
  KMG_TRY(c->masks.ensure(sizeof(uint32_t) * masks.size()));
  KMG_HIP(hipMemcpyAsync(c->masks.p, masks.data(), sizeof(uint32_t) * masks.size(),
                         hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));  // pageable source
  c->masks_k = k;
  c->masks_m = m;
  c->nmask = (int)masks.size();
  return KMG_OK;
}

// Columns per chunk of the pair (drop-two) table: the fewest expected 128-byte lines per
// row over all chunkings whose LDS accumulator fits (<= 38400 int32 columns) and whose mean
// group stays <= 190 entries (groups above 255 take the slow wide path).  Lines of a
// group of n ~ Poisson(mean) entries: ceil((16 + 2n) / 128).
int pair_chunk(int64_t n, int pmax, int k, int cap) {
  const double keys = (double)pow4(k - 2);
  const int64_t max_chunk = std::min<int64_t>(cap > 0 ? cap : 38400, 38400);
  int64_t best = std::min<int64_t>(n, max_chunk);
  double best_lines = 1e300;
  for (int64_t nch = (n + max_chunk - 1) / max_chunk; nch <= (n + max_chunk - 1) / max_chunk + 16; ++nch) {
    const int64_t ch = (n + nch - 1) / nch;
    const double mean = (double)ch * pmax / keys;
    if (mean > 190.0 && nch < (n + 7) / 8) continue;
    double e = 0.0, pr = std::exp(-mean), cdf = 0.0;  // E[ceil((16 + 2X) / 128)], X ~ Poisson
    for (int x = 0; x < 2000 && cdf < 1.0 - 1e-12; ++x) {
      if (x > 0) pr *= mean / x;
      cdf += pr;
      e += pr * (x == 0 ? 0.0 : std::ceil((16.0 + 2.0 * x) / 128.0));
    }
    const double lines = (double)nch * e;
    if (lines < best_lines) {
      best_lines = lines;
      best = ch;
    }
  }
  return (int)std::max<int64_t>(8, (best + 7) & ~7LL);
}

// Cost of a chunking, in seconds: a row reads nch x lines_per_window_chunk lines per window,
// or, for a full square K built by its upper block triangle (tri_esz > 0), (nch + 1) / 2 of
// them on average while the mirror moves 2 tri_esz (nch - 1) / (2 nch) n^2 bytes; lines are
// priced at the measured random-line rate of the Infinity Cache (54 G lines/s), the mirror at
// 5.5 TB/s.
double tri_cost(int64_t n, int pmax, double lines_per_window_chunk, int64_t nch, int tri_esz) {
  if (tri_esz <= 0) return (double)nch * lines_per_window_chunk;
  const double lines = (double)n * pmax * lines_per_window_chunk * (double)(nch + 1) / 2.0;
  const double mirror = 2.0 * tri_esz * (double)n * n * (double)(nch - 1) / (2.0 * nch);
  return lines / 54e9 + mirror / 5.5e12;
}

// Columns per chunk of the drop-one slot table.  A row reads one 128-byte line per
// (chunk, list), so the lines per row are nch x (1 + the CSR-tail cost of the groups
// past KMG_SLOT_INLINE entries): fewer, fuller chunks win until the inline line
// overflows.  Cost per list: 1 line + T with probability P(X > inline), X ~
// Poisson(chunk * pmax / 4^(k-1)), T = 6 lines: the CSR tail (offsets, then 2-byte
// entries read by two lanes) costs about six lines' time, calibrated on N=200000
// MM(9,1) (25000-row slab: 10 chunks 46.8 ms, 8 chunks 38.7, 7 chunks 34.8, 6 chunks
// 35.7; profiles/r02ac_*).  Largest chunk: the int32 LDS accumulator plus the kernel's
// tables (launch_gram_mismatch1_slots) in 160 KB, and uint16 entries (<= 65536 columns).
int slot_chunk(int64_t n, int pmax, int k, int ldp, int cap, int tri_esz) {
  const int nsub = k + 3 * k * (k - 1) / 2;
  int64_t max_chunk = (160 * 1024 / 4 - (int64_t)pmax * k - nsub - ldp) & ~7LL;
  max_chunk = std::min<int64_t>(max_chunk, 65536);
  if (cap > 0) max_chunk = std::min<int64_t>(max_chunk, std::max(8, cap));
  if (max_chunk < 8) return 8;
  const double keys = (double)pow4(k - 1);
  int64_t best = std::min<int64_t>(std::max<int64_t>(n, 8), max_chunk);
  double best_cost = 1e300;
  const int64_t nch0 = std::max<int64_t>(1, (n + max_chunk - 1) / max_chunk);
  for (int64_t nch = nch0; nch <= nch0 + 16; ++nch) {
    const int64_t ch = ((n + nch - 1) / nch + 7) & ~7LL;
    if (ch > max_chunk) continue;
    const double mean = (double)ch * pmax / keys;
    double pr = std::exp(-mean), cdf = 0.0;  // P(X <= inline)
    for (int x = 0; x <= KMG_SLOT_INLINE; ++x) {
      if (x > 0) pr *= mean / x;
      cdf += pr;
    }
    const double per = (double)nsub * (1.0 + 6.0 * std::max(0.0, 1.0 - cdf));
    const double cost = tri_cost(n, pmax, per, nch, tri_esz);
    if (cost < best_cost * (1.0 - 1e-12)) {
      best_cost = cost;
      best = ch;
    }
  }
  return (int)std::max<int64_t>(8, best);
}

// Columns per chunk of the neighbourhood-list Gram (kmg_nbhd.hip).  A row reads, per chunk,
// its windows' lists: (1 + 3k) x 2 B + 9k(k-1)/2 x b2 per occurrence (b2 = 1.08 B for a packed
// segment 2, 2 B for 16-bit lists) x P x chunk x P / 4^k, plus three padded segment tails
// per list, so the chunk count barely changes the bytes a full row reads; it only matters
// for a square K built by its upper block triangle (tri_esz > 0), where a row reads
// (nch + 1) / (2 nch) of them and writes as much of its K row, and the mirror moves
// 2 esz (nch - 1) / (2 nch) n^2 bytes.  Priced at 6 TB/s for the Gram and 5 TB/s for the
// mirror.  Largest chunk: the int32 LDS accumulator beside the row tables, and where
// segment 2 packs, the sorted fill's LDS buffer (nb_sorted_max_chunk: ~24900 at k = 9).
int nb_chunk(int64_t n, int pmax, int k, int ldp, int cap, int tri_esz, int threads, bool sorted,
             int lds512_kb = 40) {
  // two workgroups a CU (their table builds, epilogues and streams overlap; one a CU measured
  // 22 % slower at N=20000, profiles/r05g_*): the accumulator, 16 dummy columns and the row
  // table in 80 KB (1024 threads) or 40 KB (512)
  // (sizing for one workgroup a CU, chunks up to ~40000, measured slower for the config-5
  // slab too: Gram 26.0 -> 30.5 ms, profiles/r05v.jsonl)
  const int64_t lds_words = (threads == 512 ? lds512_kb : 80) * 1024 / 4;
  int64_t max_chunk = (lds_words - 16 - 4 * (int64_t)pmax - 2 - ldp) & ~7LL;
  max_chunk = std::min<int64_t>(max_chunk, 65536 - 128);
  const int smax = sorted ? nb_sorted_max_chunk(k, pmax) : 0;
  if (smax >= 8) max_chunk = std::min<int64_t>(max_chunk, smax);
  if (cap > 0) max_chunk = std::min<int64_t>(max_chunk, std::max(8, cap));
  if (max_chunk < 8) return 8;
  const int64_t nch0 = std::max<int64_t>(1, (n + max_chunk - 1) / max_chunk);
  const double n01 = 1 + 3 * k, n2 = 4.5 * k * (k - 1);
  const double b2 = smax >= 8 ? 1.08 : 2.0;
  const double dens = (double)pmax / (double)pow4(k);  // occurrences of a k-mer per column
  const int esz = tri_esz > 0 ? tri_esz : 4;
  int64_t best = std::min<int64_t>(std::max<int64_t>(n, 8), max_chunk);
  double best_cost = 1e300;
  for (int64_t nch = nch0; nch <= (tri_esz > 0 ? nch0 + 8 : nch0); ++nch) {
    const int64_t ch = ((n + nch - 1) / nch + 7) & ~7LL;
    if (ch > max_chunk) continue;
    const double f = tri_esz > 0 ? (double)(nch + 1) / (2.0 * nch) : 1.0;
    const double row_reads = (2.0 * n01 + b2 * n2) * pmax * dens * (double)n + 2.0 * 10.5 * pmax * nch;
    const double gram = (double)n * (row_reads + esz * (double)n) * f;
    const double mirror = tri_esz > 0 ? 2.0 * esz * (double)n * n * (double)(nch - 1) / (2.0 * nch) : 0.0;
    // + building the lists: ~2 ns per (chunk, k-mer) bin plus the table at ~1 TB/s (grouped
    // fill, measured: N=20000 one chunk 1.44 ms, N=200000 five chunks ~13 ms)
    const double build = (double)nch * (double)pow4(k) * 2.0e-9 +
                         (2.0 * n01 + b2 * n2) * (double)n * pmax / 1e12;
    const double cost = gram / 6e12 + mirror / 5e12 + build;
    if (cost < best_cost * (1.0 - 1e-12)) {
      best_cost = cost;
      best = ch;
    }
  }
  return (int)std::max<int64_t>(8, best);
}

// Row ranges of one Gram call: every range [row0, row1) x all n columns is written at
// `out` (row row0); the index / features / diagonal are built once per call.  `after(q)`
// runs once range q's Gram launch is enqueued (the multi-GPU path hangs its all-gather of a
// round there).
// ld > 0 / col_lo > 0: this range's own leading dimension and first written column
// (upper-triangle round slabs of kmg_gram_blocks; `out` then points at column 0 of row
// row0 of a row whose columns < col_lo are never written).
struct RowRange {
  int64_t row0, row1;
  void *out;
  int64_t ld = 0, col_lo = 0;
};
using AfterRange = std::function<int(size_t)>;

// native: the launch's kernels honour OutSpec::col_lo (spectrum, mismatch slots / pairs)
// when it is a multiple of 8; otherwise a range with col_lo > 0 is computed as full rows
// into a scratch slab and its columns >= col_lo copied out.
template <typename Launch>
int each_range(kmg_ctx *c, const std::vector<RowRange> &ranges, const OutSpec &o,
               const AfterRange &after, Launch &&launch, bool native = false) {
  const size_t esz = dtype_size(o.dtype);
  for (size_t q = 0; q < ranges.size(); ++q) {
    const RowRange &rg = ranges[q];
    OutSpec oq = o;
    oq.out = rg.out;
    if (rg.ld > 0) oq.ld = rg.ld;
    oq.col_lo = rg.col_lo;
    if (oq.col_lo > 0 && (!native || (oq.col_lo & 7)) && rg.row1 > rg.row0) {
      const int64_t n = c->cur_n, rows = rg.row1 - rg.row0;
      KMG_TRY(c->tri_scratch.ensure(esz * (size_t)rows * n));
      OutSpec of = o;
      of.out = c->tri_scratch.p;
      of.ld = n;
      of.col_lo = 0;
      {
        StageTimer t(c, ST_GRAM);
        KMG_HIP(launch(rg.row0, rg.row1, of));
      }
      KMG_HIP(hipMemcpy2DAsync((char *)rg.out + (size_t)oq.col_lo * esz, (size_t)oq.ld * esz,
                               (const char *)c->tri_scratch.p + (size_t)oq.col_lo * esz,
                               (size_t)n * esz, (size_t)(n - oq.col_lo) * esz, (size_t)rows,
                               hipMemcpyDeviceToDevice, c->stream));
    } else {
      StageTimer t(c, ST_GRAM);
      KMG_HIP(launch(rg.row0, rg.row1, oq));
    }
    if (after) KMG_TRY(after(q));
  }
  return KMG_OK;
}

// Tile order of gram_dense_kernel: S x S super-blocks of 256 x 256 tiles, super-row-major
// (tiles tm <= tn only for the full square).  The launch deals contiguous ranges of this
// order to the XCDs, so the ~32 tiles in flight on one XCD read S row panels and 2S column
// panels of F (256 x dp bytes each) that the XCD's L2 / the Infinity Cache then serve
// several times, where the plain row-band order read a fresh column panel per tile (F
// panel reads ~ the K bytes written at k = 5).  S = 4 measured best at every k
// (N=20000 int32 Gram, S = 1 / 2 / 4 / 8: SP k=5 0.425 / 0.399 / 0.377 / 0.377 ms,
// SP k=4 0.325 / 0.321 / 0.268 / 0.327, MM k=6 0.990 / 0.948 / 0.922 / 0.931;
// profiles/r02ae_dense_superblocks.jsonl).  The list is cached per geometry (one upload
// per shape, stream-synchronised).
int dense_tile_order(kmg_ctx *c, int64_t n, int64_t r0, int64_t r1, int dp, const uint32_t **out) {
  *out = nullptr;
  const int64_t rows = r1 - r0;
  const bool sym = r0 == 0 && rows == n;
  const int64_t tm_n = (rows + 255) / 256, tn_n = (n + 255) / 256;
  if (rows <= 0 || n <= 0 || tm_n > 65535 || tn_n > 65535) return KMG_OK;  // kernel's own order
  (void)dp;
  const int S = c->tune.dense_sb > 0 ? std::min(c->tune.dense_sb, 64) : 4;
  const int64_t key[4] = {tm_n, tn_n, sym ? 1 : 0, S};
  if (memcmp(key, c->dense_key, sizeof(key)) != 0) {
    std::vector<uint32_t> v;
    v.reserve((size_t)(sym ? tn_n * (tn_n + 1) / 2 : tm_n * tn_n));
    const int64_t sm = (tm_n + S - 1) / S, sn = (tn_n + S - 1) / S;
    for (int64_t TM = 0; TM < sm; ++TM)
      for (int64_t TN = sym ? TM : 0; TN < sn; ++TN)
        for (int64_t tm = TM * S; tm < std::min(tm_n, TM * S + S); ++tm)
          for (int64_t tn = TN * S; tn < std::min(tn_n, TN * S + S); ++tn)
            if (!sym || tn >= tm) v.push_back((uint32_t)tm | ((uint32_t)tn << 16));
    KMG_TRY(c->dense_tiles.ensure(sizeof(uint32_t) * v.size()));
    KMG_HIP(hipMemcpyAsync(c->dense_tiles.p, v.data(), sizeof(uint32_t) * v.size(),
                           hipMemcpyHostToDevice, c->stream));
    KMG_HIP(hipStreamSynchronize(c->stream));  // pageable source
    memcpy(c->dense_key, key, sizeof(key));
  }
  *out = c->dense_tiles.as<uint32_t>();
  return KMG_OK;
}

// F = int8 count / neighbour-count rows, diagonal ||F_i||^2, then K = F F^T (MFMA)
int gram_dense(kmg_ctx *c, int k, int m, int window, const uint8_t *d_codes,
               const int32_t *d_lens, int64_t n, int64_t ldc, const std::vector<RowRange> &ranges,
               OutSpec o, bool normalize, const AfterRange &after) {
  const int dp = (int)std::max<int64_t>(128, pow4(k));
  KMG_TRY(upload_masks(c, k, m));
  const int64_t rows_alloc = ((n + 255) & ~255LL) + 256;  // 256-row GEMM tiles, zero pad
  KMG_TRY(c->feat.ensure((size_t)rows_alloc * dp));
  KMG_TRY(c->diagv.ensure(sizeof(double) * (size_t)(n > 0 ? n : 1)));
  KMG_TRY(c->dsq.ensure(sizeof(double) * (size_t)(n > 0 ? n : 1)));
  {
    StageTimer t(c, ST_FEATURES);
    KMG_HIP(hipMemsetAsync(c->feat.as<int8_t>() + n * (int64_t)dp, 0,
                           (size_t)(rows_alloc - n) * dp, c->stream));
    KMG_HIP(launch_dense_features(d_codes, d_lens, ldc, n, k, window, dp,
                                  c->masks.as<uint32_t>(), c->nmask, c->feat.as<int8_t>(),
                                  c->diagv.as<double>(), c->dsq.as<double>(), c->stream));
  }
  if (normalize) {
    o.normalize = 1;
    o.diagv = c->diagv.as<double>();
    o.dsq = c->dsq.as<double>();
  }
  if (c->tune.algo == 3) {
    // BASELINE configs[3]'s literal "count-vector fp32 GEMM": F widened to fp32 and
    // K = F F^T by rocblas_sgemm (dense fp32 MFMA; 2 N^2 4^k flops), then written out
    KMG_TRY(c->feat32.ensure(sizeof(float) * (size_t)n * dp));
    KMG_TRY(c->k32.ensure(sizeof(float) * (size_t)n * n));
    {
      StageTimer t(c, ST_FEATURES);
      KMG_HIP(launch_i8_to_f32(c->feat.as<int8_t>(), n * (int64_t)dp, c->feat32.as<float>(), c->stream));
    }
    KMG_TRY(blas_handle(c));
    {
      StageTimer t(c, ST_GRAM);
      const float one = 1.0f, zero = 0.0f;
      // column-major view: G = F^T is dp x n (lda dp); K = G^T G (n x n, symmetric)
      const rocblas_status st = rocblas_sgemm(c->blas, rocblas_operation_transpose,
                                              rocblas_operation_none, (rocblas_int)n, (rocblas_int)n,
                                              (rocblas_int)dp, &one, c->feat32.as<float>(), dp,
                                              c->feat32.as<float>(), dp, &zero, c->k32.as<float>(),
                                              (rocblas_int)n);
      if (st != rocblas_status_success)
        return fail(KMG_EHIP, "rocblas_sgemm: %s", rocblas_status_to_string(st));
    }
    return each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
      StageTimer t(c, ST_EXTRACT);
      return launch_f32_gram_out(c->k32.as<float>(), n, r0, r1, oq, c->stream);
    });
  }
  return each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
    const uint32_t *order = nullptr;
    if (dense_tile_order(c, n, r0, r1, dp, &order) != KMG_OK) return hipErrorInvalidValue;
    return launch_gram_dense(c->feat.as<int8_t>(), dp, n, r0, r1, order, oq, c->stream,
                             c->tune.dense_bk,
                             c->tune.dense_half < 0 ? dp <= 1024 : c->tune.dense_half != 0);
  });
}

// gappy (k, g), intended semantics (kernels.py:420-455 as the report describes it): binary
// presence features over the (k-g)-mers, K = F F^T on the int8 MFMA path, normalize_K fused
int gram_gappy_intended(kmg_ctx *c, int k, int g, int window, const uint8_t *d_codes,
                        int64_t n, int64_t ldc, const std::vector<RowRange> &ranges, OutSpec o,
                        bool normalize, const AfterRange &after) {
  const int kk = k - g;
  const int dp = (int)std::max<int64_t>(128, pow4(kk));
  std::vector<uint32_t> combos;  // kept positions of every C(k, kk) combination, 4 bits each
  for (uint32_t sel = 0; sel < (1u << k); ++sel) {
    if (__builtin_popcount(sel) != kk) continue;
    uint32_t cm = 0;
    int q = 0;
    for (int pos = 0; pos < k; ++pos)
      if (sel >> pos & 1u) cm |= (uint32_t)pos << (4 * q++);
    combos.push_back(cm);
  }
  KMG_TRY(c->masks.ensure(sizeof(uint32_t) * combos.size()));
  KMG_HIP(hipMemcpyAsync(c->masks.p, combos.data(), sizeof(uint32_t) * combos.size(),
                         hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));  // pageable source
  c->masks_k = -1;                           // the neighbour-mask cache no longer holds masks
  const int64_t rows_alloc = ((n + 255) & ~255LL) + 256;  // 256-row GEMM tiles, zero pad
  KMG_TRY(c->feat.ensure((size_t)rows_alloc * dp));
  KMG_TRY(c->diagv.ensure(sizeof(double) * (size_t)(n > 0 ? n : 1)));
  KMG_TRY(c->dsq.ensure(sizeof(double) * (size_t)(n > 0 ? n : 1)));
  {
    StageTimer t(c, ST_FEATURES);
    KMG_HIP(hipMemsetAsync(c->feat.as<int8_t>() + n * (int64_t)dp, 0,
                           (size_t)(rows_alloc - n) * dp, c->stream));
    KMG_HIP(launch_gappy_features(d_codes, ldc, n, k, kk, window, dp, c->masks.as<uint32_t>(),
                                  (int)combos.size(), c->feat.as<int8_t>(),
                                  c->diagv.as<double>(), c->dsq.as<double>(), c->stream));
  }
  if (normalize) {
    o.normalize = 1;
    o.diagv = c->diagv.as<double>();
    o.dsq = c->dsq.as<double>();
  }
  return each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
    const uint32_t *order = nullptr;
    if (dense_tile_order(c, n, r0, r1, dp, &order) != KMG_OK) return hipErrorInvalidValue;
    return launch_gram_dense(c->feat.as<int8_t>(), dp, n, r0, r1, order, oq, c->stream,
                             c->tune.dense_bk,
                             c->tune.dense_half < 0 ? dp <= 1024 : c->tune.dense_half != 0);
  });
}

// ----------------------------------------------------------------- dispatch
// Formulation of a spectrum / mismatch call (one decision, used by gram_device and by
// kmg_gram_blocks' choice of the round-slab format).
// (kmg_last_plan numbers: SM_PL, round 3's pair lines, was removed in round 5)
enum SmPath { SM_DENSE, SM_HAMMING, SM_POSTING, SM_SLOTS, SM_PAIRS, SM_PL, SM_NB };
constexpr int32_t KMG_PLAN_GENERIC = 7;  // kmg_last_plan: the per-pair kernels of k > 16
SmPath sm_path(const Tuning &t, const kmg_params *p, int pmax, int64_t n) {
  const bool mm = p->kind == KMG_MISMATCH;
  const int k = p->k;
  const bool exact = !mm || p->m == 0;  // spectrum-shaped: only ham 0 counts
  // mismatch m = 1, auto (N=20000, float64 normalised, profiles/r05s_kforms.jsonl):
  //   k = 8..10: the neighbourhood lists (k = 8: 4.17 ms vs 6.71 slot table, 15.9 pair
  //     table; k = 9: 2.9-3.1 ms; k = 10: 4.14 vs 6.13 / 4.95);
  //   k = 11: the drop-two pair table (8.59 vs 9.11 slots; the lists' fill of 4^11 bins a
  //     chunk alone takes 11.5 ms);
  //   k = 12: the drop-one slot table (14.5 ms; the pair table's offsets overflow at N=20000).
  //   k < 8: the dense count-vector GEMM where counts fit (dense_ok), else all-pairs Hamming.
  const int form = t.mm_form;
  const bool s1 = mm && p->m == 1;
  const bool use_nb = s1 && k >= 4 && k <= 12 && (form == 4 || (form == 0 && k >= 8 && k <= 10));
  const bool use_pairs = s1 && !use_nb &&
                         (form == 2 ? (k >= 3 && k <= 12) : (form == 0 && k == 11));
  const bool use_slots = s1 && !use_pairs && !use_nb && k >= 8 && k <= 12 && form != 2;
  const bool use_index = (exact && k <= 12) || use_slots || use_pairs || use_nb;
  // formulation: dense int8 MFMA GEMM over 4^k count columns for small k (exact when
  // every count <= 127, i.e. <= 127 windows), posting lists for large sparse k,
  // all-pairs Hamming otherwise.  KMG_ALGO: 0 auto, 1 dense, 2 index/hamming.
  const int mm_eff = mm ? std::min(p->m, k) : 0;
  const bool dense_ok = k <= 8 && pmax <= 127 && dense_mask_count(k, mm_eff) <= 4096;
  if (t.algo == 1 || t.algo == 3 || (t.algo == 0 && dense_ok &&
                      (mm ? (k <= t.dense_kmax_mm) : (k <= t.dense_kmax_sp))))
    return SM_DENSE;  // (algo 1 without dense_ok: gram_device reports it)
  if (!use_index) return SM_HAMMING;
  if (use_pairs) return SM_PAIRS;
  if (use_nb) return SM_NB;
  return exact ? SM_POSTING : SM_SLOTS;
}

// cseq0 / ncols >= 0: a column block -- columns j of the output are sequences cseq0 + j,
// j < ncols (kmg_gram_device_cols; neighbourhood-list formulation only)
int gram_device(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes, const int32_t *d_lens,
                int maxlen, int64_t n, int64_t ldc, const std::vector<RowRange> &ranges,
                int32_t dt, int64_t ld, const AfterRange &after = nullptr, int64_t cseq0 = 0,
                int64_t ncols = -1) {
  c->last_call_first = (int)c->ev_log.size();
  c->cur_n = n;
  const bool colblk = ncols >= 0;
  if (!colblk) ncols = n;
  // column blocks: only the posting-list paths below index a block's sequences (checked
  // there); every other kernel writes whole rows, which a block's ld_out cannot hold
  if (colblk && p->kind != KMG_SPECTRUM && p->kind != KMG_MISMATCH)
    return fail(KMG_EUNSUPPORTED, "column blocks: spectrum / mismatch only");
  if (cseq0 < 0 || cseq0 + ncols > n) return fail(KMG_EINVAL, "bad column range");
  for (const RowRange &r : ranges)
    if (r.row0 < 0 || r.row1 > n || r.row0 > r.row1) return fail(KMG_EINVAL, "bad row range");
  if (n > 0 && ld < ncols) return fail(KMG_EINVAL, "ld_out < columns");
  const bool narrow = dt == KMG_U16 || dt == KMG_U8;
  if (narrow && p->kind != KMG_SPECTRUM && p->kind != KMG_MISMATCH)
    return fail(KMG_EINVAL, "internal: 8/16-bit slabs need a posting-list formulation");
  OutSpec o{nullptr, ld, dt, 0, nullptr, nullptr};
  if (narrow) {  // raw 8/16-bit slabs: counts past the slab's range raise this flag
    KMG_TRY(c->ovf.ensure(sizeof(uint32_t)));
    KMG_HIP(hipMemsetAsync(c->ovf.p, 0, sizeof(uint32_t), c->stream));
    o.ovf = c->ovf.as<uint32_t>();
    if (dt == KMG_U8 && c->esc_cap > 0) {  // escapes (kmg_gram_blocks sets the list up)
      o.esc = c->esc.as<uint4>();
      o.esc_n = c->esc_cnt.as<uint32_t>();
      o.esc_cap = c->esc_cap;
    }
  }
  if (c->tune.poison && n > 0)  // testing: no stale output can pass
    for (const RowRange &r : ranges)
      if (r.row1 > r.row0) {
        const int64_t rld = r.ld > 0 ? r.ld : ld;
        KMG_HIP(hipMemset2DAsync((char *)r.out + (size_t)r.col_lo * dtype_size(dt),
                                 (size_t)rld * dtype_size(dt), 0xA5,
                                 (size_t)(ncols - r.col_lo) * dtype_size(dt),
                                 (size_t)(r.row1 - r.row0), c->stream));
      }
  switch (p->kind) {
    case KMG_SPECTRUM:
    case KMG_MISMATCH: {
      const bool mm = p->kind == KMG_MISMATCH;
      const int k = p->k;
      if (k < 1) return fail(KMG_EINVAL, "k=%d < 1", k);
      if (mm && p->m < 0) return fail(KMG_EINVAL, "m < 0");
      IndexGeom g{};
      g.k = k;
      g.n = n;
      g.window = mm ? (p->window > 0 ? p->window : 101) : 0;
      // the mismatch window reads x[0 : window) of every row (kernels.py:171): rows narrower
      // than the window would read into the next row
      if (mm && n > 0 && ldc < g.window)
        return fail(KMG_EINVAL, "mismatch: code rows (%lld) shorter than the window %d",
                    (long long)ldc, g.window);
      // kmg_last_plan: reset first, so no return below reports the previous call's plan
      c->plan[0] = -1;
      c->plan[1] = c->plan[2] = c->plan[3] = c->plan[4] = c->plan[5] = 0;
      if (k > 16) {
        // k-mers past 32 bits: the generic per-pair kernels (kmg_generic.hip)
        c->plan[0] = KMG_PLAN_GENERIC;
        if (colblk) return fail(KMG_EUNSUPPORTED, "column blocks: k = %d past the posting-list paths", k);
        if (narrow) return fail(KMG_EINVAL, "internal: 8/16-bit slabs need a posting-list formulation");
        if (dt == KMG_I32 && p->normalize)
          return fail(KMG_EINVAL, "normalised output needs a floating dtype");
        const SeqSpec q{d_codes, d_lens, n, ldc, maxlen};
        const int sq = (ranges.size() == 1 && ranges[0].row0 == 0 && ranges[0].row1 == n &&
                        ranges[0].col_lo == 0) ? 1 : 0;
        bool unsupported = false;
        auto run = [&](hipError_t e) {
          if (e == hipErrorNotSupported) {
            unsupported = true;
            return hipSuccess;
          }
          return e;
        };
        int rc;
        if (!mm) {
          if (p->normalize) {  // normalize_K with the spectrum diagonal K(x, x)
            KMG_TRY(c->diagv.ensure(sizeof(double) * (size_t)std::max<int64_t>(1, n)));
            KMG_TRY(c->dsq.ensure(sizeof(double) * (size_t)std::max<int64_t>(1, n)));
            StageTimer t(c, ST_DIAG);
            KMG_HIP(run(launch_sp_generic_diag(q, k, c->diagv.as<double>(), c->dsq.as<double>(),
                                               c->stream)));
            o.normalize = 1;
            o.diagv = c->diagv.as<double>();
            o.dsq = c->dsq.as<double>();
          }
          rc = unsupported ? KMG_OK : each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
            return run(launch_gram_sp_generic(q, r0, r1, k, sq, oq, c->stream));
          });
        } else {
          int64_t w[33];
          mismatch_weights(k, p->m, w);
          const int maxd = std::min(k, std::min(2 * p->m, 32));
          const int P = std::max(0, g.window - k + 1);
          double wmax = 0.0;
          for (int d = 0; d <= maxd; ++d) wmax = std::max(wmax, (double)w[d]);
          if (p->m > 16 || wmax * P * P >= 4.0e18)
            return fail(KMG_EUNSUPPORTED, "mismatch (%d, %d): counts past 64 bits", k, p->m);
          KMG_TRY(upload_wtab(c, w));
          if (p->normalize) {
            KMG_TRY(c->diagv.ensure(sizeof(double) * (size_t)std::max<int64_t>(1, n)));
            KMG_TRY(c->dsq.ensure(sizeof(double) * (size_t)std::max<int64_t>(1, n)));
            StageTimer t(c, ST_DIAG);
            KMG_HIP(launch_mm_generic_diag(q, g.window, k, c->wtab.as<int64_t>(), maxd,
                                           c->diagv.as<double>(), c->dsq.as<double>(), c->stream));
            o.normalize = 1;
            o.diagv = c->diagv.as<double>();
            o.dsq = c->dsq.as<double>();
          }
          rc = each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
            return run(launch_gram_mm_generic(q, r0, r1, g.window, k, c->wtab.as<int64_t>(), maxd,
                                              sq, oq, c->stream));
          });
        }
        if (unsupported)
          return fail(KMG_EUNSUPPORTED, "k = %d: rows longer than 4096 symbols", k);
        return rc;
      }
      const int L = mm ? g.window : maxlen;
      g.pmax = L - k + 1 > 0 ? L - k + 1 : 1;
      if (g.pmax > 4095) return fail(KMG_EUNSUPPORTED, "more than 4095 k-mers per sequence");
      int64_t w[33];
      if (mm) {
        mismatch_weights(k, p->m, w);
      } else {
        for (int d = 0; d <= 32; ++d) w[d] = d == 0 ? 1 : 0;
      }
      const bool exact = !mm || p->m == 0;           // spectrum-shaped: only ham 0 counts
      SmPath path = sm_path(c->tune, p, g.pmax, n);
      if (colblk) {  // column blocks: the lists / postings over the block's sequences
        const bool cb_mm = mm && p->m == 1 && k >= 4 && k <= 12;
        const bool cb_sp = !mm && path == SM_POSTING;
        if (!(cb_mm || cb_sp) || (dt != KMG_I32 && dt != KMG_F32 && dt != KMG_F64) || after ||
            ranges.size() != 1 || ranges[0].col_lo != 0)
          return fail(KMG_EUNSUPPORTED, "column blocks: mismatch (k, 1) with 4 <= k <= 12, or the "
                      "spectrum posting-list path (6 <= k <= 12), only");
        if (cb_mm) path = SM_NB;
      }
      const bool use_pairs = path == SM_PAIRS, use_slots = path == SM_SLOTS;
      const bool use_nb = path == SM_NB;
      const bool use_index = path == SM_POSTING || use_slots || use_pairs || use_nb;
      // a full square K (one range over [0, n), every column written) of a mismatch
      // posting-list formulation: built by its upper block triangle, then mirrored
      // (OutSpec::tri; set below once the chunking is known)
      const bool square = ranges.size() == 1 && ranges[0].row0 == 0 && ranges[0].row1 == n &&
                          ranges[0].col_lo == 0 && !after && !narrow && n > 0 && !colblk;
      const int tri_esz = (c->tune.mm_tri && square && (use_slots || use_pairs || use_nb))
                              ? (int)dtype_size(dt) : 0;
      auto mirror = [&]() -> int {
        if (!o.tri) return KMG_OK;
        StageTimer t(c, ST_MIRROR);
        KMG_HIP(launch_mirror_chunks(ranges[0].out, ranges[0].ld > 0 ? ranges[0].ld : ld, n,
                                     g.chunk, (int)dtype_size(dt), c->stream));
        return KMG_OK;
      };
      // kmg_last_plan: formulation, then chunking / triangle / workgroup once chosen
      c->plan[0] = (int32_t)path;
      auto note_plan = [&](int threads) {
        c->plan[1] = g.chunk;
        c->plan[2] = g.nchunks;
        c->plan[3] = o.tri;
        c->plan[4] = threads;
      };
      if (dt == KMG_I32 && p->normalize)
        return fail(KMG_EINVAL, "normalised output needs a floating dtype");
      const int mm_eff = mm ? std::min(p->m, k) : 0;
      const bool dense = path == SM_DENSE;
      if (dense && !(k <= 8 && g.pmax <= 127 && dense_mask_count(k, mm_eff) <= 4096))
        return fail(KMG_EUNSUPPORTED, "dense formulation needs k <= 8 and <= 127 windows");
      // raw 16-bit round slabs (kmg_gram_blocks) only from the posting-list kernels
      if ((dt == KMG_U16 || dt == KMG_U8) &&
          (path == SM_DENSE || path == SM_HAMMING || (exact && g.pmax > 255)))
        return fail(KMG_EINVAL, "internal: 8/16-bit slabs need a posting-list formulation");
      if (dense)
        return gram_dense(c, k, mm_eff, mm ? g.window : 0, d_codes, d_lens, n, ldc, ranges, o,
                          mm && p->normalize, after);
      // 2-bit packed records of every sequence (kernels.py:187-193 `format`, as 2 bits a
      // letter plus a validity mask), read by the index build and the Gram kernels
      const int cw = packed_cw(ldc), mw = packed_mw(ldc);
      KMG_TRY(c->packed.ensure(sizeof(uint32_t) * (size_t)std::max<int64_t>(1, n) * (cw + mw)));
      const Packed pkd{c->packed.as<uint32_t>(), (int64_t)(cw + mw), cw};
      if (!use_index) {
        {
          StageTimer t(c, ST_PACK);
          KMG_HIP(launch_pack(d_codes, d_lens, n, ldc, g.window, c->packed.as<uint32_t>(), c->stream));
        }
        // all-pairs Hamming formulation (any m, k <= 16)
        if (g.pmax > 256) return fail(KMG_EUNSUPPORTED, "Hamming path needs <= 256 k-mers");
        g.copies = 1;
        g.nkeys = 1;
        g.chunk = (int)(n > 0 ? n : 1);
        g.nchunks = 1;
        KMG_TRY(c->kmers.ensure(sizeof(uint32_t) * (size_t)(n * g.pmax > 0 ? n * g.pmax : 1)));
        {
          StageTimer t(c, ST_EXTRACT);
          KMG_HIP(launch_extract(g, pkd, c->kmers.as<uint32_t>(), c->stream));
        }
        KMG_TRY(upload_wtab(c, w));
        if (p->normalize) {
          KMG_TRY(diag_hamming(c, g, pkd));
          o.normalize = 1;
          o.diagv = c->diagv.as<double>();
          o.dsq = c->dsq.as<double>();
        }
        return each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
          for (int64_t r = r0; r < r1; r += 65535) {  // grid.y <= 65535 rows per launch
            OutSpec os = oq;
            os.out = (char *)oq.out + (size_t)(r - r0) * oq.ld * dtype_size(dt);
            hipError_t e = launch_gram_hamming(g, c->kmers.as<uint32_t>(), r, std::min(r1, r + 65535),
                                               c->wtab.as<int64_t>(), os, c->stream);
            if (e != hipSuccess) return e;
          }
          return hipSuccess;
        });
      }
      if (use_pairs) {
        // exact k-mer index over the mismatch window (kernels.py:171), then the pair table
        // assembled from it
        g.copies = 1;
        g.nkeys = (uint32_t)pow4(k);
        choose_chunks(g, pair_chunk(n, g.pmax, k, c->tune.mm_chunk));
        o.tri = tri_esz > 0 && g.nchunks > 1;
        note_plan(1024);
        KMG_TRY(build_index(c, g, pkd, d_codes, d_lens, ldc));
        PairGeom pg{};
        pg.k = k;
        pg.nchunks = g.nchunks;
        pg.chunk = g.chunk;
        pg.nkeys2 = (uint32_t)pow4(k - 2);
        for (int pp = 0; pp < k; ++pp)
          for (int qq = pp + 1; qq < k; ++qq) pg.pq[pg.npairs++] = (uint16_t)(pp | (qq << 8));
        const int64_t nrec = pg.nrec();
        const int64_t nlines = pair_lines_bound(pg, n * g.pmax);
        if (nlines * 128 >= 0xFFFFFFF0LL)
          return fail(KMG_EUNSUPPORTED, "pair table too large for 32-bit offsets");
        KMG_TRY(c->pr_summary.ensure(sizeof(uint32_t) * 8 * (size_t)nrec));
        KMG_TRY(c->pr_rtot.ensure(sizeof(uint32_t) * (size_t)(nrec + 1)));
        KMG_TRY(c->pr_rbase.ensure(sizeof(uint32_t) * (size_t)(nrec + 1)));
        KMG_TRY(c->pr_cursor.ensure(sizeof(uint32_t) * (size_t)(nrec + 1)));
        KMG_TRY(c->partials.ensure(sizeof(uint32_t) * scan_partials_words(nrec)));
        KMG_TRY(c->pr_lines.ensure((size_t)nlines * 128));
        {
          StageTimer t(c, ST_SLOTS);
          KMG_HIP(launch_pair_count(pg, c->off.as<uint32_t>(), c->pr_summary.as<uint32_t>(),
                                    c->pr_rtot.as<uint32_t>(), c->stream));
          KMG_HIP(launch_scan(c->pr_rtot.as<uint32_t>(), c->pr_rbase.as<uint32_t>(),
                              c->pr_cursor.as<uint32_t>(), nrec, c->partials.as<uint32_t>(),
                              c->stream));
          KMG_HIP(launch_pair_pack(pg, c->off.as<uint32_t>(), c->ent.as<uint16_t>(),
                                   c->pr_rbase.as<uint32_t>(), c->pr_summary.as<uint32_t>(),
                                   c->pr_lines.as<uint4>(), c->stream));
        }
        if (p->normalize || dt == KMG_U8) {  // (8-bit slabs: the unpack's K_ii)
          KMG_TRY(upload_wtab(c, w));
          KMG_TRY(diag_hamming(c, g, pkd));
          if (p->normalize) {
            o.normalize = 1;
            o.diagv = c->diagv.as<double>();
            o.dsq = c->dsq.as<double>();
          }
        }
        KMG_TRY(each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
          return launch_gram_mismatch1_pairs(pg, g, pkd, c->pr_summary.as<uint32_t>(),
                                             c->pr_lines.as<uint4>(), nlines,
                                             c->off.as<uint32_t>(), c->ent.as<uint16_t>(), r0,
                                             r1, (int)w[0], (int)w[1], (int)w[2], oq, c->stream);
        }, true));
        return mirror();
      }
      if (use_nb) {
        // exact k-mer index over the mismatch window (kernels.py:171), then every (chunk,
        // k-mer)'s neighbourhood list assembled from it (kmg_nbhd.hip)
        g.copies = 1;
        g.nkeys = (uint32_t)pow4(k);
        // gc: the column sequences the lists are built over (all n, or a column block's)
        IndexGeom gc = g;
        gc.n = ncols;
        const int nbt = c->tune.nb_threads ? c->tune.nb_threads : colblk ? 512 : 1024;
        const int lds512 = c->tune.nb_lds512 ? c->tune.nb_lds512 : colblk ? 53 : 40;
        // the sorted fill (packed segment 2) where each list is read often enough to repay its
        // sort: reads a list = rows read x windows a row / 4^k (x (nch + 1) / (2 nch) for a
        // square by its block triangle); else 16-bit lists
        bool sorted = c->tune.nb_fill == 1;
        if (c->tune.nb_fill == 0) {
          int64_t rows_read = 0;
          for (const RowRange &r : ranges) rows_read += r.row1 - r.row0;
          const int ch = nb_chunk(ncols, g.pmax, k, (int)pkd.ldp, c->tune.mm_chunk, tri_esz, nbt,
                                  true, lds512);
          const int64_t nch = (ncols + ch - 1) / ch;
          const double f = (tri_esz > 0 && nch > 1) ? (double)(nch + 1) / (2.0 * nch) : 1.0;
          sorted = (double)rows_read * g.pmax / (double)pow4(k) * f >= (double)c->tune.nb_pack_reads;
        }
        choose_chunks(gc, nb_chunk(ncols, g.pmax, k, (int)pkd.ldp, c->tune.mm_chunk, tri_esz, nbt,
                                   sorted, lds512));
        g.chunk = gc.chunk;
        g.nchunks = gc.nchunks;
        o.tri = tri_esz > 0 && g.nchunks > 1;
        note_plan(nbt);
        c->plan[5] = (sorted && nb_sorted_cap(k, g.pmax, g.chunk) > 0) ? 1 : 0;
        if (nb_gram_lds(gc, pkd) > 160 * 1024)  // (very long windows: the row table alone)
          return fail(KMG_EUNSUPPORTED, "neighbourhood lists: %zu B of LDS at %d windows a row "
                      "(KMG_MM_FORM=1 or 2: the slot / pair tables)", nb_gram_lds(gc, pkd), g.pmax);
        if (!colblk) {
          KMG_TRY(build_index(c, gc, pkd, d_codes, d_lens, ldc));
        } else {  // every row's record, then the index over the block's (already packed) ones
          {
            StageTimer t(c, ST_PACK);
            KMG_HIP(launch_pack(d_codes, d_lens, n, ldc, g.window, c->packed.as<uint32_t>(), c->stream));
          }
          const Packed pkc{pkd.w + cseq0 * pkd.ldp, pkd.ldp, pkd.cw};
          KMG_TRY(build_index(c, gc, pkc));
        }
        const int64_t nbins = gc.nbins();
        const int64_t bound = nb_list_entries_bound(k, ncols * (int64_t)g.pmax, nbins);
        if (bound / 8 + nbins >= 0xFFFFFFF0LL)
          return fail(KMG_EUNSUPPORTED, "neighbourhood lists: more than 2^32 pieces");
        KMG_TRY(c->pr_rtot.ensure(sizeof(uint32_t) * (size_t)(nbins + 1)));
        KMG_TRY(c->pr_rbase.ensure(sizeof(uint32_t) * (size_t)(nbins + 1)));
        KMG_TRY(c->pr_cursor.ensure(sizeof(uint32_t) * (size_t)(nbins + 1)));
        KMG_TRY(c->partials.ensure(sizeof(uint32_t) * scan_partials_words(nbins)));
        KMG_TRY(c->nb_seg.ensure(sizeof(uint2) * (size_t)nbins));
        KMG_TRY(c->nb_use.ensure(sizeof(uint2) * (size_t)nbins));
        KMG_TRY(c->nb_lines.ensure(sizeof(uint16_t) * (size_t)(bound + 8)));
        {
          StageTimer t(c, ST_LISTS);  // list sizes and starts
          KMG_HIP(launch_nb_count(gc, c->off.as<uint32_t>(), c->pr_rtot.as<uint32_t>(),
                                  c->pr_rbase.as<uint32_t>(), c->pr_cursor.as<uint32_t>(),
                                  c->nb_seg.as<uint2>(), c->partials.as<uint32_t>(), c->stream));
        }
        {
          StageTimer t(c, ST_NBFILL);  // the lists themselves
          const hipError_t e = launch_nb_fill(gc, c->off.as<uint32_t>(), c->ent.as<uint16_t>(),
                                              c->pr_rbase.as<uint32_t>(), c->nb_seg.as<uint2>(),
                                              c->nb_use.as<uint2>(), c->nb_lines.as<uint16_t>(),
                                              c->stream,
                                              c->tune.nb_fill != 0 ? c->tune.nb_fill : sorted ? 0 : 5,
                                              c->tune.nb_fill_threads);
          if (e == hipErrorInvalidValue && c->tune.nb_fill == 1)
            return fail(KMG_EUNSUPPORTED, "KMG_NB_FILL=1: no sorted fill at k=%d, chunk %d", k, g.chunk);
          KMG_HIP(e);
        }
        if (c->tune.check) {
          // the Gram kernel reads table[start + rel] for rel below the list's nbuse counts
          // without a bound: a fill that left them inconsistent is reported here, before any
          // read past a list (round 5's r05ah fault)
          KMG_TRY(c->chk.ensure(2 * sizeof(uint32_t)));
          if (c->tune.check == 2)  // test hook: a fill that left every list's counts stale
            KMG_HIP(hipMemsetD32Async((hipDeviceptr_t)c->nb_use.p, 0x7FFFFFFFu, 2 * (size_t)nbins,
                                      c->stream));
          KMG_HIP(hipMemsetD32Async((hipDeviceptr_t)c->chk.p, 0u, 1, c->stream));
          KMG_HIP(hipMemsetD32Async((hipDeviceptr_t)(c->chk.as<uint32_t>() + 1), 0xFFFFFFFFu, 1, c->stream));
          KMG_HIP(launch_nb_check(nbins, c->pr_rbase.as<uint32_t>(), c->nb_seg.as<uint2>(),
                                  c->nb_use.as<uint2>(), (uint64_t)(bound + 8) / 8,
                                  c->chk.as<uint32_t>(), c->stream));
          uint32_t res[2] = {0u, 0u};
          KMG_HIP(hipMemcpyAsync(res, c->chk.p, sizeof(res), hipMemcpyDeviceToHost, c->stream));
          KMG_HIP(hipStreamSynchronize(c->stream));
          if (res[0])
            return fail(KMG_EINTERNAL, "KMG_CHECK: neighbourhood list %u (chunk %u, k-mer %u) has "
                        "inconsistent metadata after the fill (KMG_NB_FILL=%d)", res[1],
                        res[1] >> (2 * k), res[1] & (uint32_t)(pow4(k) - 1), c->tune.nb_fill);
        }
        if (p->normalize || dt == KMG_U8) {  // (8-bit slabs: the unpack's K_ii)
          KMG_TRY(upload_wtab(c, w));
          KMG_TRY(diag_hamming(c, g, pkd));
          if (p->normalize) {
            o.normalize = 1;
            o.diagv = c->diagv.as<double>();
            o.dsq = c->dsq.as<double>();
          }
        }
        o.col_seq0 = cseq0;
        auto nb_launch = [&](int64_t r0, int64_t r1, const OutSpec &oq) {
          return launch_gram_mismatch1_nb(gc, pkd, c->pr_rbase.as<uint32_t>(), c->nb_seg.as<uint2>(),
                                          c->nb_use.as<uint2>(), c->nb_lines.as<uint4>(), r0, r1,
                                          (int)w[0], (int)w[1], (int)w[2], oq, c->stream, nbt,
                                          c->tune.nb_unroll ? c->tune.nb_unroll
                                                            : (o.tri || c->plan[5] ? 4 : 8));
        };
        KMG_TRY(each_range(c, ranges, o, after, nb_launch, true));
        return mirror();
      }
      // gi: the geometry of the columns (the index and the chunking); g keeps all n rows (the
      // diagonal).  A spectrum column block indexes only its own ncols sequences.
      IndexGeom gi = g;
      if (exact) {
        g.copies = 1;
        g.nkeys = (uint32_t)pow4(k);
        gi = g;
        gi.n = ncols;
        // a column block of up to KMG_SP_CB_CHUNK columns is ONE chunk: N=100000, the G=4
        // block (25000 columns) 2.06 -> 1.73 ms against two chunks of 12504
        // (profiles/r06k_colblock_rows_g24.jsonl); wider blocks and full rows keep
        // KMG_SP_CHUNK (a 25000-column chunk's index slice outgrows the XCD's L2: full K
        // 6.3 -> 7.4 ms, profiles/r06k_colblock_chunk_g2.jsonl)
        const int maxc = colblk && ncols <= c->tune.sp_cb_chunk ? c->tune.sp_cb_chunk : c->tune.sp_chunk;
        choose_chunks(gi, std::min(65536, maxc));
        g.chunk = gi.chunk;
        g.nchunks = gi.nchunks;
      } else {
        g.copies = k;
        g.rot = 1;
        g.nkeys = (uint32_t)pow4(k);
        choose_chunks(g, slot_chunk(n, g.pmax, k, (int)pkd.ldp, c->tune.mm_chunk, tri_esz));
        o.tri = use_slots && tri_esz > 0 && g.nchunks > 1;
        gi = g;
      }
      note_plan(1024);
      if (!colblk) {
        KMG_TRY(build_index(c, gi, pkd, d_codes, d_lens, ldc));
      } else {  // every row's record, then the index over the block's (already packed) ones
        {
          StageTimer t(c, ST_PACK);
          KMG_HIP(launch_pack(d_codes, d_lens, n, ldc, g.window, c->packed.as<uint32_t>(), c->stream));
        }
        const Packed pkc{pkd.w + cseq0 * pkd.ldp, pkd.ldp, pkd.cw};
        KMG_TRY(build_index(c, gi, pkc));
        o.col_seq0 = cseq0;
      }
      if (use_slots) {
        KMG_TRY(c->slots.ensure((size_t)(g.nbins() >> 2) * KMG_SLOT_BYTES));
        StageTimer t(c, ST_SLOTS);
        KMG_HIP(launch_slot_pack(g, c->off.as<uint32_t>(), c->ent.as<uint16_t>(),
                                 c->slots.as<uint4>(), c->stream));
      }
      if (p->normalize || dt == KMG_U8) {  // (8-bit slabs: the unpack's K_ii)
        KMG_TRY(upload_wtab(c, w));
        KMG_TRY(diag_hamming(c, g, pkd));
        if (p->normalize) {
          o.normalize = 1;
          o.diagv = c->diagv.as<double>();
          o.dsq = c->dsq.as<double>();
        }
      }
      KMG_TRY(each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
        return exact ? launch_gram_spectrum(gi, pkd, c->off.as<uint32_t>(), c->ent.as<uint16_t>(),
                                            r0, r1, oq, c->stream, c->tune.sp_store,
                                            c->tune.sp_order, c->tune.sp_rows)
                     : launch_gram_mismatch1_slots(g, pkd, c->slots.as<uint4>(),
                                                   c->off.as<uint32_t>(), c->ent.as<uint16_t>(),
                                                   r0, r1, (int)w[0], (int)w[1], (int)w[2], oq,
                                                   c->stream);
      }, true));
      return mirror();
    }
    case KMG_WD:
    case KMG_WDS: {
      if (p->d < 0 || p->d > KMG_MAX_COEF) return fail(KMG_EUNSUPPORTED, "d outside [0,64]");
      if (p->kind == KMG_WDS && p->S < 0) return fail(KMG_EINVAL, "S < 0");
      if (p->kind == KMG_WDS && p->S >= KMG_MAX_COEF)
        return fail(KMG_EUNSUPPORTED, "S outside [0,%d]", KMG_MAX_COEF - 1);
      if (dt == KMG_I32) return fail(KMG_EINVAL, "WD/WDS produce float64 values");
      if (p->span < 0) return fail(KMG_EINVAL, "span < 0");
      if (p->span > 0) {
        // the kernels count positions below min(len_x, len_y, span): a span past a row's
        // end would miss the reference's clipped-slice matches (kernels.py:75-80, 127-134)
        uint32_t mc = 0, ml = 0;
        KMG_TRY(row_stats(c, d_codes, d_lens, n, ldc, mc, ml));
        const int64_t need = (int64_t)p->span + (p->kind == KMG_WDS ? p->S : 0);
        if (n > 0 && need > (int64_t)ml)
          return fail(KMG_EUNSUPPORTED, "WD/WDS: span %d%s exceeds the shortest row (%u); pad the rows",
                      p->span, p->kind == KMG_WDS ? " + S" : "", ml);
      }
      SeqSpec q{d_codes, d_lens, n, ldc, maxlen};
      Packed pkd{nullptr, 0, 0};
      const bool packed_wd = p->kind == KMG_WD && c->tune.wd_form == 0 && maxlen <= 256 &&
                             p->span <= 256;
      if (packed_wd) {  // 2-bit records: 7 words a pair at L = 101 (kmg_pairwise.hip)
        const int cw = packed_cw(ldc), mw = packed_mw(ldc);
        KMG_TRY(c->packed.ensure(sizeof(uint32_t) * (size_t)std::max<int64_t>(1, n) * (cw + mw)));
        pkd = Packed{c->packed.as<uint32_t>(), (int64_t)(cw + mw), cw};
        StageTimer t(c, ST_PACK);
        KMG_HIP(launch_pack(d_codes, d_lens, n, ldc, 0, c->packed.as<uint32_t>(), c->stream));
      }
      bool unsupported = false;
      // past the specialised kernels' shift / length limits (WDS S > 15, or S > 7 above 128
      // symbols; WD / WDS above 256): the generic per-pair kernel (kmg_generic.hip), the
      // coefficients in a device buffer
      const bool sq = ranges.size() == 1 && ranges[0].row0 == 0 && ranges[0].row1 == n &&
                      ranges[0].col_lo == 0;
      auto generic = [&](int64_t r0, int64_t r1, const OutSpec &oq) -> hipError_t {
        if (p->kind == KMG_WD && p->span > 0) return hipErrorNotSupported;
        if (!c->gcoef.p) {
          if (c->gcoef.ensure(2 * KMG_MAX_COEF * sizeof(double)) != KMG_OK) return hipErrorOutOfMemory;
        }
        double h[2 * KMG_MAX_COEF];
        memcpy(h, p->coef_a, sizeof(double) * KMG_MAX_COEF);
        if (p->kind == KMG_WD) {
          for (int t = 0; t < KMG_MAX_COEF; ++t) h[KMG_MAX_COEF + t] = 0.0;
          h[KMG_MAX_COEF] = 0.5;  // delta_0: a WD match adds 0.5 * 2 = 1.0 exactly
        } else {
          memcpy(h + KMG_MAX_COEF, p->coef_b, sizeof(double) * KMG_MAX_COEF);
        }
        hipError_t e = hipMemcpyAsync(c->gcoef.p, h, sizeof(h), hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // pageable source
        if (e != hipSuccess) return e;
        const double *ca = c->gcoef.as<double>();
        return launch_gram_wds_generic(q, r0, r1, p->d, p->kind == KMG_WD ? 0 : p->S, p->span, ca,
                                       ca + KMG_MAX_COEF, p->kind == KMG_WD ? 1 : 0,
                                       sq && r0 == 0 && r1 == n ? 1 : 0, oq, c->stream);
      };
      const int r = each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
        hipError_t e = p->kind == KMG_WD
                           ? (packed_wd ? launch_gram_wd_packed(q, pkd, r0, r1, p->d, p->span,
                                                                p->coef_a, oq, c->stream)
                                        : launch_gram_wd(q, r0, r1, p->d, p->span, p->coef_a, oq,
                                                         c->stream))
                           : launch_gram_wds(q, r0, r1, p->d, p->S, p->span, p->coef_a,
                                             p->coef_b, oq, c->stream);
        if (e == hipErrorNotSupported) e = generic(r0, r1, oq);
        if (e == hipErrorNotSupported) {
          unsupported = true;
          return hipSuccess;
        }
        return e;
      });
      if (unsupported)
        return fail(KMG_EUNSUPPORTED, "WD/WDS: sequence length %d / shift %d not supported",
                    maxlen, p->S);
      return r;
    }
    case KMG_SUBSTRING: {
      if (p->k < 0) return fail(KMG_EINVAL, "k < 0");
      if (dt == KMG_I32) return fail(KMG_EINVAL, "SS produces float64 values");
      // la_mode KMG_MODE_SS_B: B_k(lbda, k, x, y) (kernels.py:322-342) instead of K_k
      if (p->la_mode != KMG_MODE_REFERENCE && p->la_mode != KMG_MODE_SS_B)
        return fail(KMG_EINVAL, "SS: unknown la_mode %d", p->la_mode);
      const int bmode = p->la_mode == KMG_MODE_SS_B ? 1 : 0;
      // k <= 33 at sequence lengths <= 127 (grouped sweep), k <= 16 at any length (strips)
      SeqSpec q{d_codes, d_lens, n, ldc, maxlen};
      // one range covering the whole matrix: upper triangle + mirror (kernels.py:378-381)
      const int mirror = (ranges.size() == 1 && ranges[0].row0 == 0 && ranges[0].row1 == n) ? 1 : 0;
      bool unsupported = false;
      const int r = each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
        hipError_t e = launch_gram_ss(q, r0, r1, p->k, p->lambda, p->lambda2, mirror, oq, c->stream,
                                      c->tune.ss_lpp, bmode);
        if (e == hipErrorNotSupported) {
          unsupported = true;
          return hipSuccess;
        }
        return e;
      });
      if (unsupported)
        return fail(KMG_EUNSUPPORTED, "SS: k = %d with sequences of length %d (k <= 33 up to "
                    "length 127, k <= 16 beyond; B_k: k <= 32 up to length 127)", p->k, maxlen);
      return r;
    }
    case KMG_LOCALALIGN: {
      if (dt == KMG_I32) return fail(KMG_EINVAL, "LA produces float64 values");
      if (p->la_mode == KMG_LA_INTENDED) {
        // the recurrence the reference means (kernels.py:226-270 with its aliasing, loop
        // bounds and gap signs fixed; gram_la_kernel): parity unpinned
        if (!(p->la_beta > 0.0)) return fail(KMG_EINVAL, "LA: beta must be > 0");
        // (no length check here: the launch picks the grouped sweep up to length 127, the
        // strip kernel with 4..1 pairs a block up to ~5100, and reports longer as unsupported)
        {  // the substitution matrix S covers A, C, G, T only (kernels.py:223)
          uint32_t mc = 0, ml = 0;
          KMG_TRY(row_stats(c, d_codes, d_lens, n, ldc, mc, ml));
          if (mc > 3) return fail(KMG_EINVAL, "LA: symbol other than A/C/G/T (code %u)", mc);
        }
        SeqSpec q{d_codes, d_lens, n, ldc, maxlen};
        bool unsupported = false;
        const int r = each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
          const bool full = r0 == 0 && r1 == n;  // square: upper triangle + mirror
          for (int64_t a = r0; a < r1; a += 65535) {
            OutSpec os = oq;
            os.out = (char *)oq.out + (size_t)(a - r0) * oq.ld * dtype_size(dt);
            const int64_t b = std::min(r1, a + 65535);
            hipError_t e = launch_gram_la(q, a, b, p->la_e, p->la_d, p->la_beta, p->smith,
                                          full && b - a == n ? 1 : 0, os, c->stream,
                                          c->tune.la_lpp);
            if (e == hipErrorNotSupported) {
              unsupported = true;
              return hipSuccess;
            }
            if (e != hipSuccess) return e;
          }
          return hipSuccess;
        });
        if (unsupported)
          return fail(KMG_EUNSUPPORTED, "LA: sequences of length %d (the boundary rows of a "
                      "64-row strip must fit the 160 KB LDS: length <= ~5100)", maxlen);
        return r;
      }
      if (p->la_mode != KMG_LA_REFERENCE) return fail(KMG_EINVAL, "LA: unknown la_mode");
      // The reference aliases M,X,Y,X2,Y2 to one array and never writes cell
      // [n_x, n_y] (kernels.py:238-240, 262-264): every entry is log(1+0)/beta = 0.
      return each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
        if (r1 <= r0 || n == 0) return hipSuccess;
        return hipMemset2DAsync(oq.out, (size_t)ld * dtype_size(dt), 0, (size_t)n * dtype_size(dt),
                                (size_t)(r1 - r0), c->stream);
      });
    }
    case KMG_GAPPY: {
      const int W = p->window > 0 ? p->window : 101;
      // windows read x[0 : W) of every row (kernels.py:430): narrower rows would read into
      // the next row (padding codes >= 4 inside a row are skipped)
      if (n > 0 && ldc < W)
        return fail(KMG_EINVAL, "gappy: code rows (%lld) shorter than the window %d",
                    (long long)ldc, W);
      if (p->la_mode == KMG_MODE_INTENDED) {
        if (p->k < 1 || p->k > 15 || p->g < 0 || p->g >= p->k || p->k - p->g > 8)
          return fail(KMG_EUNSUPPORTED, "intended gappy: need 1 <= k <= 15, 0 <= g < k, k-g <= 8");
        if (dt == KMG_I32 && p->normalize) return fail(KMG_EINVAL, "normalised GP is float64");
        return gram_gappy_intended(c, p->k, p->g, W, d_codes, n, ldc, ranges, o,
                                   p->normalize != 0, after);
      }
      if (!(p->k == 1 && p->g == 0))
        return fail(KMG_EUNSUPPORTED, "gappy kernel defined only for k=1, g=0");
      if (dt == KMG_I32) return fail(KMG_EINVAL, "GP produces float64 values");
      SeqSpec q{d_codes, d_lens, n, ldc, maxlen};
      KMG_TRY(c->diagv.ensure(sizeof(double) * (size_t)(n > 0 ? n : 1)));
      KMG_TRY(c->dsq.ensure(sizeof(double) * (size_t)(n > 0 ? n : 1)));
      o.normalize = 1;
      o.diagv = c->diagv.as<double>();
      o.dsq = c->dsq.as<double>();
      return each_range(c, ranges, o, after, [&](int64_t r0, int64_t r1, const OutSpec &oq) {
        return launch_gram_gappy1(q, r0, r1, W, oq, c->diagv.as<double>(), c->dsq.as<double>(),
                                  c->stream);
      });
    }
    default:
      return fail(KMG_EINVAL, "unknown kernel kind %d", p->kind);
  }
}

}  // namespace

// =================================================================== C ABI
extern "C" {

int kmg_version(void) { return KMG_ABI_VERSION; }

const char *kmg_last_error(void) { return g_err.c_str(); }

int kmg_device_count(int *n) {
  if (!n) return fail(KMG_EINVAL, "n is NULL");
  int cnt = 0;
  hipError_t e = hipGetDeviceCount(&cnt);
  if (e != hipSuccess) cnt = 0;
  *n = cnt;
  return KMG_OK;
}

int kmg_create(kmg_ctx **out, int device_id) {
  if (!out) return fail(KMG_EINVAL, "ctx is NULL");
  *out = nullptr;
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0)
    return fail(KMG_ENODEV, "no HIP device visible");
  if (device_id < 0 || device_id >= cnt)
    return fail(KMG_EINVAL, "device %d outside [0,%d)", device_id, cnt);
  KMG_HIP(hipSetDevice(device_id));
  kmg_ctx *c = new kmg_ctx();
  c->device = device_id;
  read_tuning(c->tune);
  // LDS a workgroup may take: the largest of what the runtime reports per block, per block
  // opt-in and per CU (runtimes differ in which one carries gfx950's 160 KB)
  for (hipDeviceAttribute_t a : {hipDeviceAttributeMaxSharedMemoryPerBlock, hipDeviceAttributeSharedMemPerBlockOptin,
                                 hipDeviceAttributeMaxSharedMemoryPerMultiprocessor}) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, a, device_id) == hipSuccess) c->lds_max = std::max(c->lds_max, v);
  }
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(KMG_EHIP, "hipStreamCreate: %s", hipGetErrorString(e));
  }
  *out = c;
  return KMG_OK;
}

int kmg_destroy(kmg_ctx *c) {
  if (!c) return KMG_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->blas) rocblas_destroy_handle(c->blas);
  DevBuf *bufs[] = {&c->kmers, &c->partials, &c->tmp, &c->esc, &c->esc_all, &c->esc_cnt,
                    &c->off,   &c->ent,    &c->diagv, &c->dsq,     &c->wtab,     &c->h_codes,
                    &c->h_lens, &c->h_out, &c->feat,    &c->masks,  &c->slots, &c->packed,
                    &c->pr_summary, &c->pr_rtot, &c->pr_rbase, &c->pr_cursor, &c->pr_lines,
                    &c->hcnt,  &c->hstart, &c->cmb_k, &c->cmb_ptrs, &c->cmb_vec,
                    &c->cmb_out, &c->cmb_tmp, &c->sv_mat, &c->sv_vec, &c->sv_info, &c->sv_inv, &c->sv_panel,
                    &c->tri_stage, &c->tri_scratch, &c->dense_tiles, &c->ovf, &c->slabs,
                    &c->gcoef, &c->feat32, &c->k32, &c->ft_cols,
                    &c->nb_seg, &c->nb_use, &c->nb_lines, &c->chk, &c->cb_scratch};
  for (DevBuf *b : bufs) b->release();
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
  if (c->ev_sync) (void)hipEventDestroy(c->ev_sync);
  if (c->unpack_stream) (void)hipStreamDestroy(c->unpack_stream);
  for (hipEvent_t e : c->ev_gath)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_tri)
    if (e) (void)hipEventDestroy(e);
  if (c->d2h_stream) (void)hipStreamDestroy(c->d2h_stream);
  if (c->chol_stream) (void)hipStreamDestroy(c->chol_stream);
  for (hipEvent_t e : c->ev_chol)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_slab)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_out)
    if (e) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return KMG_OK;
}

int kmg_gram(kmg_ctx *c, const kmg_params *p, const uint8_t *codes, const int32_t *lens,
             int64_t n, int64_t ldc, int32_t out_dtype, void *out, int64_t ld_out) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_TRY(check_params(p, n, ldc, out_dtype));
  if (n > 0 && (!codes || !lens || !out)) return fail(KMG_EINVAL, "NULL buffer");
  if (n > 0 && ld_out < n) return fail(KMG_EINVAL, "ld_out < n");
  KMG_HIP(hipSetDevice(c->device));
  if (n == 0) return KMG_OK;
  int maxlen = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (lens[i] < 0 || lens[i] > ldc) return fail(KMG_EINVAL, "lens[%lld] outside [0,ldc]", (long long)i);
    if (lens[i] > maxlen) maxlen = lens[i];
  }
  if (p->kind == KMG_MISMATCH) {
    const int W = p->window > 0 ? p->window : 101;
    for (int64_t i = 0; i < n; ++i)
      if (lens[i] < W) return fail(KMG_EINVAL, "mismatch kernel needs sequences of length >= %d", W);
  }
  const size_t esz = dtype_size(out_dtype);
  const int64_t ldd = (n + 3) & ~3LL;
  KMG_TRY(c->h_codes.ensure((size_t)n * ldc));
  KMG_TRY(c->h_lens.ensure(sizeof(int32_t) * (size_t)n));
  KMG_TRY(c->h_out.ensure(esz * (size_t)n * ldd));
  KMG_HIP(hipMemcpyAsync(c->h_codes.p, codes, (size_t)n * ldc, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipMemcpyAsync(c->h_lens.p, lens, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  KMG_TRY(gram_device(c, p, c->h_codes.as<uint8_t>(), c->h_lens.as<int32_t>(), maxlen, n, ldc,
                      {RowRange{0, n, c->h_out.p}}, out_dtype, ldd));
  KMG_HIP(hipMemcpy2DAsync(out, (size_t)ld_out * esz, c->h_out.p, (size_t)ldd * esz,
                           (size_t)n * esz, (size_t)n, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

// kmg_features (cols: uint32 base-4 codes) and kmg_features_sym (cols: 16 symbol bytes each;
// flags bit 0: numpy's broadcast of short k-mers, get_phi_km on rows shorter than the window)
static int features_impl(kmg_ctx *c, const kmg_params *p, const uint8_t *codes, const int32_t *lens,
                         int64_t n, int64_t ldc, const void *cols, bool sym, int32_t flags,
                         int64_t ncols, double *out, int64_t ld_out) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  if (!p) return fail(KMG_EINVAL, "params is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  if (n < 0 || ncols < 0 || ldc < 0) return fail(KMG_EINVAL, "negative size");
  if (n == 0 || ncols == 0) return KMG_OK;
  if (!codes || !lens || !cols || !out) return fail(KMG_EINVAL, "NULL buffer");
  if (ld_out < ncols) return fail(KMG_EINVAL, "ld_out < ncols");
  int k = p->k, m = 0, window = 0, binary = 0;
  const int bcast = sym && (flags & KMG_FEATURES_BCAST) ? 1 : 0;
  switch (p->kind) {
    case KMG_SPECTRUM: break;  // get_phi_u: windows range(len(x) - k + 1)
    case KMG_MISMATCH:         // get_phi_km: windows range(101 - k + 1)
      m = p->m;
      window = p->window > 0 ? p->window : 101;
      if (m < 0) return fail(KMG_EINVAL, "m < 0");
      break;
    case KMG_GAPPY:  // gappy_k (k = 1, g = 0): letters of x[0:101]
      if (sym) return fail(KMG_EUNSUPPORTED, "symbol columns: spectrum or mismatch only");
      if (!(p->k == 1 && p->g == 0)) return fail(KMG_EUNSUPPORTED, "gappy features: k=1, g=0 only");
      window = p->window > 0 ? p->window : 101;
      binary = 1;
      break;
    default:
      return fail(KMG_EUNSUPPORTED, "features: spectrum, mismatch or gappy only");
  }
  if (k < 1 || k > 16) return fail(KMG_EUNSUPPORTED, "features: 1 <= k <= 16 (k = %d)", k);
  for (int64_t i = 0; i < n; ++i) {
    if (lens[i] < 0 || lens[i] > ldc) return fail(KMG_EINVAL, "lens[%lld] outside [0,ldc]", (long long)i);
    if (p->kind == KMG_MISMATCH && lens[i] < window && !bcast)
      return fail(KMG_EINVAL, "mismatch features need sequences of length >= %d", window);
    if (bcast && p->kind == KMG_MISMATCH && lens[i] < window) {
      // windows of ln = min(k, len - a) symbols, a < window - k + 1: numpy broadcasts ln = 1
      // (and ln = 0 against a 1-letter beta); any other short window raises in the reference
      const int first_short = std::max(0, (int)lens[i] - k + 1);
      for (int a2 = first_short; a2 < window - k + 1; ++a2) {
        const int ln = std::max(0, std::min(k, (int)lens[i] - a2));
        if (ln != k && ln != 1 && !(ln == 0 && k == 1))
          return fail(KMG_EINVAL, "features: a %d-symbol window of row %lld does not broadcast "
                      "against a %d-mer", ln, (long long)i, k);
      }
    }
    if ((window > 0 ? std::min<int64_t>(window, lens[i]) : lens[i]) - k + 1 > KMG_FEAT_MAXW)
      return fail(KMG_EUNSUPPORTED, "features: more than %d windows per sequence", KMG_FEAT_MAXW);
  }
  KMG_HIP(hipSetDevice(c->device));
  // rows per launch: the device output slab stays <= 1 GiB (and grid.y <= 65535)
  const int64_t slab = std::max<int64_t>(1, std::min<int64_t>({n, 65535, (1LL << 27) / ncols}));
  KMG_TRY(c->h_codes.ensure((size_t)n * std::max<int64_t>(1, ldc)));
  KMG_TRY(c->h_lens.ensure(sizeof(int32_t) * (size_t)n));
  const size_t csz = sym ? 16 : sizeof(uint32_t);
  KMG_TRY(c->ft_cols.ensure(csz * (size_t)ncols));
  KMG_TRY(c->h_out.ensure(sizeof(double) * (size_t)slab * ncols));
  KMG_HIP(hipMemcpyAsync(c->h_codes.p, codes, (size_t)n * ldc, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipMemcpyAsync(c->h_lens.p, lens, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipMemcpyAsync(c->ft_cols.p, cols, csz * ncols, hipMemcpyHostToDevice, c->stream));
  for (int64_t r0 = 0; r0 < n; r0 += slab) {
    const int64_t rows = std::min(slab, n - r0);
    {
      StageTimer t(c, ST_FEATURES);
      if (sym)
        KMG_HIP(launch_features_sym(c->h_codes.as<uint8_t>(), c->h_lens.as<int32_t>(), ldc, r0, rows,
                                    k, m, window, bcast, c->ft_cols.as<uint4>(), ncols,
                                    c->h_out.as<double>(), ncols, c->stream));
      else
        KMG_HIP(launch_features(c->h_codes.as<uint8_t>(), c->h_lens.as<int32_t>(), ldc, r0, rows, k,
                                m, window, binary, c->ft_cols.as<uint32_t>(), ncols,
                                c->h_out.as<double>(), ncols, c->stream));
    }
    KMG_HIP(hipMemcpy2DAsync(out + (size_t)r0 * ld_out, (size_t)ld_out * sizeof(double), c->h_out.p,
                             (size_t)ncols * sizeof(double), (size_t)ncols * sizeof(double),
                             (size_t)rows, hipMemcpyDeviceToHost, c->stream));
    // (the next slab reuses the device buffer: hipMemcpy2DAsync to pageable memory returns
    // once the copy has been staged, and the stream orders the next launch behind it)
  }
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

int kmg_features(kmg_ctx *c, const kmg_params *p, const uint8_t *codes, const int32_t *lens,
                 int64_t n, int64_t ldc, const uint32_t *cols, int64_t ncols, double *out,
                 int64_t ld_out) {
  return features_impl(c, p, codes, lens, n, ldc, cols, false, 0, ncols, out, ld_out);
}

int kmg_features_sym(kmg_ctx *c, const kmg_params *p, const uint8_t *codes, const int32_t *lens,
                     int64_t n, int64_t ldc, const uint8_t *cols, int64_t ncols, int32_t flags,
                     double *out, int64_t ld_out) {
  return features_impl(c, p, codes, lens, n, ldc, cols, true, flags, ncols, out, ld_out);
}

int kmg_gram_device(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes,
                    const int32_t *d_lens, int64_t n, int64_t ldc, int64_t row0, int64_t row1,
                    int32_t out_dtype, void *d_out, int64_t ld_out) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_TRY(check_params(p, n, ldc, out_dtype));
  KMG_HIP(hipSetDevice(c->device));
  // device-resident path: sequence lengths are device data; the caller promises
  // max(lens) <= ldc (checked in the host path).  maxlen = ldc bounds every kernel.
  return gram_device(c, p, d_codes, d_lens, (int)ldc, n, ldc, {RowRange{row0, row1, d_out}},
                     out_dtype, ld_out);
}

int kmg_gram_device_cols(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes,
                         const int32_t *d_lens, int64_t n, int64_t ldc, int64_t col0,
                         int64_t col1, int32_t out_dtype, void *d_out, int64_t ld_out) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_TRY(check_params(p, n, ldc, out_dtype));
  if (col0 < 0 || col1 > n || col0 >= col1) return fail(KMG_EINVAL, "bad column range");
  KMG_HIP(hipSetDevice(c->device));
  return gram_device(c, p, d_codes, d_lens, (int)ldc, n, ldc, {RowRange{0, n, d_out}},
                     out_dtype, ld_out, nullptr, col0, col1 - col0);
}

int kmg_gram_to_host(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes,
                     const int32_t *d_lens, int64_t n, int64_t ldc, int32_t out_dtype,
                     int64_t slab_rows, void *h_out, int64_t ld_host) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_TRY(check_params(p, n, ldc, out_dtype));
  if (n == 0) return KMG_OK;
  if (!h_out || ld_host < n || slab_rows < 1) return fail(KMG_EINVAL, "bad host output / slab_rows");
  KMG_HIP(hipSetDevice(c->device));
  const size_t esz = dtype_size(out_dtype);
  slab_rows = std::min<int64_t>(slab_rows, n);
  const size_t sb = (size_t)slab_rows * (size_t)n * esz;
  KMG_TRY(c->slabs.ensure(2 * sb));
  if (!c->d2h_stream) {
    KMG_HIP(hipStreamCreateWithFlags(&c->d2h_stream, hipStreamNonBlocking));
    for (int b = 0; b < 2; ++b) {
      KMG_HIP(hipEventCreateWithFlags(&c->ev_slab[b], hipEventDisableTiming));
      KMG_HIP(hipEventCreateWithFlags(&c->ev_out[b], hipEventDisableTiming));
    }
  }
  std::vector<RowRange> ranges;
  for (int64_t r0 = 0, q = 0; r0 < n; r0 += slab_rows, ++q)
    ranges.push_back(RowRange{r0, std::min(n, r0 + slab_rows), (char *)c->slabs.p + (q & 1) * sb, n});
  // slab q's copy: on the d2h stream behind slab q's Gram, into host rows [r0, r1)
  auto copy_out = [&](size_t q) -> int {
    const RowRange &rg = ranges[q];
    KMG_HIP(hipStreamWaitEvent(c->d2h_stream, c->ev_slab[q & 1], 0));
    KMG_HIP(hipMemcpy2DAsync((char *)h_out + (size_t)rg.row0 * ld_host * esz, (size_t)ld_host * esz,
                             rg.out, (size_t)n * esz, (size_t)n * esz, (size_t)(rg.row1 - rg.row0),
                             hipMemcpyDeviceToHost, c->d2h_stream));
    KMG_HIP(hipEventRecord(c->ev_out[q & 1], c->d2h_stream));
    return KMG_OK;
  };
  // after slab q's Gram is enqueued: copy slab q - 1 out (overlapping slab q's Gram), and
  // hold slab q + 1's Gram (same buffer as q - 1) until that copy has landed
  AfterRange after = [&](size_t q) -> int {
    KMG_HIP(hipEventRecord(c->ev_slab[q & 1], c->stream));
    if (q >= 1) {
      KMG_TRY(copy_out(q - 1));
      KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_out[(q - 1) & 1], 0));
    }
    return KMG_OK;
  };
  const int rc = [&]() -> int {
    KMG_TRY(gram_device(c, p, d_codes, d_lens, (int)ldc, n, ldc, ranges, out_dtype, n, after));
    return copy_out(ranges.size() - 1);
  }();
  // on every exit path: no slab copy into the caller's buffer may still be running when
  // this returns (a failed call's caller may unmap the buffer right away)
  const hipError_t e_d2h = hipStreamSynchronize(c->d2h_stream);
  const hipError_t e_ctx = hipStreamSynchronize(c->stream);
  if (rc != KMG_OK) return rc;
  KMG_HIP(e_d2h);
  KMG_HIP(e_ctx);
  return KMG_OK;
}

int kmg_reload_tuning(kmg_ctx *c) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  read_tuning(c->tune);
  return KMG_OK;
}

int64_t kmg_rows_padded(int64_t n, int32_t nranks, int64_t block) {
  if (n <= 0 || nranks < 1 || block < 1) return n > 0 ? n : 0;
  const int64_t round = (int64_t)nranks * block;
  return (n + round - 1) / round * round;
}

namespace {
constexpr int KMG_RETRY_WIDE = 1000;  // internal: a 16-bit slab overflowed, redo with 32 bits

int gram_blocks_impl(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes,
                     const int32_t *d_lens, int64_t n, int64_t ldc, int32_t out_dtype,
                     void *d_out, int64_t ld_out, int32_t nranks, int32_t rank, int64_t block,
                     int32_t gather, int narrow_bits);
}  // namespace

namespace {
// Column blocks (gather 5 / 6): rank q computes the column block K[:, C_q], C_q = [q * block,
// min(n, (q + 1) * block)), with the neighbourhood lists built over its own |C_q| sequences
// (kmg_gram_device_cols: every list read by all n rows, so they pack), transposes it into
// K's rows C_q (the row slab: K is symmetric), and the slabs are all-gathered in place over
// RCCL (gather 5; one equal-count ncclAllGather, d_out holds nranks * block rows).  gather 6
// computes every rank's block on this GPU (the one-GPU rehearsal, no RCCL).  The transposes
// are timed as "unpack", the all-gather as "gather".
int gram_colblocks_impl(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes,
                        const int32_t *d_lens, int64_t n, int64_t ldc, int32_t out_dtype,
                        void *d_out, int64_t ld_out, int32_t nranks, int32_t rank, int64_t block,
                        int32_t gather) {
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(KMG_EINVAL, "bad rank %d of %d", rank, nranks);
  if (block < 1 || (int64_t)nranks * block < n)
    return fail(KMG_EINVAL, "column blocks: nranks * block = %lld rows must cover n = %lld",
                (long long)nranks * (long long)block, (long long)n);
  if (n > 0 && (!d_out || ld_out < n)) return fail(KMG_EINVAL, "bad output");
  if (out_dtype != KMG_I32 && out_dtype != KMG_F32 && out_dtype != KMG_F64)
    return fail(KMG_EINVAL, "bad output dtype %d", out_dtype);
  const bool rccl = gather == 5 && (nranks > 1 || (c->comm && c->nranks == 1));
  if (rccl && (!c->comm || c->nranks != nranks || c->rank != rank))
    return fail(KMG_EINVAL, "gather needs a communicator of %d ranks with this rank %d", nranks, rank);
  KMG_HIP(hipSetDevice(c->device));
  const size_t esz = dtype_size(out_dtype);
  c->last_wire_bytes = (int)esz;
  if (n == 0) return KMG_OK;
  KMG_TRY(c->cb_scratch.ensure((size_t)n * (size_t)block * esz));
  for (int32_t q = 0; q < nranks; ++q) {
    if (gather != 6 && q != rank) continue;
    const int64_t c0 = std::min(n, (int64_t)q * block), c1 = std::min(n, c0 + block), w = c1 - c0;
    if (w <= 0) continue;
    KMG_TRY(gram_device(c, p, d_codes, d_lens, (int)ldc, n, ldc, {RowRange{0, n, c->cb_scratch.p}},
                        out_dtype, w, nullptr, c0, w));
    StageTimer t(c, ST_UNPACK);
    KMG_HIP(launch_transpose(c->cb_scratch.p, w, n, w, (char *)d_out + (size_t)c0 * ld_out * esz,
                             ld_out, (int)esz, c->stream));
  }
  if (rccl) {  // in place: rank q's slab at rows q * block (send = recv + rank * count)
    if (!c->comm_stream) KMG_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
    if (!c->ev_sync) KMG_HIP(hipEventCreateWithFlags(&c->ev_sync, hipEventDisableTiming));
    KMG_HIP(hipEventRecord(c->ev_sync, c->stream));
    KMG_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_sync, 0));
    const size_t count = (size_t)block * (size_t)ld_out * esz;
    hipEvent_t b = nullptr, e = nullptr;
    if (c->timing) {
      b = pool_event(c);
      e = pool_event(c);
      KMG_HIP(hipEventRecord(b, c->comm_stream));
    }
    ncclResult_t r = ncclAllGather((char *)d_out + (size_t)rank * count, d_out, count, ncclChar, c->comm,
                                   c->comm_stream);
    if (r != ncclSuccess) return fail(KMG_ERCCL, "ncclAllGather (column blocks): %s", ncclGetErrorString(r));
    if (c->timing) {
      KMG_HIP(hipEventRecord(e, c->comm_stream));
      c->ev_log.push_back({ST_GATHER, {b, e}});
    }
    KMG_HIP(hipEventRecord(c->ev_sync, c->comm_stream));
    KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_sync, 0));
  }
  return KMG_OK;
}
}  // namespace

int kmg_gram_blocks(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes,
                    const int32_t *d_lens, int64_t n, int64_t ldc, int32_t out_dtype, void *d_out,
                    int64_t ld_out, int32_t nranks, int32_t rank, int64_t block, int32_t gather) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_TRY(check_params(p, n, ldc, out_dtype));
  if (gather == 5 || gather == 6)
    return gram_colblocks_impl(c, p, d_codes, d_lens, n, ldc, out_dtype, d_out, ld_out, nranks,
                               rank, block, gather);
  // round slabs as narrow as the counts allow: 8 bits, else 16, else the output dtype
  int r = KMG_RETRY_WIDE;
  for (int bits : {8, 16, 0}) {
    r = gram_blocks_impl(c, p, d_codes, d_lens, n, ldc, out_dtype, d_out, ld_out, nranks, rank,
                         block, gather, bits);
    if (r != KMG_RETRY_WIDE) break;
  }
  return r;
}

int kmg_gram_blocks_wire(kmg_ctx *c) { return c ? c->last_wire_bytes : 0; }

namespace {
// Escapes of uint8 round slabs (counts >= 255): the ranks all-gather their lists (the
// per-rank counts first, then max-count entries from every rank) and every rank patches
// them into its K after the unpacks (context stream, which already waits for them).
int patch_escapes(kmg_ctx *c, const kmg_params *p, int64_t n, void *d_out, int64_t ld_out,
                  int32_t out_dtype, int32_t nranks, int32_t rank, bool rccl) {
  uint32_t *cnt = c->esc_cnt.as<uint32_t>();  // [0] this process's count, [1..] gathered
  const double *diagv = c->diagv.as<double>(), *dsq = c->dsq.as<double>();
  if (!rccl || nranks == 1) {
    KMG_HIP(launch_tri_patch8(c->esc.as<uint4>(), cnt, 1, c->esc_cap, c->esc_cap, d_out, ld_out,
                              out_dtype, p->normalize, diagv, dsq, c->stream));
    return KMG_OK;
  }
  KMG_HIP(hipMemcpyAsync(cnt + 1 + rank, cnt, sizeof(uint32_t), hipMemcpyDeviceToDevice, c->stream));
  KMG_HIP(hipEventRecord(c->ev_sync, c->stream));
  KMG_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_sync, 0));
  ncclResult_t r = ncclAllGather(cnt + 1 + rank, cnt + 1, 1, ncclUint32, c->comm, c->comm_stream);
  if (r != ncclSuccess) return fail(KMG_ERCCL, "ncclAllGather (escape counts): %s", ncclGetErrorString(r));
  std::vector<uint32_t> counts((size_t)nranks);
  KMG_HIP(hipMemcpyAsync(counts.data(), cnt + 1, sizeof(uint32_t) * nranks, hipMemcpyDeviceToHost,
                         c->comm_stream));
  KMG_HIP(hipStreamSynchronize(c->comm_stream));
  uint32_t maxc = 0;
  for (uint32_t v : counts) maxc = std::max(maxc, std::min(v, c->esc_cap));
  if (maxc == 0) return KMG_OK;
  KMG_TRY(c->esc_all.ensure(sizeof(uint4) * (size_t)maxc * nranks));
  r = ncclAllGather(c->esc.p, c->esc_all.p, sizeof(uint4) * (size_t)maxc, ncclChar, c->comm,
                    c->comm_stream);
  if (r != ncclSuccess) return fail(KMG_ERCCL, "ncclAllGather (escapes): %s", ncclGetErrorString(r));
  KMG_HIP(hipEventRecord(c->ev_sync, c->comm_stream));
  KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_sync, 0));
  KMG_HIP(launch_tri_patch8(c->esc_all.as<uint4>(), cnt + 1, nranks, maxc, maxc, d_out, ld_out,
                            out_dtype, p->normalize, diagv, dsq, c->stream));
  return KMG_OK;
}

int gram_blocks_impl(kmg_ctx *c, const kmg_params *p, const uint8_t *d_codes,
                     const int32_t *d_lens, int64_t n, int64_t ldc, int32_t out_dtype,
                     void *d_out, int64_t ld_out, int32_t nranks, int32_t rank, int64_t block,
                     int32_t gather, int narrow_bits) {
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(KMG_EINVAL, "bad rank %d of %d", rank, nranks);
  if (block < 1) return fail(KMG_EINVAL, "block < 1");
  if (gather < 0 || gather > 4) return fail(KMG_EINVAL, "gather must be 0..6");
  const bool packed = gather == 4;  // this rank's blocks, packed (no collective)
  if (packed) gather = 0;
  if (n > 0 && (!d_out || ld_out < n)) return fail(KMG_EINVAL, "bad output");
  const bool tri = gather >= 2;               // upper-triangle round slabs + local mirror
  // RCCL path: more than one rank, or a communicator of exactly this one rank (a 1-rank
  // all-gather is an in-place no-op: the one-GPU test of the stream / event ordering)
  const bool rccl = (gather == 1 || gather == 2) && (nranks > 1 || (c->comm && c->nranks == 1));
  if (rccl && (!c->comm || c->nranks != nranks || c->rank != rank))
    return fail(KMG_EINVAL, "gather needs a communicator of %d ranks with this rank %d", nranks, rank);
  KMG_HIP(hipSetDevice(c->device));
  const size_t esz = dtype_size(out_dtype);
  const int64_t round = (int64_t)nranks * block;
  const int64_t nround = (n + round - 1) / round;
  // Upper-triangle round slabs travel as raw uint16 counts whenever a posting-list kernel
  // builds them (spectrum: every count <= P_max^2 <= 65025 for P_max <= 255; mismatch:
  // checked, a count above 65535 sets a flag and the build is redone with 32-bit slabs):
  // half the xGMI bytes of an int32 K, a quarter of a float64 one; the unpack pass widens
  // (and normalises) them into K.
  // Slabs as raw uint8 (diagonal left out; every rank computes K_ii itself) or uint16
  // counts when a posting-list kernel builds them; a count past the slab's range sets a
  // flag the ranks agree on, and the build is redone one width up (kmg_gram_blocks).
  int32_t wire = out_dtype;
  bool check16 = false;
  if (gather >= 2 && narrow_bits && (p->kind == KMG_SPECTRUM || p->kind == KMG_MISMATCH) &&
      p->k >= 1 && p->k <= 16) {
    const bool mm = p->kind == KMG_MISMATCH;
    const int L = mm ? (p->window > 0 ? p->window : 101) : (int)ldc;  // gram_device's maxlen
    const int pmax = std::max(1, L - p->k + 1);
    const SmPath path = sm_path(c->tune, p, pmax, n);
    // 8-bit slabs for every posting-list path: an off-diagonal count >= 255 (a pair sharing
    // a long k-mer; ~1e-4 of random 101-mer pairs for MM(9,1)) travels in an escape list
    // that is all-gathered after the slabs and patched into K; a full list redoes the
    // build with 16-bit slabs
    if ((path == SM_POSTING && pmax <= 255) || path == SM_SLOTS || path == SM_PAIRS ||
        path == SM_NB) {
      wire = narrow_bits == 8 ? KMG_U8 : KMG_U16;
      check16 = wire == KMG_U8 || path != SM_POSTING;  // spectrum counts <= P^2 < 65536
    } else if (narrow_bits == 8) {
      return KMG_RETRY_WIDE;
    }
  }
  const size_t wsz = dtype_size(wire);
  c->last_wire_bytes = (int)(gather >= 2 ? wsz : esz);
  if (rccl && !c->comm_stream) KMG_HIP(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
  if ((rccl || tri) && !c->ev_sync) KMG_HIP(hipEventCreateWithFlags(&c->ev_sync, hipEventDisableTiming));
  // unpack (mirror) stream: its own stream over RCCL, so the unpack of round t overlaps the
  // all-gather of round t + 1 on the comm stream
  if (rccl && tri && !c->unpack_stream) {
    KMG_HIP(hipStreamCreateWithFlags(&c->unpack_stream, hipStreamNonBlocking));
    for (int b = 0; b < 2; ++b) KMG_HIP(hipEventCreateWithFlags(&c->ev_gath[b], hipEventDisableTiming));
  }
  hipStream_t post = rccl ? (tri ? c->unpack_stream : c->comm_stream) : c->stream;
  auto gather_bytes = [&](char *recv, size_t count) -> int {  // in place, rank r at r * count
    hipEvent_t b = nullptr, e = nullptr;
    if (c->timing) {
      b = pool_event(c);
      e = pool_event(c);
      KMG_HIP(hipEventRecord(b, c->comm_stream));
    }
    ncclResult_t r = ncclAllGather(recv + (size_t)rank * count, recv, count, ncclChar, c->comm,
                                   c->comm_stream);
    if (r != ncclSuccess) return fail(KMG_ERCCL, "ncclAllGather: %s", ncclGetErrorString(r));
    if (c->timing) {
      KMG_HIP(hipEventRecord(e, c->comm_stream));
      c->ev_log.push_back({ST_GATHER, {b, e}});
    }
    return KMG_OK;
  };
  std::vector<RowRange> ranges;
  std::vector<int64_t> last_of_round;  // range index -> round it completes (-1: none)
  AfterRange after = nullptr;
  if (!tri) {
    // this rank's block of every round: rows [t*round + rank*block, +block) clipped to n
    for (int64_t t = 0; t < nround; ++t) {
      const int64_t r0 = std::min(n, t * round + (int64_t)rank * block);
      const int64_t r1 = std::min(n, r0 + block);
      const int64_t orow = packed ? t * block : r0;  // output row of K's row r0
      ranges.push_back(RowRange{r0, r1, (char *)d_out + (size_t)orow * ld_out * esz});
    }
    if (rccl) {
      after = [&](size_t t) -> int {
        // round t's rows [t*round, (t+1)*round) are contiguous in d_out: rank q's block sits
        // at q * block rows, i.e. send = recv + rank * count, so the all-gather is in place.
        // It runs on its own stream behind an event of this rank's Gram launch, overlapped
        // with the next round's Gram kernels (one event suffices: hipStreamWaitEvent
        // captures the record made just before it).
        KMG_HIP(hipEventRecord(c->ev_sync, c->stream));
        KMG_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_sync, 0));
        return gather_bytes((char *)d_out + (size_t)(t * round) * ld_out * esz,
                            (size_t)block * ld_out * esz);
      };
    }
  } else {
    // Upper triangle: round t computes only columns >= c_t = t*round of its
    // rows, into a contiguous round slab S_t [round][w_t], w_t = n - c_t (rank q's block at
    // q * block rows), which is all-gathered in place (half the xGMI bytes of full rows),
    // copied into K's rows [c_t, c_t + round) at columns >= c_t, and mirrored into the
    // columns [c_t, c_t + round) of every later row (K[x][c_t + y] = S_t[y][x - c_t]).
    // Two slabs alternate; round t waits for the mirror of round t - 2 before reusing its
    // slab.  gather = 3 computes every rank's blocks locally (a one-GPU rehearsal of the
    // same layout, no RCCL).
    const size_t slab = (size_t)round * (size_t)std::max<int64_t>(n, 1) * wsz;
    KMG_TRY(c->tri_stage.ensure(2 * slab));
    for (int64_t t = 0; t < nround; ++t) {
      const int64_t c0 = t * round, w = n - c0;
      char *S = (char *)c->tri_stage.p + (size_t)(t & 1) * slab;
      for (int32_t q = 0; q < nranks; ++q) {
        if (gather != 3 && q != rank) continue;
        const int64_t r0 = std::min(n, c0 + (int64_t)q * block);
        const int64_t r1 = std::min(n, r0 + block);
        // `out` addresses column 0 of row r0: columns < c0 are never written
        char *out = S + ((int64_t)q * block * w - c0) * (int64_t)wsz;
        ranges.push_back(RowRange{r0, r1, out, w, c0});
        last_of_round.push_back(-1);
      }
      last_of_round.back() = t;
    }
    if (!c->ev_tri[0]) {
      for (int b = 0; b < 2; ++b)
        KMG_HIP(hipEventCreateWithFlags(&c->ev_tri[b], hipEventDisableTiming));
    }
    after = [&](size_t q) -> int {
      const int64_t t = last_of_round[q];
      if (t < 0) return KMG_OK;
      const int64_t c0 = t * round, w = n - c0;
      char *S = (char *)c->tri_stage.p + (size_t)(t & 1) * slab;
      if (rccl) {
        KMG_HIP(hipEventRecord(c->ev_sync, c->stream));
        KMG_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_sync, 0));
        KMG_TRY(gather_bytes(S, (size_t)block * w * wsz));
        KMG_HIP(hipEventRecord(c->ev_gath[t & 1], c->comm_stream));
        KMG_HIP(hipStreamWaitEvent(post, c->ev_gath[t & 1], 0));
      }
      // unpack / mirror: timed when it runs on the context stream (no RCCL; the one-GPU
      // rehearsal the bench's multi-GPU projection reads)
      std::unique_ptr<StageTimer> ut(post == c->stream ? new StageTimer(c, ST_UNPACK) : nullptr);
      if (wire == KMG_U8)
        KMG_HIP(launch_tri_unpack8((const uint8_t *)S, w, round, c0, n, d_out, ld_out, out_dtype,
                                   p->normalize, c->diagv.as<double>(), c->dsq.as<double>(), post));
      else if (wire == KMG_U16)
        KMG_HIP(launch_tri_unpack16((const uint16_t *)S, w, round, c0, n, d_out, ld_out, out_dtype,
                                    p->normalize, c->diagv.as<double>(), c->dsq.as<double>(), post));
      else
        KMG_HIP(launch_tri_unpack(S, w, round, c0, n, d_out, ld_out, (int)esz, post));
      ut.reset();
      KMG_HIP(hipEventRecord(c->ev_tri[t & 1], post));
      // the next Gram launch (round t + 1) writes the slab round t - 1 used
      if (t >= 1) KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_tri[(t - 1) & 1], 0));
      return KMG_OK;
    };
  }
  c->esc_cap = 0;
  if (wire == KMG_U8 && n > 0) {
    // escape list sized for ~1/512 of this process's upper-triangle pairs (random 101-mers:
    // ~1e-4 of MM(9,1) pairs reach 255), at least 65536 entries
    const double pairs = 0.5 * (double)n * (double)n / (gather == 3 ? 1.0 : (double)nranks);
    const int64_t cap = c->tune.esc_cap > 0
                            ? (int64_t)c->tune.esc_cap
                            : std::min<int64_t>(1 << 24, std::max<int64_t>(65536, (int64_t)(pairs / 512.0)));
    KMG_TRY(c->esc.ensure(sizeof(uint4) * (size_t)cap));
    KMG_TRY(c->esc_cnt.ensure(sizeof(uint32_t) * (size_t)(1 + nranks)));
    KMG_HIP(hipMemsetAsync(c->esc_cnt.p, 0, sizeof(uint32_t), c->stream));
    c->esc_cap = (uint32_t)cap;
  }
  KMG_TRY(gram_device(c, p, d_codes, d_lens, (int)ldc, n, ldc, ranges, tri ? wire : out_dtype,
                      ld_out, after));
  if (rccl) {  // stream order: later work on the context stream sees the full K
    KMG_HIP(hipEventRecord(c->ev_sync, c->comm_stream));
    KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_sync, 0));
    if (post != c->comm_stream) {
      KMG_HIP(hipEventRecord(c->ev_sync, post));
      KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_sync, 0));
    }
  }
  if (check16 && n > 0) {
    // one 4-byte read per build; all ranks agree (max over ranks) before any redoes
    if (rccl) {
      KMG_HIP(hipEventRecord(c->ev_sync, c->stream));
      KMG_HIP(hipStreamWaitEvent(c->comm_stream, c->ev_sync, 0));
      ncclResult_t r = ncclAllReduce(c->ovf.p, c->ovf.p, 1, ncclUint32, ncclMax, c->comm,
                                     c->comm_stream);
      if (r != ncclSuccess) return fail(KMG_ERCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
      KMG_HIP(hipEventRecord(c->ev_sync, c->comm_stream));
      KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_sync, 0));
    }
    uint32_t flag = 0;
    KMG_HIP(hipMemcpyAsync(&flag, c->ovf.p, sizeof(flag), hipMemcpyDeviceToHost, c->stream));
    KMG_HIP(hipStreamSynchronize(c->stream));
    if (flag) return KMG_RETRY_WIDE;
  }
  if (c->esc_cap > 0) KMG_TRY(patch_escapes(c, p, n, d_out, ld_out, out_dtype, nranks, rank, rccl));
  return KMG_OK;
}
}  // namespace

int kmg_normalize(kmg_ctx *c, double *K, int64_t n, int64_t ld, int32_t *skipped) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  if (skipped) *skipped = 0;
  if (n <= 0) return KMG_OK;
  if (!K || ld < n) return fail(KMG_EINVAL, "bad matrix");
  if (K[0] == 1.0) {  // kernels.py:404-405: already normalised -> unchanged
    if (skipped) *skipped = 1;
    return KMG_OK;
  }
  KMG_HIP(hipSetDevice(c->device));
  KMG_TRY(c->h_out.ensure(sizeof(double) * (size_t)n * n));
  double *d = c->h_out.as<double>();
  KMG_HIP(hipMemcpy2DAsync(d, n * 8, K, ld * 8, n * 8, n, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(launch_normalize_dense(d, n, n, c->stream));
  KMG_HIP(hipMemcpy2DAsync(K, ld * 8, d, n * 8, n * 8, n, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

int kmg_center(kmg_ctx *c, const double *K, int64_t ldk, double *out, int64_t ld_out, int64_t n) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  if (n <= 0) return KMG_OK;
  if (!K || !out || ldk < n || ld_out < n) return fail(KMG_EINVAL, "bad matrix");
  KMG_HIP(hipSetDevice(c->device));
  const size_t mat = sizeof(double) * (size_t)n * n;
  KMG_TRY(c->h_out.ensure(2 * mat + sizeof(double) * (2 * (size_t)n + 1)));
  double *dK = c->h_out.as<double>();
  double *dO = dK + (size_t)n * n;
  double *rm = dO + (size_t)n * n;
  double *cm = rm + n;
  double *tot = cm + n;
  KMG_HIP(hipMemcpy2DAsync(dK, n * 8, K, ldk * 8, n * 8, n, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(launch_center_dense(dK, n, dO, n, n, rm, cm, tot, c->stream));
  KMG_HIP(hipMemcpy2DAsync(out, ld_out * 8, dO, n * 8, n * 8, n, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

int kmg_dmalloc(kmg_ctx *c, void **ptr, size_t bytes) {
  if (!c || !ptr) return fail(KMG_EINVAL, "NULL argument");
  KMG_HIP(hipSetDevice(c->device));
  KMG_HIP(hipMalloc(ptr, bytes ? bytes : 1));
  return KMG_OK;
}
int kmg_dfree(kmg_ctx *c, void *ptr) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  KMG_HIP(hipSetDevice(c->device));
  if (ptr) KMG_HIP(hipFree(ptr));
  return KMG_OK;
}
int kmg_h2d(kmg_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  KMG_HIP(hipSetDevice(c->device));
  KMG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}
int kmg_d2h(kmg_ctx *c, void *dst, const void *src, size_t bytes) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  KMG_HIP(hipSetDevice(c->device));
  KMG_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}
int kmg_memset(kmg_ctx *c, void *dst, int value, size_t bytes) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  KMG_HIP(hipSetDevice(c->device));
  StageTimer t(c, ST_MEMSET);
  KMG_HIP(hipMemsetAsync(dst, value, bytes, c->stream));
  return KMG_OK;
}
int kmg_synchronize(kmg_ctx *c) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  KMG_HIP(hipSetDevice(c->device));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}
int kmg_stream(kmg_ctx *c, void **s) {
  if (!c || !s) return fail(KMG_EINVAL, "NULL argument");
  *s = (void *)c->stream;
  return KMG_OK;
}

int kmg_set_timing(kmg_ctx *c, int32_t enable) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  c->timing = enable == 2 ? 2 : (enable != 0 ? 1 : 0);
  return KMG_OK;
}

int kmg_timing_reset(kmg_ctx *c) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  KMG_HIP(hipStreamSynchronize(c->stream));
  c->ev_log.clear();
  c->ev_used = 0;
  c->last_call_first = 0;
  return KMG_OK;
}

static int stage_index(const char *stage) {
  for (int s = 0; s < kNumStages; ++s)
    if (strcmp(stage, kStageNames[s]) == 0) return s;
  return -1;
}

static int stage_sum(kmg_ctx *c, int idx, size_t first, double *total, int32_t *count) {
  double t = 0.0;
  int32_t n = 0;
  for (size_t q = first; q < c->ev_log.size(); ++q) {
    if (c->ev_log[q].first != idx) continue;
    KMG_HIP(hipEventSynchronize(c->ev_log[q].second.second));
    float f = 0.f;
    KMG_HIP(hipEventElapsedTime(&f, c->ev_log[q].second.first, c->ev_log[q].second.second));
    t += f;
    ++n;
  }
  *total = t;
  *count = n;
  return KMG_OK;
}

int kmg_stage_ms(kmg_ctx *c, const char *stage, double *ms) {
  if (!c || !stage || !ms) return fail(KMG_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(c->mu);
  const int idx = stage_index(stage);
  if (idx < 0) return fail(KMG_EINVAL, "unknown stage '%s'", stage);
  double t;
  int32_t n;
  KMG_TRY(stage_sum(c, idx, (size_t)c->last_call_first, &t, &n));
  *ms = n ? t : -1.0;
  return KMG_OK;
}

int kmg_last_factorisation(kmg_ctx *c, int32_t *kind) {
  if (!c || !kind) return fail(KMG_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(c->mu);
  *kind = c->last_factor;
  return KMG_OK;
}

int kmg_last_plan(kmg_ctx *c, int32_t plan[6]) {
  if (!c || !plan) return fail(KMG_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(c->mu);
  for (int q = 0; q < 6; ++q) plan[q] = c->plan[q];
  return KMG_OK;
}

int kmg_stage_stats(kmg_ctx *c, const char *stage, double *total_ms, int32_t *count) {
  if (!c || !stage || !total_ms || !count) return fail(KMG_EINVAL, "NULL argument");
  std::lock_guard<std::mutex> lk(c->mu);
  const int idx = stage_index(stage);
  if (idx < 0) return fail(KMG_EINVAL, "unknown stage '%s'", stage);
  return stage_sum(c, idx, 0, total_ms, count);
}

// ------------------------------------------------------------------ combination consumers
static int check_combine(kmg_ctx *c, const void *K, int32_t p, int64_t n, int64_t ld) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  if (!K) return fail(KMG_EINVAL, "K is NULL");
  if (p < 1 || p > KMG_COMBINE_PMAX) return fail(KMG_EUNSUPPORTED, "p=%d outside [1,%d]", p, KMG_COMBINE_PMAX);
  if (n < 0 || (n > 0 && ld < n)) return fail(KMG_EINVAL, "bad matrix shape");
  return KMG_OK;
}

// device array of the p matrix pointers
static int upload_ptrs(kmg_ctx *c, const double *const *ptrs, int32_t p) {
  KMG_TRY(c->cmb_ptrs.ensure(sizeof(double *) * (size_t)p));
  KMG_HIP(hipMemcpyAsync(c->cmb_ptrs.p, ptrs, sizeof(double *) * (size_t)p, hipMemcpyHostToDevice,
                         c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));  // pageable source
  return KMG_OK;
}

// host matrices -> one device slab [p][n][n]; returns the device pointer array
static int stage_host_kernels(kmg_ctx *c, const double *const *K, int32_t p, int64_t n, int64_t ld,
                              std::vector<const double *> &dptrs) {
  const size_t mat = sizeof(double) * (size_t)n * (size_t)n;
  KMG_TRY(c->cmb_k.ensure(mat * (size_t)p));
  dptrs.resize(p);
  for (int m = 0; m < p; ++m) {
    if (!K[m]) return fail(KMG_EINVAL, "K[%d] is NULL", m);
    double *dst = c->cmb_k.as<double>() + (size_t)m * n * n;
    KMG_HIP(hipMemcpy2DAsync(dst, n * 8, K[m], ld * 8, n * 8, n, hipMemcpyHostToDevice, c->stream));
    dptrs[m] = dst;
  }
  return upload_ptrs(c, dptrs.data(), p);
}

int kmg_combine_device(kmg_ctx *c, const double *const *d_K, int32_t p, const double *d_u,
                       int32_t degree, int64_t n, int64_t ld, double *d_out, int64_t ld_out) {
  KMG_TRY(check_combine(c, d_K, p, n, ld));
  std::lock_guard<std::mutex> lk(c->mu);
  if (degree < 0) return fail(KMG_EINVAL, "degree < 0");
  if (n > 0 && ld_out < n) return fail(KMG_EINVAL, "ld_out < n");
  KMG_HIP(hipSetDevice(c->device));
  KMG_TRY(upload_ptrs(c, d_K, p));
  StageTimer t(c, ST_COMBINE);
  KMG_HIP(launch_combine(c->cmb_ptrs.as<const double *>(), d_u, p, degree, n, ld, d_out, ld_out,
                         c->stream));
  return KMG_OK;
}

int kmg_combine(kmg_ctx *c, const double *const *K, int32_t p, const double *u, int32_t degree,
                int64_t n, int64_t ld, double *out, int64_t ld_out) {
  KMG_TRY(check_combine(c, K, p, n, ld));
  std::lock_guard<std::mutex> lk(c->mu);
  if (degree < 0) return fail(KMG_EINVAL, "degree < 0");
  if (!u || !out || (n > 0 && ld_out < n)) return fail(KMG_EINVAL, "bad u / out");
  KMG_HIP(hipSetDevice(c->device));
  if (n == 0) return KMG_OK;
  std::vector<const double *> dptrs;
  KMG_TRY(stage_host_kernels(c, K, p, n, ld, dptrs));
  KMG_TRY(c->cmb_vec.ensure(sizeof(double) * (size_t)p));
  KMG_TRY(c->cmb_out.ensure(sizeof(double) * (size_t)n * n));
  KMG_HIP(hipMemcpyAsync(c->cmb_vec.p, u, sizeof(double) * p, hipMemcpyHostToDevice, c->stream));
  {
    StageTimer t(c, ST_COMBINE);
    KMG_HIP(launch_combine(c->cmb_ptrs.as<const double *>(), c->cmb_vec.as<double>(), p, degree,
                           n, n, c->cmb_out.as<double>(), n, c->stream));
  }
  KMG_HIP(hipMemcpy2DAsync(out, ld_out * 8, c->cmb_out.p, n * 8, n * 8, n, hipMemcpyDeviceToHost,
                           c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

int kmg_nlck_grad_device(kmg_ctx *c, const double *const *d_K, int32_t p, const double *d_u,
                         int32_t degree, const double *d_alpha, int64_t n, int64_t ld,
                         double *d_grad) {
  KMG_TRY(check_combine(c, d_K, p, n, ld));
  std::lock_guard<std::mutex> lk(c->mu);
  if (degree < 1) return fail(KMG_EINVAL, "degree < 1");
  KMG_HIP(hipSetDevice(c->device));
  if (n == 0) return KMG_OK;
  KMG_TRY(upload_ptrs(c, d_K, p));
  KMG_TRY(c->cmb_tmp.ensure(sizeof(double) * (size_t)n * p));
  StageTimer t(c, ST_COMBINE);
  KMG_HIP(launch_nlck_grad(c->cmb_ptrs.as<const double *>(), d_u, p, degree, d_alpha, n, ld,
                           c->cmb_tmp.as<double>(), d_grad, c->stream));
  return KMG_OK;
}

int kmg_nlck_grad(kmg_ctx *c, const double *const *K, int32_t p, const double *u,
                  int32_t degree, const double *alpha, int64_t n, int64_t ld, double *grad) {
  KMG_TRY(check_combine(c, K, p, n, ld));
  std::lock_guard<std::mutex> lk(c->mu);
  if (degree < 1) return fail(KMG_EINVAL, "degree < 1");
  if (!u || !alpha || !grad) return fail(KMG_EINVAL, "NULL buffer");
  KMG_HIP(hipSetDevice(c->device));
  if (n == 0) {
    for (int m = 0; m < p; ++m) grad[m] = -0.0 * degree;
    return KMG_OK;
  }
  std::vector<const double *> dptrs;
  KMG_TRY(stage_host_kernels(c, K, p, n, ld, dptrs));
  KMG_TRY(c->cmb_vec.ensure(sizeof(double) * (size_t)(2 * p + n)));
  double *du = c->cmb_vec.as<double>(), *dg = du + p, *da = dg + p;
  KMG_HIP(hipMemcpyAsync(du, u, sizeof(double) * p, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipMemcpyAsync(da, alpha, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
  KMG_TRY(c->cmb_tmp.ensure(sizeof(double) * (size_t)n * p));
  {
    StageTimer t(c, ST_COMBINE);
    KMG_HIP(launch_nlck_grad(c->cmb_ptrs.as<const double *>(), du, p, degree, da, n, n,
                             c->cmb_tmp.as<double>(), dg, c->stream));
  }
  KMG_HIP(hipMemcpyAsync(grad, dg, sizeof(double) * p, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

static int alignf_run(kmg_ctx *c, const double *const *dptrs_dev, int32_t p, const double *d_y,
                      int64_t n, int64_t ld, double *d_out) {
  const size_t stride = (size_t)p + (size_t)p * (p + 1) / 2;
  KMG_TRY(c->cmb_tmp.ensure(sizeof(double) * ((size_t)n * stride + 2 * (size_t)p * n + p)));
  double *part = c->cmb_tmp.as<double>();
  double *rmean = part + (size_t)n * stride, *cmean = rmean + (size_t)p * n;
  double *tmean = cmean + (size_t)p * n;
  StageTimer t(c, ST_COMBINE);
  KMG_HIP(launch_alignf(dptrs_dev, p, d_y, n, ld, rmean, cmean, tmean, part, d_out, c->stream));
  return KMG_OK;
}

int kmg_alignf_device(kmg_ctx *c, const double *const *d_K, int32_t p, const double *d_y,
                      int64_t n, int64_t ld, double *d_out) {
  KMG_TRY(check_combine(c, d_K, p, n, ld));
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  if (n == 0) return KMG_OK;
  KMG_TRY(upload_ptrs(c, d_K, p));
  return alignf_run(c, c->cmb_ptrs.as<const double *>(), p, d_y, n, ld, d_out);
}

int kmg_alignf(kmg_ctx *c, const double *const *K, int32_t p, const double *y, int64_t n,
               int64_t ld, double *a, double *M) {
  KMG_TRY(check_combine(c, K, p, n, ld));
  std::lock_guard<std::mutex> lk(c->mu);
  if (!y || !a || !M) return fail(KMG_EINVAL, "NULL buffer");
  KMG_HIP(hipSetDevice(c->device));
  const size_t stride = (size_t)p + (size_t)p * (p + 1) / 2;
  std::vector<double> host(stride, 0.0);
  if (n > 0) {
    std::vector<const double *> dptrs;
    KMG_TRY(stage_host_kernels(c, K, p, n, ld, dptrs));
    KMG_TRY(c->cmb_vec.ensure(sizeof(double) * ((size_t)n + stride)));
    double *dy = c->cmb_vec.as<double>(), *dout = dy + n;
    KMG_HIP(hipMemcpyAsync(dy, y, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    KMG_TRY(alignf_run(c, c->cmb_ptrs.as<const double *>(), p, dy, n, n, dout));
    KMG_HIP(hipMemcpyAsync(host.data(), dout, sizeof(double) * stride, hipMemcpyDeviceToHost,
                           c->stream));
    KMG_HIP(hipStreamSynchronize(c->stream));
  }
  for (int m = 0; m < p; ++m) a[m] = host[m];
  size_t q = p;
  for (int l = 0; l < p; ++l)
    for (int m = l; m < p; ++m, ++q) M[(size_t)l * p + m] = M[(size_t)m * p + l] = host[q];
  return KMG_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ dense learners on K
// KRR.fit (KRR.py:33) and KLR.fit (KLR.py:30-75): the reference inverts the n x n system
// with np.linalg.inv and multiplies; here the same system is factorised on the device
// (rocSOLVER Cholesky; LU with partial pivoting when the matrix is not positive definite,
// as inv() would still succeed there) and solved for the one right-hand side.
static int blas_handle(kmg_ctx *c) {
  if (!c->blas) {
    if (rocblas_create_handle(&c->blas) != rocblas_status_success) {
      c->blas = nullptr;
      return fail(KMG_EHIP, "rocblas_create_handle failed");
    }
  }
  if (rocblas_set_stream(c->blas, c->stream) != rocblas_status_success)
    return fail(KMG_EHIP, "rocblas_set_stream failed");
  return KMG_OK;
}

#define KMG_BLAS(expr)                                                                \
  do {                                                                                \
    rocblas_status _s = (expr);                                                       \
    if (_s != rocblas_status_success)                                                 \
      return fail(KMG_EHIP, "%s failed: %s (%s:%d)", #expr, rocblas_status_to_string(_s), \
                  __FILE__, __LINE__);                                                \
  } while (0)

// K != K^T (bitwise)?  The reference inverts whatever K it is given (KRR.py:33,
// KLR.py:55), so an asymmetric K (hand-made, or centred with rounding) must not be read
// through one triangle by the Cholesky path.
static int is_asymmetric(kmg_ctx *c, const double *d_K, int64_t ld, int64_t n, bool *asym) {
  int *flag = (int *)(c->sv_info.as<rocblas_int>() + 2);
  KMG_HIP(hipMemsetAsync(flag, 0, sizeof(int), c->stream));
  KMG_HIP(launch_asymmetry(d_K, ld, n, flag, c->stream));
  int h = 0;
  KMG_HIP(hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  *asym = h != 0;
  return KMG_OK;
}

// Right-looking blocked Cholesky of the symmetric n x n B (column-major lower, ld n) in
// place, 128-column blocks: the diagonal block and its inverse Y (launch_chol_diag: one
// workgroup, then 128 one-column workgroups), the panel below it as one GEMM (L21 = A21 Y^T,
// into sv_panel, copied back), the trailing triangle by rank-128 updates (a few GEMMs over
// its lower trapezoid: rocBLAS dsyrk recurses into many small ones).  Look-ahead: the
// next block column is updated first (one GEMM), the next diagonal block is factorised on a
// second stream while the rest of the trailing triangle takes its dsyrk here, so the
// latency-bound diagonal work hides behind the MFMA-bound update.  rocSOLVER's potrf issues
// ~22 kernels a block at n = 9000 (trtri, copies, recursive GEMMs; profiles/r05ba_*).
// The inverses (Y and Y^T of every block) stay in sv_inv for chol_solve.  *info (device)
// ends 0 or the 1-based column of the first non-positive pivot; nothing is read back here.
static constexpr int CHOL_BLK = 128;

// The in-tree factorisation (KMG_CHOL=1, not KMG_POTRF_UPPER) where the device has the LDS
// its diagonal-block inverse takes (gfx950's 160 KB); else rocSOLVER potrf / potrs.  One
// rule for KRR, KLR and the C-SVM.
static bool use_own_chol(const kmg_ctx *c) {
  return c->tune.chol && !c->tune.potrf_upper && (size_t)c->lds_max >= chol_diag_lds_bytes();
}

static int chol_factor(kmg_ctx *c, double *B, int64_t n, rocblas_int *info) {
  const int64_t nblk = (n + CHOL_BLK - 1) / CHOL_BLK;
  KMG_TRY(c->sv_inv.ensure(sizeof(double) * 2 * CHOL_BLK * CHOL_BLK * (size_t)nblk));
  KMG_TRY(c->sv_panel.ensure(sizeof(double) * CHOL_BLK * (size_t)n));
  if (!c->chol_stream) KMG_HIP(hipStreamCreateWithFlags(&c->chol_stream, hipStreamNonBlocking));
  for (hipEvent_t &e : c->ev_chol)
    if (!e) KMG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  double *inv = c->sv_inv.as<double>(), *T = c->sv_panel.as<double>();
  const double one = 1.0, mone = -1.0, zero = 0.0;
  const rocblas_int ld = (rocblas_int)n;
  auto diag = [&](int64_t b, hipStream_t st) -> int {
    const int64_t j0 = b * CHOL_BLK;
    const int jb = (int)std::min<int64_t>(CHOL_BLK, n - j0);
    double *Y = inv + 2 * CHOL_BLK * CHOL_BLK * b;
    KMG_HIP(launch_chol_diag(B + j0 + j0 * n, n, jb, (int)j0, (int *)info, Y, Y + CHOL_BLK * CHOL_BLK, st));
    return KMG_OK;
  };
  KMG_HIP(hipMemsetAsync(info, 0, sizeof(rocblas_int), c->stream));
  KMG_TRY(diag(0, c->stream));
  // Nothing is read back while the blocks are enqueued: after a non-positive pivot the later
  // diagonal / inverse launches return at once, but every panel GEMM and trailing update still
  // runs on stale inverses (their result is discarded: the caller rebuilds the system for LU).
  // An indefinite system therefore pays about one full factorisation before the LU fallback
  // (once per IRLS / interior-point step that meets one) -- the price of no host sync here.
  auto blocks = [&]() -> int {
    for (int64_t b = 0; b < nblk; ++b) {
      const int64_t j0 = b * CHOL_BLK;
      const int jb = (int)std::min<int64_t>(CHOL_BLK, n - j0);
      const rocblas_int m = (rocblas_int)(n - j0 - jb);
      if (m == 0) break;
      if (b > 0) KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_chol[1], 0));  // block b factorised
      double *Ajj = B + j0 + j0 * n, *A21 = Ajj + jb, *Y = inv + 2 * CHOL_BLK * CHOL_BLK * b;
      KMG_BLAS(rocblas_dgemm(c->blas, rocblas_operation_none, rocblas_operation_transpose, m, jb, jb, &one,
                             A21, ld, Y, CHOL_BLK, &zero, T, m));
      KMG_HIP(hipMemcpy2DAsync(A21, sizeof(double) * n, T, sizeof(double) * m, sizeof(double) * m, jb,
                               hipMemcpyDeviceToDevice, c->stream));
      // the next block column (its m x jb2 panel, the diagonal block's upper part included:
      // never read), then its diagonal block on the side stream
      const rocblas_int jb2 = std::min<rocblas_int>(CHOL_BLK, m);
      double *A22 = A21 + (size_t)jb * n;
      KMG_BLAS(rocblas_dgemm(c->blas, rocblas_operation_none, rocblas_operation_transpose, m, jb2, jb, &mone,
                             T, m, T, m, &one, A22, ld));
      KMG_HIP(hipEventRecord(c->ev_chol[0], c->stream));
      KMG_HIP(hipStreamWaitEvent(c->chol_stream, c->ev_chol[0], 0));
      KMG_TRY(diag(b + 1, c->chol_stream));
      KMG_HIP(hipEventRecord(c->ev_chol[1], c->chol_stream));
      if (m > jb2) {  // the rest of the trailing triangle
        const rocblas_int mr = m - jb2;
        double *Ar = A22 + jb2 + (size_t)jb2 * n;
        const int np = c->tune.chol_panels;
        if (np <= 0 || mr < 1024) {
          KMG_BLAS(rocblas_dsyrk(c->blas, rocblas_fill_lower, rocblas_operation_none, mr, jb, &mone, T + jb2, m,
                                 &one, Ar, ld));
        } else {  // lower trapezoid as np column panels, one GEMM each (square tops: upper never read)
          const rocblas_int w = (mr + np - 1) / np;
          for (rocblas_int p0 = 0; p0 < mr; p0 += w) {
            const rocblas_int pw = std::min(w, mr - p0);
            KMG_BLAS(rocblas_dgemm(c->blas, rocblas_operation_none, rocblas_operation_transpose, mr - p0, pw, jb,
                                   &mone, T + jb2 + p0, m, T + jb2 + p0, m, &one, Ar + p0 + (size_t)p0 * n, ld));
          }
        }
      }
    }
    return KMG_OK;
  };
  if (const int rc = blocks()) {  // (an error mid-way: no side-stream work outlives the call)
    (void)hipStreamSynchronize(c->chol_stream);
    return rc;
  }
  if (nblk > 1) KMG_HIP(hipStreamWaitEvent(c->stream, c->ev_chol[1], 0));  // the last block
  return KMG_OK;
}

// x = (L L^T)^-1 b in place for chol_factor's L and inverses: a forward sweep into sv_panel
// then a backward sweep back into b, one launch_tri_sweep a block each (rocSOLVER's potrs
// runs two rocBLAS trsv at ~2.3 ms each at n = 9000, latency-bound;
// profiles/r05z_downstream_kernel_stats.csv).
static int chol_solve(kmg_ctx *c, const double *L, int64_t n, double *b) {
  const int64_t nblk = (n + CHOL_BLK - 1) / CHOL_BLK;
  const double *inv = c->sv_inv.as<double>();
  double *y = c->sv_panel.as<double>();
  for (int64_t k = 0; k < nblk; ++k) {  // L y = b (b's trailing rows updated in place)
    const int64_t j0 = k * CHOL_BLK;
    const int jb = (int)std::min<int64_t>(CHOL_BLK, n - j0);
    KMG_HIP(launch_tri_sweep(L, n, inv + 2 * CHOL_BLK * CHOL_BLK * k, j0, jb, 0, b, y, c->stream));
  }
  for (int64_t k = nblk - 1; k >= 0; --k) {  // L^T x = y (y's leading rows updated in place)
    const int64_t j0 = k * CHOL_BLK;
    const int jb = (int)std::min<int64_t>(CHOL_BLK, n - j0);
    KMG_HIP(launch_tri_sweep(L, n, inv + 2 * CHOL_BLK * CHOL_BLK * k + CHOL_BLK * CHOL_BLK, j0, jb, 1, y,
                             b, c->stream));
  }
  return KMG_OK;
}

// Build the system into sv_mat (build()), factorise, solve in place into rhs.
// B = diag(s) K diag(s) + shift I is symmetric when K is, so its row-major image is its
// own column-major image and rocSOLVER's column-major routines apply unchanged; an
// asymmetric K goes straight to LU on the transposed view.
template <typename Build>
static int solve_system(kmg_ctx *c, Build build, int64_t n, double *rhs, bool asym = false) {
  if (n > INT32_MAX / 2) return fail(KMG_EUNSUPPORTED, "n=%lld too large for rocSOLVER", (long long)n);
  const rocblas_int ni = (rocblas_int)n;
  double *B = c->sv_mat.as<double>();
  rocblas_int *info = c->sv_info.as<rocblas_int>();
  rocblas_int *ipiv = info + 4;
  rocblas_int hinfo = 0;
  KMG_TRY(build());
  if (asym) {
    c->last_factor = KMG_FACTOR_LU_ASYMMETRIC;
    KMG_BLAS(rocsolver_dgetrf(c->blas, ni, ni, B, ni, ipiv, info));
    KMG_HIP(hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, c->stream));
    KMG_HIP(hipStreamSynchronize(c->stream));
    if (hinfo != 0) return fail(KMG_ESINGULAR, "Singular matrix");
    KMG_BLAS(rocsolver_dgetrs(c->blas, rocblas_operation_transpose, ni, 1, B, ni, ipiv, rhs, ni));
    return KMG_OK;
  }
  // B is symmetric: either triangle is the matrix (KMG_POTRF_UPPER selects rocSOLVER's
  // upper-triangle variant)
  const bool own = use_own_chol(c);
  const rocblas_fill fill = c->tune.potrf_upper ? rocblas_fill_upper : rocblas_fill_lower;
  if (own)
    KMG_TRY(chol_factor(c, B, n, info));
  else
    KMG_BLAS(rocsolver_dpotrf(c->blas, fill, ni, B, ni, info));
  KMG_HIP(hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  if (hinfo == 0) {
    c->last_factor = KMG_FACTOR_CHOLESKY;
    if (own)
      KMG_TRY(chol_solve(c, B, n, rhs));
    else
      KMG_BLAS(rocsolver_dpotrs(c->blas, fill, ni, 1, B, ni, rhs, ni));
    return KMG_OK;
  }
  c->last_factor = KMG_FACTOR_LU_INDEFINITE;
  KMG_TRY(build());  // not positive definite: rebuild and use LU, like inv()
  KMG_BLAS(rocsolver_dgetrf(c->blas, ni, ni, B, ni, ipiv, info));
  KMG_HIP(hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  if (hinfo != 0) return fail(KMG_ESINGULAR, "Singular matrix");
  // B holds the row-major A, i.e. A^T in column-major terms: solve A^T^T x = rhs
  KMG_BLAS(rocsolver_dgetrs(c->blas, rocblas_operation_transpose, ni, 1, B, ni, ipiv, rhs, ni));
  return KMG_OK;
}

static int solver_workspace(kmg_ctx *c, int64_t n, size_t nvec) {
  KMG_TRY(blas_handle(c));
  KMG_TRY(c->sv_mat.ensure(sizeof(double) * (size_t)n * (size_t)n));
  KMG_TRY(c->sv_vec.ensure(sizeof(double) * (size_t)n * nvec + 64));
  KMG_TRY(c->sv_info.ensure(sizeof(rocblas_int) * ((size_t)n + 8)));
  return KMG_OK;
}

static int krr_run(kmg_ctx *c, const double *d_K, int64_t ld, int64_t n, const double *d_y,
                   double lambda, double *d_alpha) {
  KMG_TRY(solver_workspace(c, n, 0));
  StageTimer t(c, ST_SOLVE);
  KMG_HIP(hipMemcpyAsync(d_alpha, d_y, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice,
                         c->stream));
  const double shift = lambda * (double)n;  // self.lbda * self.n (KRR.py:33)
  auto build = [&]() -> int {
    KMG_HIP(launch_shift_scale(d_K, ld, nullptr, shift, nullptr, n, c->sv_mat.as<double>(), n, c->stream));
    return KMG_OK;
  };
  bool asym = false;
  KMG_TRY(is_asymmetric(c, d_K, ld, n, &asym));
  return solve_system(c, build, n, d_alpha, asym);
}

static int klr_run(kmg_ctx *c, const double *d_K, int64_t ld, int64_t n, const double *d_y,
                   double lambda, double tol, int32_t maxiter, double *d_alpha, int32_t *iters) {
  KMG_TRY(solver_workspace(c, n, 5));
  StageTimer t(c, ST_SOLVE);
  double *prev = c->sv_vec.as<double>(), *m = prev + n, *s = m + n, *rhs = s + n;
  double *cur = rhs + n, *dsum = cur + n;
  KMG_HIP(hipMemsetAsync(prev, 0, sizeof(double) * (size_t)n, c->stream));
  const double shift = (double)n * lambda;  // self.n * self.lbda (KLR.py:53)
  const double one = 1.0, zero = 0.0;
  auto build = [&]() -> int {
    KMG_HIP(launch_shift_scale(d_K, ld, s, shift, nullptr, n, c->sv_mat.as<double>(), n, c->stream));
    return KMG_OK;
  };
  bool asym = false;
  KMG_TRY(is_asymmetric(c, d_K, ld, n, &asym));
  double diff = INFINITY;
  int32_t it = 0;
  for (int32_t r = 0; r < maxiter; ++r) {
    if (!(diff > tol)) continue;  // the reference keeps looping without work (KLR.py:68-69)
    // m = K . alpha_prev: row-major K is K^T column-major, so apply the transpose
    KMG_BLAS(rocblas_dgemv(c->blas, rocblas_operation_transpose, (rocblas_int)n, (rocblas_int)n,
                           &one, d_K, (rocblas_int)ld, prev, 1, &zero, m, 1));
    KMG_HIP(launch_irls(m, d_y, n, s, rhs, c->stream));
    KMG_TRY(solve_system(c, build, n, rhs, asym));
    KMG_HIP(launch_scale_diff(s, rhs, prev, n, cur, dsum, c->stream));
    double h = 0.0;
    KMG_HIP(hipMemcpyAsync(&h, dsum, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    KMG_HIP(hipMemcpyAsync(prev, cur, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice,
                           c->stream));
    KMG_HIP(hipStreamSynchronize(c->stream));
    diff = std::sqrt(h);
    ++it;
  }
  KMG_HIP(hipMemcpyAsync(d_alpha, prev, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice,
                         c->stream));
  if (iters) *iters = it;
  return KMG_OK;
}


// C_SVM.fit (SVM.py:78-89): min 1/2 a'Ka - y'a, 0 <= y_i a_i <= C, by the primal-dual
// interior-point iteration of kmg_solve.hip; one factorisation and two solves per step.
static int svm_run(kmg_ctx *c, const double *d_K, int64_t ld, int64_t n, const double *d_y,
                   double C, double tol, int32_t maxiter, double *d_alpha, int32_t *iters,
                   double *objective) {
  KMG_TRY(blas_handle(c));
  KMG_TRY(c->sv_mat.ensure(sizeof(double) * (size_t)n * (size_t)n));
  KMG_TRY(c->sv_vec.ensure(sizeof(double) * ((size_t)n * KMG_SVM_NVEC + 16)));
  KMG_TRY(c->sv_info.ensure(sizeof(rocblas_int) * ((size_t)n + 8)));
  if (n > INT32_MAX / 2) return fail(KMG_EUNSUPPORTED, "n=%lld too large for rocSOLVER", (long long)n);
  StageTimer t(c, ST_SOLVE);
  const rocblas_int ni = (rocblas_int)n;
  double *vec = c->sv_vec.as<double>(), *sc = vec + (size_t)n * KMG_SVM_NVEC;
  double *v = vec + (size_t)n * KMG_SVM_V, *u = vec + (size_t)n * KMG_SVM_U;
  double *rhs = vec + (size_t)n * KMG_SVM_RHS, *D = vec + (size_t)n * 4;
  double *B = c->sv_mat.as<double>();
  rocblas_int *info = c->sv_info.as<rocblas_int>(), *ipiv = info + 4;
  const double one = 1.0, zero = 0.0;
  double h[3] = {0, 0, 0};
  auto residual = [&]() -> int {
    KMG_HIP(launch_svm(1, d_y, n, C, vec, sc, nullptr, c->stream));
    KMG_BLAS(rocblas_dgemv(c->blas, rocblas_operation_transpose, ni, ni, &one, d_K,
                           (rocblas_int)ld, v, 1, &zero, u, 1));
    KMG_HIP(launch_svm(2, d_y, n, C, vec, sc, nullptr, c->stream));
    KMG_HIP(hipMemcpyAsync(h, sc, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    KMG_HIP(hipStreamSynchronize(c->stream));
    return KMG_OK;
  };
  KMG_HIP(launch_svm(0, d_y, n, C, vec, sc, nullptr, c->stream));
  int32_t it = 0;
  for (; it < maxiter; ++it) {
    KMG_TRY(residual());
    const double gap = 2.0 * (double)n * h[0];
    if (gap <= tol * std::max(1.0, std::fabs(h[2])) && h[1] <= tol) break;
    // M = YKY + diag(D), factorised once, solved for the predictor and the corrector
    KMG_HIP(launch_shift_scale(d_K, ld, d_y, 0.0, D, n, B, n, c->stream));
    const bool own = use_own_chol(c);
    if (own)
      KMG_TRY(chol_factor(c, B, n, info));
    else
      KMG_BLAS(rocsolver_dpotrf(c->blas, rocblas_fill_lower, ni, B, ni, info));
    rocblas_int hinfo = 0;
    KMG_HIP(hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, c->stream));
    KMG_HIP(hipStreamSynchronize(c->stream));
    bool lu = false;
    if (hinfo != 0) {  // K not numerically PSD: LU on the same system
      KMG_HIP(launch_shift_scale(d_K, ld, d_y, 0.0, D, n, B, n, c->stream));
      KMG_BLAS(rocsolver_dgetrf(c->blas, ni, ni, B, ni, ipiv, info));
      KMG_HIP(hipMemcpyAsync(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost, c->stream));
      KMG_HIP(hipStreamSynchronize(c->stream));
      if (hinfo != 0) return fail(KMG_ESINGULAR, "Singular KKT system");
      lu = true;
    }
    auto solve = [&]() -> int {
      if (lu)
        KMG_BLAS(rocsolver_dgetrs(c->blas, rocblas_operation_transpose, ni, 1, B, ni, ipiv, rhs, ni));
      else if (own)
        KMG_TRY(chol_solve(c, B, n, rhs));
      else
        KMG_BLAS(rocsolver_dpotrs(c->blas, rocblas_fill_lower, ni, 1, B, ni, rhs, ni));
      return KMG_OK;
    };
    KMG_TRY(solve());
    KMG_HIP(launch_svm(3, d_y, n, C, vec, sc, nullptr, c->stream));
    KMG_TRY(solve());
    KMG_HIP(launch_svm(4, d_y, n, C, vec, sc, nullptr, c->stream));
  }
  if (it == maxiter) KMG_TRY(residual());  // objective of the last iterate
  KMG_HIP(launch_svm(5, d_y, n, C, vec, sc, d_alpha, c->stream));
  if (iters) *iters = it;
  if (objective) *objective = h[2];
  return KMG_OK;
}

static int check_solver(kmg_ctx *c, const void *K, int64_t n, int64_t ld, const void *y,
                        const void *alpha) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  if (n < 0 || (n > 0 && ld < n)) return fail(KMG_EINVAL, "bad matrix shape");
  if (n > 0 && (!K || !y || !alpha)) return fail(KMG_EINVAL, "NULL buffer");
  return KMG_OK;
}

// host K / y -> device (K into sv staging cmb_k, y and alpha into cmb_vec)
static int stage_solver_inputs(kmg_ctx *c, const double *K, int64_t ld, int64_t n,
                               const double *y, double **dK, double **dy, double **da) {
  KMG_TRY(c->cmb_k.ensure(sizeof(double) * (size_t)n * (size_t)n));
  KMG_TRY(c->cmb_vec.ensure(sizeof(double) * 2 * (size_t)n));
  *dK = c->cmb_k.as<double>();
  *dy = c->cmb_vec.as<double>();
  *da = *dy + n;
  KMG_HIP(hipMemcpy2DAsync(*dK, n * 8, K, ld * 8, n * 8, n, hipMemcpyHostToDevice, c->stream));
  KMG_HIP(hipMemcpyAsync(*dy, y, sizeof(double) * (size_t)n, hipMemcpyHostToDevice, c->stream));
  return KMG_OK;
}

extern "C" {

int kmg_krr_solve_device(kmg_ctx *c, const double *d_K, int64_t ld, int64_t n, const double *d_y,
                         double lambda, double *d_alpha) {
  KMG_TRY(check_solver(c, d_K, n, ld, d_y, d_alpha));
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  if (n == 0) return KMG_OK;
  return krr_run(c, d_K, ld, n, d_y, lambda, d_alpha);
}

int kmg_krr_solve(kmg_ctx *c, const double *K, int64_t ld, int64_t n, const double *y,
                  double lambda, double *alpha) {
  KMG_TRY(check_solver(c, K, n, ld, y, alpha));
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  if (n == 0) return KMG_OK;
  double *dK, *dy, *da;
  KMG_TRY(stage_solver_inputs(c, K, ld, n, y, &dK, &dy, &da));
  KMG_TRY(krr_run(c, dK, n, n, dy, lambda, da));
  KMG_HIP(hipMemcpyAsync(alpha, da, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

int kmg_klr_fit_device(kmg_ctx *c, const double *d_K, int64_t ld, int64_t n, const double *d_y,
                       double lambda, double tol, int32_t maxiter, double *d_alpha,
                       int32_t *iters) {
  KMG_TRY(check_solver(c, d_K, n, ld, d_y, d_alpha));
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  if (iters) *iters = 0;
  if (n == 0) return KMG_OK;
  return klr_run(c, d_K, ld, n, d_y, lambda, tol, maxiter, d_alpha, iters);
}

int kmg_klr_fit(kmg_ctx *c, const double *K, int64_t ld, int64_t n, const double *y,
                double lambda, double tol, int32_t maxiter, double *alpha, int32_t *iters) {
  KMG_TRY(check_solver(c, K, n, ld, y, alpha));
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  if (iters) *iters = 0;
  if (n == 0) return KMG_OK;
  double *dK, *dy, *da;
  KMG_TRY(stage_solver_inputs(c, K, ld, n, y, &dK, &dy, &da));
  KMG_TRY(klr_run(c, dK, n, n, dy, lambda, tol, maxiter, da, iters));
  KMG_HIP(hipMemcpyAsync(alpha, da, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

int kmg_svm_fit_device(kmg_ctx *c, const double *d_K, int64_t ld, int64_t n, const double *d_y,
                       double C, double tol, int32_t maxiter, double *d_alpha, int32_t *iters,
                       double *objective) {
  KMG_TRY(check_solver(c, d_K, n, ld, d_y, d_alpha));
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  if (iters) *iters = 0;
  if (objective) *objective = 0.0;
  if (!(C > 0)) return fail(KMG_EINVAL, "C must be > 0");
  if (n == 0) return KMG_OK;
  return svm_run(c, d_K, ld, n, d_y, C, tol, maxiter, d_alpha, iters, objective);
}

int kmg_svm_fit(kmg_ctx *c, const double *K, int64_t ld, int64_t n, const double *y, double C,
                double tol, int32_t maxiter, double *alpha, int32_t *iters, double *objective) {
  KMG_TRY(check_solver(c, K, n, ld, y, alpha));
  std::lock_guard<std::mutex> lk(c->mu);
  KMG_HIP(hipSetDevice(c->device));
  if (iters) *iters = 0;
  if (objective) *objective = 0.0;
  if (!(C > 0)) return fail(KMG_EINVAL, "C must be > 0");
  if (n == 0) return KMG_OK;
  for (int64_t i = 0; i < n; ++i)
    if (y[i] != 1.0 && y[i] != -1.0) return fail(KMG_EINVAL, "labels must be -1 or 1");
  double *dK, *dy, *da;
  KMG_TRY(stage_solver_inputs(c, K, ld, n, y, &dK, &dy, &da));
  KMG_TRY(svm_run(c, dK, n, n, dy, C, tol, maxiter, da, iters, objective));
  KMG_HIP(hipMemcpyAsync(alpha, da, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  KMG_HIP(hipStreamSynchronize(c->stream));
  return KMG_OK;
}

// ------------------------------------------------------------------ RCCL
int kmg_comm_unique_id(uint8_t id[128]) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return fail(KMG_ERCCL, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  memcpy(id, &u, 128);
  return KMG_OK;
}

int kmg_comm_init(kmg_ctx *c, const uint8_t id[128], int32_t nranks, int32_t rank) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  KMG_HIP(hipSetDevice(c->device));
  ncclUniqueId u;
  memcpy(&u, id, 128);
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) return fail(KMG_ERCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
  c->nranks = nranks;
  c->rank = rank;
  return KMG_OK;
}

int kmg_allgather_rows(kmg_ctx *c, void *d_K, int64_t n, int64_t ld, int32_t dt,
                       const int64_t *splits) {
  if (!c || !c->comm) return fail(KMG_EINVAL, "communicator not initialised");
  if (!splits) return fail(KMG_EINVAL, "splits is NULL");
  if (!d_K && n > 0) return fail(KMG_EINVAL, "d_K is NULL");
  if (dt != KMG_I32 && dt != KMG_F32 && dt != KMG_F64) return fail(KMG_EINVAL, "unknown dtype %d", dt);
  if (n < 0 || (n > 0 && ld < n)) return fail(KMG_EINVAL, "ld < n");
  // rank r owns rows [splits[r], splits[r+1]): 0 = splits[0] <= ... <= splits[nranks] = n
  if (splits[0] != 0 || splits[c->nranks] != n)
    return fail(KMG_EINVAL, "splits must start at 0 and end at n");
  for (int q = 0; q < c->nranks; ++q)
    if (splits[q + 1] < splits[q]) return fail(KMG_EINVAL, "splits must be non-decreasing");
  KMG_HIP(hipSetDevice(c->device));
  const size_t esz = dtype_size(dt);
  // rows of rank r are contiguous ([splits[r], splits[r+1]) x ld): an all-gather with
  // per-rank counts = one broadcast per root, issued as one RCCL group.
  ncclResult_t r = ncclGroupStart();
  for (int q = 0; q < c->nranks && r == ncclSuccess; ++q) {
    const int64_t a = splits[q], b = splits[q + 1];
    if (b <= a) continue;
    char *base = (char *)d_K + (size_t)a * ld * esz;
    r = ncclBroadcast(base, base, (size_t)(b - a) * ld * esz, ncclChar, q, c->comm, c->stream);
  }
  ncclResult_t r2 = ncclGroupEnd();
  if (r != ncclSuccess || r2 != ncclSuccess)
    return fail(KMG_ERCCL, "ncclBroadcast group: %s",
                ncclGetErrorString(r != ncclSuccess ? r : r2));
  return KMG_OK;
}

int kmg_comm_destroy(kmg_ctx *c) {
  if (!c) return fail(KMG_EINVAL, "ctx is NULL");
  if (c->comm) ncclCommDestroy(c->comm);
  c->comm = nullptr;
  c->nranks = 1;
  c->rank = 0;
  return KMG_OK;
}

}  // extern "C"
