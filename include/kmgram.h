/*
 * kmgram.h — C ABI of libkmgram.so, the MI355X (gfx950) string-kernel Gram engine.
 *
 * This is the drop-in boundary for the Gram-matrix hot path of
 * afiliot/Kernel-Methods-For-Genomics `kernels.py`.  The reference boundary is
 * pure Python (`kernels.select_method(X, method) -> np.ndarray`, kernels.py:461-505);
 * its Python mirror (`kernel-methods-for-genomics_amd/kernels.py`) calls the
 * entry points below through ctypes.  Every entry point cites the reference
 * interface it replaces.
 *
 * Conventions
 *   - Status: every function returns int; 0 (KMG_OK) on success.  No C++ exception
 *     or abort crosses the ABI.  kmg_last_error() gives a thread-local message.
 *   - Sequences enter as symbol codes, uint8 [n][ldc] row-major, plus int32 lengths.
 *     'A','C','G','T' -> 0,1,2,3.  Any other character -> a code >= 4 (distinct
 *     characters get distinct codes, so WD/WDS/SS character equality is preserved;
 *     spectrum treats codes >= 4 as "k-mer matches no beta", kernels.py:21-24).
 *   - Ownership: the caller owns every buffer it passes.  The context owns all
 *     device workspace and keeps no caller pointer after a call returns.
 *   - Threading: a context is not re-entrant (internal mutex); one context per
 *     device; one process per GPU for multi-GPU (RCCL communicator per context).
 */
#ifndef KMGRAM_H
#define KMGRAM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMG_ABI_VERSION 1

/* status codes */
enum {
  KMG_OK = 0,
  KMG_EINVAL = 1,       /* bad argument (shape, range, alphabet) */
  KMG_EUNSUPPORTED = 2, /* parameter combination not implemented on device */
  KMG_EHIP = 3,         /* HIP runtime error */
  KMG_ENOMEM = 4,       /* device allocation failed */
  KMG_ERCCL = 5,        /* RCCL error */
  KMG_ENODEV = 6,       /* no HIP device visible */
  KMG_ESINGULAR = 7,    /* dense learner: the system matrix is singular (LinAlgError) */
  KMG_EINTERNAL = 8     /* an internal consistency check failed (KMG_CHECK=1: the neighbourhood
                           lists' metadata after a fill); nothing past the check was launched */
};

/* kernel families (one per reference get_*_K) */
enum {
  KMG_SPECTRUM = 1,   /* get_spectrum_K   kernels.py:28-47   */
  KMG_MISMATCH = 2,   /* get_mismatch_K   kernels.py:196-217 */
  KMG_WD = 3,         /* get_WD_K         kernels.py:84-101  */
  KMG_WDS = 4,        /* get_WDShifts_K   kernels.py:138-155 */
  KMG_SUBSTRING = 5,  /* get_string_K     kernels.py:367-382 */
  KMG_LOCALALIGN = 6, /* get_LA_K         kernels.py:273-302 */
  KMG_GAPPY = 7       /* get_gappy_K      kernels.py:436-455 (la_mode KMG_MODE_REFERENCE: the
                         reference's behaviour, defined for k=1,g=0 -- every other (k,g) raises
                         there under numpy 2; KMG_MODE_INTENDED: any 0 <= g < k,
                         k <= 15, k-g <= 8) */
};

/* output element types */
enum { KMG_I32 = 1, KMG_F32 = 2, KMG_F64 = 3 };

/* semantics modes (kmg_params.la_mode; LA and GP) */
enum { KMG_LA_REFERENCE = 0 /* bit-for-bit the reference: all zeros (kernels.py:238,262) */,
       KMG_LA_INTENDED = 1  /* five DP arrays (no aliasing), cells up to [n_x, n_y] on
                               x[i-1], y[j-1], gap factors exp(-beta e) / exp(-beta d):
                               kernels.py:226-270 as meant; parity unpinned */ };
enum { KMG_MODE_REFERENCE = 0 /* the reference's behaviour (GP: k=1,g=0 only) */,
       KMG_MODE_INTENDED = 1  /* GP: binary (k-g)-mer presence over the gapped subsequences
                                 of every 101-window k-mer, normalised (kernels.py:420-455 as
                                 report §3.7 describes it); parity unpinned */,
       KMG_MODE_SS_B = 2      /* SS: the auxiliary B_k(lbda, k, x, y) of the recursion
                                 (kernels.py:322-342) at the full prefixes instead of
                                 K_k (kernels.py:344-364); rows <= 127 symbols */ };

#define KMG_MAX_COEF 64

typedef struct kmg_params {
  int32_t kind;      /* KMG_* family */
  int32_t k;         /* SP/MM/GP k-mer length; SS subsequence length */
  int32_t m;         /* MM maximal mismatches */
  int32_t d;         /* WD/WDS maximal degree */
  int32_t S;         /* WDS maximal shift */
  int32_t g;         /* GP gap */
  int32_t window;    /* MM/GP: fixed window the reference hard-codes (101, kernels.py:171,430) */
  int32_t normalize; /* 1: fused normalize_K epilogue (kernels.py:398-415) */
  int32_t smith;     /* LA: 1 = Smith_Waterman max form */
  int32_t la_mode;   /* LA: KMG_LA_REFERENCE / KMG_LA_INTENDED; GP: KMG_MODE_* */
  int32_t span;      /* WD/WDS: summation length L of get_WD_d / get_WDShifts_d (kernels.py:64,
                        115); 0 = len(x) of the smaller-index row, as get_*_K pass it */
  int32_t reserved[5];
  double lambda;     /* SS lambda */
  double lambda2;    /* SS lambda**2 exactly as the host language computes it */
  double la_e, la_d, la_beta; /* LA gap open / extend / beta */
  double coef_a[KMG_MAX_COEF]; /* WD/WDS: beta_k for k=1..d at [k-1] (kernels.py:53-61) */
  double coef_b[KMG_MAX_COEF]; /* WDS: delta_s for s=0..S at [s]   (kernels.py:106-112) */
  double diag_value; /* WD: the closed-form diagonal L-1+(1-d)/3 (kernels.py:96); NaN = per row */
} kmg_params;

typedef struct kmg_ctx kmg_ctx;

int kmg_version(void);
const char *kmg_last_error(void);
int kmg_device_count(int *n);

/* Create a context bound to one HIP device (one stream, workspace arena). */
int kmg_create(kmg_ctx **ctx, int device_id);
int kmg_destroy(kmg_ctx *ctx);

/*
 * Full Gram matrix, host buffers in and out (drop-in path).
 * Replaces kernels.select_method / get_*_K (kernels.py:461-505 and the functions it
 * dispatches to).  out: n x n, row stride ld_out elements, dtype out_dtype.
 */
int kmg_gram(kmg_ctx *ctx, const kmg_params *p, const uint8_t *codes, const int32_t *lens,
             int64_t n, int64_t ldc, int32_t out_dtype, void *out, int64_t ld_out);

/*
 * Device-resident Gram rows [row0, row1) x all n columns (bench / multi-GPU path).
 * d_codes/d_lens/d_out are device pointers (kmg_dmalloc).  d_out points at row row0.
 * Runs on the context stream; returns without synchronising.
 */
int kmg_gram_device(kmg_ctx *ctx, const kmg_params *p, const uint8_t *d_codes,
                    const int32_t *d_lens, int64_t n, int64_t ldc, int64_t row0, int64_t row1,
                    int32_t out_dtype, void *d_out, int64_t ld_out);

/*
 * Device-resident column block: K[i][col0 + j] for every row i in [0, n) and j in
 * [0, col1 - col0), at d_out[i * ld_out + j].  K is symmetric, so this is the row slab
 * [col0, col1) x all n transposed: one GPU's 1/G share of a sharded build (the pair loops
 * of kernels.py:211-215 split by columns), with the neighbourhood lists built over the
 * block's sequences only -- each list read by all n rows.  Mismatch (k, 1), 4 <= k <= 12
 * (get_mismatch_K, kernels.py:196-217), and the spectrum posting-list path (get_spectrum_K,
 * kernels.py:28-47, 6 <= k <= 12: the posting index over the block's sequences only); other
 * kernels return KMG_EUNSUPPORTED.  Runs on the context stream; returns without synchronising.
 */
int kmg_gram_device_cols(kmg_ctx *ctx, const kmg_params *p, const uint8_t *d_codes,
                         const int32_t *d_lens, int64_t n, int64_t ldc, int64_t col0,
                         int64_t col1, int32_t out_dtype, void *d_out, int64_t ld_out);

/*
 * The full K of all n rows into HOST memory h_out (row stride ld_host elements; e.g. a
 * memory-mapped .npy), built on the device in slabs of slab_rows rows: the posting index /
 * features / diagonal are built once for all slabs, and slab t's device-to-host copy (a
 * second stream) overlaps slab t+1's Gram.  The slab unit of utils.get_training_datas'
 * K cache at N >= 100k (utils.py:139-155, select_method kernels.py:461-505).  Returns
 * after the last copy has landed.
 */
int kmg_gram_to_host(kmg_ctx *ctx, const kmg_params *p, const uint8_t *d_codes,
                     const int32_t *d_lens, int64_t n, int64_t ldc, int32_t out_dtype,
                     int64_t slab_rows, void *h_out, int64_t ld_host);

/*
 * Feature vectors of n sequences over caller-chosen k-mer columns (host buffers): the
 * reference's per-sequence feature maps, evaluated on the device.  out[i][j] (float64, row
 * stride ld_out) for column code cols[j] (base-4 k-mer, first letter most significant, the
 * index of ''.join(c) in itertools.product('ACGT', repeat=k); 0xFFFFFFFF = a beta no window
 * can equal, value 0):
 *   KMG_SPECTRUM  get_phi_u(x, k, betas)      kernels.py:12-25: windows range(len(x)-k+1)
 *                 equal to the beta (a window holding a non-ACGT symbol equals none)
 *   KMG_MISMATCH  get_phi_km(x, k, m, betas)  kernels.py:161-175: windows range(window-k+1)
 *                 (window = 101) within Hamming distance m of the beta, a non-ACGT symbol
 *                 mismatching every letter; rows shorter than the window are KMG_EINVAL
 *                 (the reference raises while broadcasting the short k-mer)
 *   KMG_GAPPY     gappy_k(x, 1, 0, betas)     kernels.py:420-433 (k=1, g=0): 1.0 when the
 *                 letter occurs in x[0:window], else 0.0
 * k <= 16.
 */
int kmg_features(kmg_ctx *ctx, const kmg_params *p, const uint8_t *codes, const int32_t *lens,
                 int64_t n, int64_t ldc, const uint32_t *cols, int64_t ncols, double *out,
                 int64_t ld_out);

/*
 * kmg_features over SYMBOL columns: column j is cols[16 j .. 16 j + k), k symbol codes in the
 * code space of `codes` (any uint8 but the padding code 255), so every symbol compares by
 * identity: get_phi_u(x, k, betas) with betas holding letters outside A/C/G/T (string
 * equality, kernels.py:23-24: the beta 'GTN' counts the windows 'GTN'), get_phi_km(x, k, m,
 * betas) with format()ed values outside 1..4 in x or in the betas (integer comparison,
 * kernels.py:174).  KMG_SPECTRUM or KMG_MISMATCH only.  flags KMG_FEATURES_BCAST (mismatch):
 * rows shorter than the window take numpy's broadcasting of their short k-mers -- a 1-symbol
 * window compares that symbol against every letter of the beta, an empty one (k = 1) counts
 * with 0 mismatches -- and a row whose short windows would not broadcast is KMG_EINVAL (the
 * reference raises).  Note: the Gram paths (kmg_gram, KMG_MISMATCH) give a window holding a
 * non-ACGT symbol weight 0, where get_phi_km counts the symbol as one mismatch; the reference's
 * get_mismatch_K never meets such a window (format() raises on letters outside A/C/G/T,
 * kernels.py:193), so that Gram case has no reference counterpart (parity unpinned).
 */
#define KMG_FEATURES_BCAST 1
int kmg_features_sym(kmg_ctx *ctx, const kmg_params *p, const uint8_t *codes, const int32_t *lens,
                     int64_t n, int64_t ldc, const uint8_t *cols, int64_t ncols, int32_t flags,
                     double *out, int64_t ld_out);

/* normalize_K (kernels.py:398-415) in place on a host float64 matrix, including the
 * "K[0,0]==1 -> unchanged" rule (returns 1 in *skipped then). */
int kmg_normalize(kmg_ctx *ctx, double *K, int64_t n, int64_t ld, int32_t *skipped);

/* center_K (kernels.py:387-395): out = (I - 11^T/n) K (I - 11^T/n), float64 host buffers. */
int kmg_center(kmg_ctx *ctx, const double *K, int64_t ldk, double *out, int64_t ld_out, int64_t n);

/*
 * Kernel-combination consumers of the Gram matrices (the callers of the Gram path in
 * run.py / main.py).  K is an array of p pointers to n x n float64 matrices (row stride
 * ld), p <= 12.  The plain functions take host buffers (copied in, result copied out);
 * the _device functions take device pointers for everything (K, u, alpha, y and the
 * outputs), e.g. Grams produced by kmg_gram_device, and return without synchronising.
 */
/* NLCK.svm_step / NLCK.get_K (NLCKernels.py:52, 97): out = (sum_m u[m] K_m) ** degree */
int kmg_combine(kmg_ctx *ctx, const double *const *K, int32_t p, const double *u, int32_t degree,
                int64_t n, int64_t ld, double *out, int64_t ld_out);
int kmg_combine_device(kmg_ctx *ctx, const double *const *d_K, int32_t p, const double *d_u,
                       int32_t degree, int64_t n, int64_t ld, double *d_out, int64_t ld_out);
/* NLCK.grad (NLCKernels.py:61-66): grad[m] = -degree * alpha^T (K_t o K_m) alpha,
 * K_t = (sum_m u[m] K_m) ** (degree - 1) */
int kmg_nlck_grad(kmg_ctx *ctx, const double *const *K, int32_t p, const double *u,
                  int32_t degree, const double *alpha, int64_t n, int64_t ld, double *grad);
int kmg_nlck_grad_device(kmg_ctx *ctx, const double *const *d_K, int32_t p, const double *d_u,
                         int32_t degree, const double *d_alpha, int64_t n, int64_t ld,
                         double *d_grad);
/* ALIGNF.get_a / ALIGNF.get_M (ALIGNF.py:43-58) on Kc_m = center_K(K_m) (kernels.py:387-395):
 * a[m] = sum(Kc_m * outer(y, y)), M[l][m] = sum(Kc_l * Kc_m) (p x p, symmetric) */
int kmg_alignf(kmg_ctx *ctx, const double *const *K, int32_t p, const double *y, int64_t n,
               int64_t ld, double *a, double *M);
/* device form: out = a[0..p) followed by the upper triangle of M row by row (l <= m) */
int kmg_alignf_device(kmg_ctx *ctx, const double *const *d_K, int32_t p, const double *d_y,
                      int64_t n, int64_t ld, double *d_out);

/*
 * Dense learners on a Gram matrix.  K: n x n float64, row stride ld.
 * The system is factorised on the device (blocked Cholesky of kmg_solve.hip -- rocSOLVER
 * potrf with KMG_CHOL=0 --, rocSOLVER LU with partial pivoting if it is not positive
 * definite); KMG_ESINGULAR where np.linalg.inv raises LinAlgError.
 */
/* KRR.fit (KRR.py:33): alpha = inv(K + lambda * n * I) . y */
int kmg_krr_solve(kmg_ctx *ctx, const double *K, int64_t ld, int64_t n, const double *y,
                  double lambda, double *alpha);
int kmg_krr_solve_device(kmg_ctx *ctx, const double *d_K, int64_t ld, int64_t n,
                         const double *d_y, double lambda, double *d_alpha);
/* KLR.fit (KLR.py:30-75): IRLS from alpha = 0; each step m = K.alpha, W = s(m)s(-m),
 * z = m + y / s(-y m), alpha = W^1/2 inv(W^1/2 K W^1/2 + n lambda I) W^1/2 z, repeated
 * while ||alpha - alpha_prev||_2 > tol, at most maxiter times; iters = steps taken */
int kmg_klr_fit(kmg_ctx *ctx, const double *K, int64_t ld, int64_t n, const double *y,
                double lambda, double tol, int32_t maxiter, double *alpha, int32_t *iters);
int kmg_klr_fit_device(kmg_ctx *ctx, const double *d_K, int64_t ld, int64_t n,
                       const double *d_y, double lambda, double tol, int32_t maxiter,
                       double *d_alpha, int32_t *iters);

/* C_SVM.fit, solver 'CVX' (SVM.py:78-89): the QP cvxopt.solvers.qp(P=K, q=-y,
 * G=[diag(y); -diag(y)], h=[C; 0]) = min 1/2 a'Ka - y'a s.t. 0 <= y_i a_i <= C (y in {-1,1}),
 * by a Mehrotra predictor-corrector interior-point method; stops when the duality gap
 * <= tol * max(1, |objective|) and ||dual residual||_inf <= tol (or after maxiter steps).
 * iters = steps taken, objective = 1/2 a'Ka - y'a at the returned a. */
int kmg_svm_fit(kmg_ctx *ctx, const double *K, int64_t ld, int64_t n, const double *y, double C,
                double tol, int32_t maxiter, double *alpha, int32_t *iters, double *objective);
int kmg_svm_fit_device(kmg_ctx *ctx, const double *d_K, int64_t ld, int64_t n,
                       const double *d_y, double C, double tol, int32_t maxiter,
                       double *d_alpha, int32_t *iters, double *objective);

/*
 * Multi-GPU full-K build ("the N x N tile space shards across the GPUs with a
 * final RCCL all-gather over xGMI").  Rows are dealt block-cyclically: with `block` rows a
 * block, round t holds rows [t*R, (t+1)*R), R = nranks * block, and rank r computes the
 * block [t*R + r*block, +block) of every round (clipped to n).  The index is built once;
 * the Gram kernel runs once per round.  gather = 1: as soon as a round's block is enqueued,
 * the round is all-gathered IN PLACE (ncclAllGather(send = recv + rank*count), one
 * contiguous R-row slab) on a second stream, overlapped with the next round's Gram kernel;
 * when the call's work completes (context-stream order) every rank holds the full K.
 * d_out: n_pad x ld_out elements, n_pad = kmg_rows_padded(n, nranks, block) (the padding
 * rows of the last round travel but are never written by a kernel); gather = 0 writes only
 * this rank's blocks and needs n rows.  gather = 2 (upper triangle): round t
 * computes only the columns >= t*R of its rows into a contiguous round slab, the slab is
 * all-gathered in place (half the xGMI bytes of gather = 1) and every rank copies it into
 * K and mirrors it into the lower triangle locally (K[x][t*R + y] = K[t*R + y][x]).
 * gather = 3: the gather = 2 layout with every rank's blocks computed on this GPU (a
 * one-GPU rehearsal of the multi-rank assembly; no RCCL).  gather = 4: like 0 (no data-path
 * collective) with this rank's blocks packed: row t*block + y of d_out holds row
 * t*R + rank*block + y of K (d_out needs ceil(n / R) * block rows: a rank's share of a K
 * that no single GPU could hold).  gather = 5 (column blocks, mismatch (k, 1) with 4 <= k <= 12
 * only, KMG_EUNSUPPORTED otherwise): one round, nranks * block >= n; rank r computes the column
 * block K[:, C_r], C_r = [r*block, min(n, (r+1)*block)), with the neighbourhood lists built over
 * its own |C_r| sequences (kmg_gram_device_cols), transposes it into K's rows C_r (K is
 * symmetric) and the slabs are all-gathered in place over RCCL; d_out holds nranks * block rows.
 * gather = 6: the gather = 5 layout with every rank's block computed on this GPU (no RCCL).
 * gather = 1, 2 or 5 with nranks > 1 needs kmg_comm_init with the same nranks / rank.  Replaces the whole-matrix pair loops of get_spectrum_K /
 * get_mismatch_K (kernels.py:41-45, 211-215) split over GPUs.
 */
int64_t kmg_rows_padded(int64_t n, int32_t nranks, int64_t block);
int kmg_gram_blocks(kmg_ctx *ctx, const kmg_params *p, const uint8_t *d_codes,
                    const int32_t *d_lens, int64_t n, int64_t ldc, int32_t out_dtype, void *d_out,
                    int64_t ld_out, int32_t nranks, int32_t rank, int64_t block, int32_t gather);
/* Bytes per slab element the last kmg_gram_blocks call sent over the all-gather (gather 2/3:
 * 1 = uint8 counts, 2 = uint16, else the output dtype's size; gather 0/1: the output's). */
int kmg_gram_blocks_wire(kmg_ctx *ctx);

/* Re-read the KMG_* tuning variables of the environment (read once at kmg_create). */
int kmg_reload_tuning(kmg_ctx *ctx);

/* device memory / stream helpers for device-resident callers */
int kmg_dmalloc(kmg_ctx *ctx, void **ptr, size_t bytes);
int kmg_dfree(kmg_ctx *ctx, void *ptr);
int kmg_h2d(kmg_ctx *ctx, void *dst, const void *src, size_t bytes);
int kmg_d2h(kmg_ctx *ctx, void *dst, const void *src, size_t bytes);
int kmg_memset(kmg_ctx *ctx, void *dst, int value, size_t bytes);
int kmg_synchronize(kmg_ctx *ctx);
int kmg_stream(kmg_ctx *ctx, void **hip_stream);

/* Per-stage device timings from HIP events recorded on the context stream around
 * every launch while timing is enabled (kmg_set_timing(ctx,1); kmg_set_timing(ctx,2)
 * times only the "gram", "gather", "unpack", "mirror" and "memset" stages, 2 events per
 * Gram launch instead of 2 per stage); nothing is synchronised until a stage time is read.
 * Stage names: "count", "scan", "place", "fine", "diag", "gram", "extract", "features",
 * "pack" (2-bit packing of the input), "slots" (mismatch slot / pair tables, neighbourhood
 * lists), "lists" (neighbourhood-list sizes and starts), "combine",
 * "solve", "memset", "gather" (the RCCL all-gathers of kmg_gram_blocks, timed on their own
 * stream), "unpack" (round-slab assembly), "mirror" (lower block triangle of a full square
 * mismatch K built by its upper block triangle).
 *   kmg_stage_ms:    that stage in the last call (-1 if it did not run)
 *   kmg_stage_stats: sum and count over every call since kmg_timing_reset */
int kmg_set_timing(kmg_ctx *ctx, int32_t enable);
int kmg_timing_reset(kmg_ctx *ctx);
int kmg_stage_ms(kmg_ctx *ctx, const char *stage, double *ms);
int kmg_stage_stats(kmg_ctx *ctx, const char *stage, double *total_ms, int32_t *count);

/* How the last spectrum / mismatch Gram call on ctx was built (for roofline accounting):
 * plan[0] formulation (0 dense count-vector GEMM, 1 all-pairs Hamming, 2 posting lists,
 * 3 mismatch drop-one slot table, 4 drop-two pair table, 5 (unused: round 3's pair lines,
 * removed), 6 neighbourhood lists, 7 the generic per-pair kernels of k > 16; -1 none yet or the call failed before
 * choosing),
 * plan[1] columns per chunk, plan[2] column chunks, plan[3] 1 when a full square K was built
 * by its upper block triangle and mirrored, plan[4] Gram workgroup threads (0 where the
 * formulation has no column chunks), plan[5] neighbourhood lists only: 1 when their Hamming-2
 * segments were sorted and packed (1 B + 1/15 of 2 B an entry), 0 when they stayed 16-bit.
 * No reference counterpart (diagnostics). */
int kmg_last_plan(kmg_ctx *ctx, int32_t plan[6]);

/* The factorisation of the last KRR / KLR solve on ctx (diagnostics, no reference
 * counterpart; the reference inverts with numpy's LU, KRR.py:33, KLR.py:55-56):
 * KMG_FACTOR_CHOLESKY for a bitwise-symmetric positive-definite system (every Gram kmg_gram
 * returns), KMG_FACTOR_LU_ASYMMETRIC when K != K^T bitwise, KMG_FACTOR_LU_INDEFINITE when
 * Cholesky failed; 0 before any solve. */
#define KMG_FACTOR_CHOLESKY 1
#define KMG_FACTOR_LU_ASYMMETRIC 2
#define KMG_FACTOR_LU_INDEFINITE 3
int kmg_last_factorisation(kmg_ctx *ctx, int32_t *kind);

/* RCCL (one rank per process / GPU).  id is an opaque 128-byte ncclUniqueId. */
int kmg_comm_unique_id(uint8_t id[128]);
int kmg_comm_init(kmg_ctx *ctx, const uint8_t id[128], int32_t nranks, int32_t rank);
/* Assemble the full n x n K on every rank: rank r owns rows [splits[r], splits[r+1])
 * (0 = splits[0] <= ... <= splits[nranks] = n, checked); one RCCL group of per-root
 * broadcasts.  kmg_gram_blocks is the overlapped in-place ncclAllGather form. */
int kmg_allgather_rows(kmg_ctx *ctx, void *d_K, int64_t n, int64_t ld, int32_t dtype,
                       const int64_t *splits);
int kmg_comm_destroy(kmg_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* KMGRAM_H */
