/*
 * ORACLE — plain-C restatement of the reference Gram path.  TEST INFRASTRUCTURE ONLY.
 *
 * Used only by tests/ (as the checker at sizes the pure-Python oracle cannot reach),
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Never linked into
 * libkmgram.so.  Built with -ffp-contract=off so float64 expressions round exactly as
 * the reference's CPython float arithmetic does.
 *
 * Reference: afiliot/Kernel-Methods-For-Genomics kernels.py (v1).
 *   kmo_spectrum      get_spectrum_K   kernels.py:28-47   (phi: get_phi_u 12-25)
 *   kmo_mismatch_raw  get_mismatch_K   kernels.py:196-215 (phi: get_phi_km 161-175),
 *                     via the closed form sum_{a,b} w[ham(x_a, y_b)]
 *   kmo_wd            get_WD_K         kernels.py:84-101  (get_WD_d 64-81)
 *   kmo_wds           get_WDShifts_K   kernels.py:138-155 (get_WDShifts_d 115-135)
 *   kmo_ss            get_string_K     kernels.py:367-382 (K_k 344-364, B_k 322-342)
 * Symbol codes: A,C,G,T = 0..3, other characters >= 4.
 * Rows [row0,row1) x all n columns are produced into out[(i-row0)*n + j].
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return x < y ? -1 : x > y;
}

/* k-mer codes of sequence s (windows range(P), P = L-k+1); invalid windows dropped.
 * Returns count written to dst (sorted ascending when sort != 0). */
static int kmers_of(const uint8_t *s, int L, int k, uint32_t *dst, int sort) {
  int P = L - k + 1, cnt = 0;
  for (int a = 0; a < P; ++a) {
    uint32_t c = 0;
    int bad = 0;
    for (int q = 0; q < k; ++q) {
      bad |= s[a + q] >= 4;
      c = (c << 2) | (s[a + q] & 3u);
    }
    if (!bad) dst[cnt++] = c;
  }
  if (sort) qsort(dst, cnt, sizeof(uint32_t), cmp_u32);
  return cnt;
}

/* K_ij = sum_u phi_i(u) phi_j(u) = #{(a,b): x_a == y_b}: merge of sorted k-mer lists */
int kmo_spectrum(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc, int k,
                 int64_t row0, int64_t row1, int64_t *out) {
  if (k < 1 || k > 16) return 1;
  int maxp = 1;
  for (int64_t i = 0; i < n; ++i)
    if (lens[i] - k + 1 > maxp) maxp = lens[i] - k + 1;
  uint32_t *km = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)n * maxp);
  int *cnt = (int *)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
  if (!km || !cnt) return 2;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) cnt[i] = kmers_of(codes + i * ldc, lens[i], k, km + i * maxp, 1);
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t i = row0; i < row1; ++i) {
    const uint32_t *a = km + i * maxp;
    const int na = cnt[i];
    for (int64_t j = 0; j < n; ++j) {
      const uint32_t *b = km + j * maxp;
      const int nb = cnt[j];
      int64_t s = 0;
      int p = 0, q = 0;
      while (p < na && q < nb) {
        if (a[p] < b[q]) {
          ++p;
        } else if (a[p] > b[q]) {
          ++q;
        } else {
          const uint32_t v = a[p];
          int ca = 0, cb = 0;
          while (p < na && a[p] == v) ++p, ++ca;
          while (q < nb && b[q] == v) ++q, ++cb;
          s += (int64_t)ca * cb;
        }
      }
      out[(i - row0) * n + j] = s;
    }
  }
  free(km);
  free(cnt);
  return 0;
}

/* raw mismatch kernel: sum_{a,b} w[ham(x_a, y_b)], windows range(window-k+1) */
int kmo_mismatch_raw(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc, int k,
                     int window, const int64_t *w, int64_t row0, int64_t row1, int64_t *out) {
  if (k < 1 || k > 16) return 1;
  const int P = window - k + 1;
  if (P <= 0) return 1;
  for (int64_t i = 0; i < n; ++i)
    if (lens[i] < window) return 3;
  uint32_t *km = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)n * P);
  if (!km) return 2;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) kmers_of(codes + i * ldc, window, k, km + i * P, 0);
  const uint32_t mask = (k >= 16) ? 0x55555555u : (0x55555555u & ((1u << (2 * k)) - 1u));
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = row0; i < row1; ++i) {
    const uint32_t *a = km + i * P;
    for (int64_t j = 0; j < n; ++j) {
      const uint32_t *b = km + j * P;
      int64_t s = 0;
      for (int p = 0; p < P; ++p)
        for (int q = 0; q < P; ++q) {
          const uint32_t x = a[p] ^ b[q];
          s += w[__builtin_popcount((x | (x >> 1)) & mask)];
        }
      out[(i - row0) * n + j] = s;
    }
  }
  free(km);
  return 0;
}

/* raw self-kernels (diagonal) for normalisation */
int kmo_mismatch_diag(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc, int k,
                      int window, const int64_t *w, int64_t *diag) {
  const int P = window - k + 1;
  if (k < 1 || k > 16 || P <= 0) return 1;
  const uint32_t mask = (k >= 16) ? 0x55555555u : (0x55555555u & ((1u << (2 * k)) - 1u));
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    uint32_t a[256];
    if (P > 256 || lens[i] < window) {
      diag[i] = -1;
      continue;
    }
    kmers_of(codes + i * ldc, window, k, a, 0);
    int64_t s = 0;
    for (int p = 0; p < P; ++p)
      for (int q = 0; q < P; ++q) {
        const uint32_t x = a[p] ^ a[q];
        s += w[__builtin_popcount((x | (x >> 1)) & mask)];
      }
    diag[i] = s;
  }
  return 0;
}

static int slice_eq(const uint8_t *x, int Lx, int ox, const uint8_t *y, int Ly, int oy, int k) {
  /* Python x[ox:ox+k] == y[oy:oy+k] on strings (slices clip at the end) */
  int lx = Lx - ox, ly = Ly - oy;
  if (lx > k) lx = k;
  if (ly > k) ly = k;
  if (lx < 0) lx = 0;
  if (ly < 0) ly = 0;
  if (lx != ly) return 0;
  return memcmp(x + ox, y + oy, (size_t)lx) == 0;
}

int kmo_wd(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc, int d,
           const double *beta, int64_t row0, int64_t row1, double *out) {
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t i = row0; i < row1; ++i) {
    for (int64_t j = 0; j < n; ++j) {
      double v;
      if (i == j) {
        const int L = lens[i];
        v = (double)(L - 1) + (double)(1 - d) / 3.0; /* kernels.py:96 */
      } else {
        const int64_t a = i < j ? i : j, b = i < j ? j : i;
        const uint8_t *x = codes + a * ldc, *y = codes + b * ldc;
        const int L = lens[a], Ly = lens[b];
        double ct = 0.0;
        for (int k = 1; k <= d; ++k) {
          long cst = 0;
          for (int l = 1; l <= L - k; ++l) cst += slice_eq(x, L, l, y, Ly, l, k);
          const double t = beta[k - 1] * (double)cst;
          ct = ct + t;
        }
        v = ct;
      }
      out[(i - row0) * n + j] = v;
    }
  }
  return 0;
}

int kmo_wds(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc, int d, int S,
            const double *beta, const double *delta, int64_t row0, int64_t row1, double *out) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = row0; i < row1; ++i) {
    for (int64_t j = 0; j < n; ++j) {
      const int64_t a = i <= j ? i : j, b = i <= j ? j : i;
      const uint8_t *x = codes + a * ldc, *y = codes + b * ldc;
      const int L = lens[a], Ly = lens[b];
      double ct = 0.0;
      for (int k = 1; k <= d; ++k) {
        double cst = 0.0;
        for (int ii = 1; ii <= L - k; ++ii)
          for (int s = 0; s <= S; ++s)
            if (s + ii < L) {
              const int m = slice_eq(x, L, ii + s, y, Ly, ii, k) + slice_eq(x, L, ii, y, Ly, ii + s, k);
              const double t = delta[s] * (double)m;
              cst = cst + t;
            }
        const double t = beta[k - 1] * cst;
        ct = ct + t;
      }
      out[(i - row0) * n + j] = ct;
    }
  }
  return 0;
}

static double ss_pair(const uint8_t *x, int n, const uint8_t *y, int m, int k, double lam,
                      double lam2, double *work) {
  if (k == 0) return 1.0;
  if (n < k || m < k) return 0.0;
  /* work: k levels x (n+1) x (m+1) */
  const size_t plane = (size_t)(n + 1) * (m + 1);
#define B(t, r, c) work[(size_t)(t) * plane + (size_t)(r) * (m + 1) + (c)]
  for (int r = 0; r <= n; ++r)
    for (int c = 0; c <= m; ++c) B(0, r, c) = 1.0;
  for (int t = 1; t < k; ++t)
    for (int r = 0; r <= n; ++r)
      for (int c = 0; c <= m; ++c) {
        if (r < t || c < t) {
          B(t, r, c) = 0.0;
          continue;
        }
        const double a1 = lam * B(t, r - 1, c);
        const double a2 = lam * B(t, r, c - 1);
        double v = a1 + a2;
        const double a3 = lam2 * B(t, r - 1, c - 1);
        v = v - a3;
        if (x[r - 1] == y[c - 1]) {
          const double a4 = lam2 * B(t - 1, r - 1, c - 1);
          v = v + a4;
        }
        B(t, r, c) = v;
      }
  double K = 0.0;
  for (int i = k; i <= n; ++i) {
    double s = 0.0;
    for (int c = 0; c < m; ++c)
      if (y[c] == x[i - 1]) s = s + B(k - 1, i - 1, c);
    const double t = lam2 * s;
    K = K + t;
  }
#undef B
  return K;
}

int kmo_ss(const uint8_t *codes, const int32_t *lens, int64_t n, int64_t ldc, int k, double lam,
           double lam2, int64_t row0, int64_t row1, double *out) {
  int maxl = 1;
  for (int64_t i = 0; i < n; ++i)
    if (lens[i] > maxl) maxl = lens[i];
  const size_t wsz = (size_t)(k > 0 ? k : 1) * (maxl + 1) * (maxl + 1);
#pragma omp parallel
  {
    double *work = (double *)malloc(sizeof(double) * wsz);
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = row0; i < row1; ++i)
      for (int64_t j = 0; j < n; ++j) {
        const int64_t a = i <= j ? i : j, b = i <= j ? j : i;
        out[(i - row0) * n + j] =
            ss_pair(codes + a * ldc, lens[a], codes + b * ldc, lens[b], k, lam, lam2, work);
      }
    free(work);
  }
  return 0;
}
