"""ORACLE — CPU restatement of the reference Gram path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker (never as the thing measured or shipped).

It restates afiliot/Kernel-Methods-For-Genomics kernels.py (v1) function by function,
keeping the reference's float64 operation order where results are floating point.
Parity of this oracle is pinned against golden vectors produced by running the
unmodified reference in the build container (tests/golden/make_golden.py ->
tests/golden/golden.npz; checked by tests/test_oracle_golden.py).

Symbol codes: A,C,G,T = 0..3, anything else >= 4 (kmgram.encode).
"""
import numpy as np
import scipy.sparse as sp


def _codes_list(codes, lens):
    return [codes[i, : lens[i]].astype(np.int64) for i in range(len(lens))]


# --------------------------------------------------------------------- spectrum
def kmer_codes(seq, k, window=None):
    """Base-4 codes of the k-mers x[i:i+k], i in range(len(x)-k+1) (kernels.py:21-22),
    or range(window-k+1) for the mismatch kernel (kernels.py:171).  Windows holding a
    non-ACGT symbol map to -1 (they match no beta, kernels.py:23-24)."""
    L = len(seq) if window is None else window
    P = L - k + 1
    if P <= 0:
        return np.zeros(0, dtype=np.int64)
    out = np.zeros(P, dtype=np.int64)
    bad = np.zeros(P, dtype=bool)
    for q in range(k):
        col = seq[q:q + P]
        bad |= col >= 4
        out = out * 4 + (col & 3)
    out[bad] = -1
    return out


def spectrum(codes, lens, k):
    """get_spectrum_K (kernels.py:28-47): K = Phi Phi^T with Phi the k-mer count matrix
    (get_phi_u, kernels.py:12-25).  Exact integers (int64)."""
    seqs = _codes_list(codes, lens)
    rows, cols = [], []
    for i, s in enumerate(seqs):
        c = kmer_codes(s, k)
        c = c[c >= 0]
        rows.append(np.full(len(c), i))
        cols.append(c)
    n = len(seqs)
    r = np.concatenate(rows) if rows else np.zeros(0, dtype=np.int64)
    c = np.concatenate(cols) if cols else np.zeros(0, dtype=np.int64)
    Phi = sp.csr_matrix((np.ones(len(r), dtype=np.int64), (r, c)), shape=(n, 4 ** k))
    return (Phi @ Phi.T).toarray().astype(np.int64)


def spectrum_windows(codes, lens, k):
    """get_spectrum_K for any k (kernels.py:28-47) by counting windows: K[i, j] =
    sum_w c_i(w) c_j(w) over the all-ACGT windows w of length k (a window holding another
    character equals none of the 4^k ACGT betas, kernels.py:23-24).  The same count as
    spectrum() without the 4^k-column Phi, so it also covers k past 31; checked against
    spectrum() for small k in tests/test_oracle_generic.py."""
    from collections import Counter
    seqs = _codes_list(codes, lens)
    cnt = []
    for s in seqs:
        c = Counter()
        for a in range(len(s) - k + 1):
            win = s[a:a + k]
            if np.all(win < 4):
                c[win.tobytes()] += 1
        cnt.append(c)
    n = len(seqs)
    K = np.zeros((n, n), dtype=np.int64)
    for i in range(n):
        for j in range(i, n):
            a, b = (cnt[i], cnt[j]) if len(cnt[i]) <= len(cnt[j]) else (cnt[j], cnt[i])
            K[i, j] = K[j, i] = sum(v * b.get(w, 0) for w, v in a.items())
    return K


# --------------------------------------------------------------------- mismatch
def mismatch_weights(k, m):
    """Closed form of <Phi_x, Phi_y> per k-mer pair at Hamming distance h (see
    kmgram.params.mismatch_weights; verified here by brute force in tests)."""
    from math import comb
    w = []
    for h in range(k + 1):
        tot = 0
        for i in range(k - h + 1):
            for a in range(h + 1):
                for b in range(h - a + 1):
                    c = h - a - b
                    if i + b + c <= m and i + a + c <= m:
                        tot += comb(k - h, i) * 3 ** i * comb(h, a) * comb(h - a, b) * 2 ** c
        w.append(tot)
    return np.array(w, dtype=np.int64)


def _ham_matrix(a, b, k):
    x = a[:, None] ^ b[None, :]
    y = (x | (x >> 1)) & int("01" * k, 2)
    # popcount
    cnt = np.zeros(y.shape, dtype=np.int64)
    while np.any(y):
        cnt += y & 1
        y >>= 1
    return cnt


def mismatch_raw(codes, lens, k, m, window=101):
    """Raw <Phi_km(x), Phi_km(y)> (kernels.py:206-215) = sum_{a,b} w_m[ham(x_a, y_b)]."""
    seqs = _codes_list(codes, lens)
    km = [kmer_codes(s, k, window) for s in seqs]
    w = mismatch_weights(k, m)
    n = len(seqs)
    K = np.zeros((n, n), dtype=np.int64)
    for i in range(n):
        for j in range(i, n):
            H = _ham_matrix(km[i], km[j], k)
            K[i, j] = K[j, i] = int(w[H].sum())
    return K


def mismatch_raw_windows(codes, lens, k, m, window=101):
    """The C ABI's mismatch (k, m) over any rows (beyond the reference, which raises for
    rows shorter than the window or holding a non-ACGT symbol, kernels.py:171-174, 193):
    sum_{a,b} w[ham(x_a, y_b)] over the windows a, b < window - k + 1 that lie inside their
    row and hold only A/C/G/T (the k <= 16 kernels' pk_window rule).  Explicit window
    pairs, small cases only."""
    w = mismatch_weights(k, m)
    P = window - k + 1
    wins = []
    for i in range(len(lens)):
        s = codes[i, : lens[i]].astype(np.int64)
        ws = [s[a:a + k] for a in range(P) if a + k <= len(s) and np.all(s[a:a + k] < 4)]
        wins.append(np.stack(ws) if ws else np.zeros((0, k), dtype=np.int64))
    n = len(lens)
    K = np.zeros((n, n), dtype=np.int64)
    for i in range(n):
        for j in range(i, n):
            H = (wins[i][:, None, :] != wins[j][None, :, :]).sum(axis=2)
            K[i, j] = K[j, i] = int(w[np.minimum(H, k)].sum()) if H.size else 0
    return K


def normalize(K):
    """normalize_K (kernels.py:398-415) on a copy: K_ij / (d_i * d_j), d = sqrt(diag),
    upper triangle mirrored, diagonal := 1; unchanged if K[0,0] == 1."""
    K = np.array(K, dtype=np.float64)
    if K[0, 0] == 1:
        return K
    d = np.sqrt(np.diag(K))
    iu = np.triu_indices(K.shape[0], 1)
    vals = K[iu] / (d[iu[0]] * d[iu[1]])
    K[iu] = vals
    K[(iu[1], iu[0])] = vals
    np.fill_diagonal(K, 1.0)
    return K


def mismatch(codes, lens, k, m, window=101):
    """get_mismatch_K (kernels.py:196-217)."""
    return normalize(mismatch_raw(codes, lens, k, m, window).astype(np.float64))


def mismatch_phi_bruteforce(codes, lens, k, m, window=101):
    """Literal restatement of get_phi_km + np.dot (kernels.py:161-175, 211-215) over all
    4^k betas.  Tiny k only (verifies the closed form)."""
    seqs = _codes_list(codes, lens)
    betas = np.array([[(b >> (2 * (k - 1 - q))) & 3 for q in range(k)] for b in range(4 ** k)])
    Phi = np.zeros((len(seqs), 4 ** k), dtype=np.int64)
    for i, s in enumerate(seqs):
        for a in range(window - k + 1):
            kmer = s[a:a + k]
            Phi[i] += (np.sum(kmer[None, :] != betas, axis=1) <= m)
    return Phi @ Phi.T


# --------------------------------------------------------------------- WD / WDS
def wd(codes, lens, d):
    """get_WD_K (kernels.py:84-101) with get_WD_d (kernels.py:64-81), same fp64 order."""
    seqs = _codes_list(codes, lens)
    n = len(seqs)
    K = np.zeros((n, n))
    bet = [2 * (d - k + 1) / d / (d + 1) for k in range(1, d + 1)]
    for i in range(n):
        x = seqs[i]
        L = len(x)
        K[i, i] = L - 1 + (1 - d) / 3
        for j in range(i + 1, n):
            y = seqs[j]
            c_t = 0
            for k in range(1, d + 1):
                c_st = 0
                for l in range(1, L - k + 1):
                    xs, ys = x[l:l + k], y[l:l + k]
                    c_st += bool(len(xs) == len(ys) and np.array_equal(xs, ys))
                c_t += bet[k - 1] * c_st
            K[i, j] = K[j, i] = c_t
    return K


def _eq(a, b):
    return len(a) == len(b) and np.array_equal(a, b)


def wds(codes, lens, d, S):
    """get_WDShifts_K (kernels.py:138-155) with get_WDShifts_d (kernels.py:115-135)."""
    seqs = _codes_list(codes, lens)
    n = len(seqs)
    K = np.zeros((n, n))
    bet = [2 * (d - k + 1) / d / (d + 1) for k in range(1, d + 1)]
    dlt = [1 / 2 / (s + 1) for s in range(S + 1)]
    for i in range(n):
        x = seqs[i]
        L = len(x)
        for j in range(i, n):
            y = seqs[j]
            c_t = 0
            for k in range(1, d + 1):
                c_st = 0
                for ii in range(1, L - k + 1):
                    for s in range(0, S + 1):
                        if s + ii < L:
                            c_st += dlt[s] * (_eq(x[ii + s:ii + s + k], y[ii:ii + k]) +
                                              _eq(x[ii:ii + k], y[ii + s:ii + s + k]))
                c_t += bet[k - 1] * c_st
            K[i, j] = K[j, i] = c_t
    return K


def wd_pair(x, y, d, L):
    """get_WD_d(x, y, d, L) (kernels.py:64-81) for any L: the slices clip at the end of
    each string and are compared as strings (x, y: str)."""
    c_t = 0
    for k in range(1, d + 1):
        c_st = 0
        for l in range(1, L - k + 1):
            c_st += (x[l:l + k] == y[l:l + k])
        c_t += (2 * (d - k + 1) / d / (d + 1)) * c_st
    return c_t


def wds_pair(x, y, d, S, L):
    """get_WDShifts_d(x, y, d, S, L) (kernels.py:115-135) for any L (x, y: str)."""
    c_t = 0
    for k in range(1, d + 1):
        c_st = 0
        for i in range(1, L - k + 1):
            for s in range(0, S + 1):
                if s + i < L:
                    c_st += (1 / 2 / (s + 1)) * ((x[i + s:i + s + k] == y[i:i + k]) +
                                                 (x[i:i + k] == y[i + s:i + s + k]))
        c_t += (2 * (d - k + 1) / d / (d + 1)) * c_st
    return c_t


# --------------------------------------------------------------------- substring
def ss_pair(x, y, lbda, k):
    """K_k(lbda, k, x, y) (kernels.py:344-364) by bottom-up DP over B_t (kernels.py:322-342)
    with the reference's expression order."""
    if k == 0:
        return 1
    n, m = len(x), len(y)
    if n < k or m < k:
        return 0
    lam2 = lbda ** 2
    # B[t][r][c] = B_t(x[:r], y[:c])
    B = [[[1] * (m + 1) for _ in range(n + 1)]]
    for t in range(1, k):
        Bt = [[0] * (m + 1) for _ in range(n + 1)]
        prev = B[t - 1]
        for r in range(n + 1):
            for c in range(m + 1):
                if r < t or c < t:
                    Bt[r][c] = 0
                    continue
                v = lbda * Bt[r - 1][c] + lbda * Bt[r][c - 1] - lam2 * Bt[r - 1][c - 1]
                v = v + (lam2 * prev[r - 1][c - 1] if x[r - 1] == y[c - 1] else 0)
                Bt[r][c] = v
        B.append(Bt)
    Bk1 = B[k - 1]
    K = 0
    for i in range(k, n + 1):
        a = x[i - 1]
        s = sum(Bk1[i - 1][c] for c in range(m) if y[c] == a)
        K = K + lam2 * s
    return K


def ss_b(x, y, lbda, k):
    """B_k(lbda, k, x, y) (kernels.py:322-342) by the bottom-up table of ss_pair: the level-k
    value at the full prefixes; 1 for k = 0, 0 when a string is shorter than k."""
    if k == 0:
        return 1
    n, m = len(x), len(y)
    if n < k or m < k:
        return 0
    lam2 = lbda ** 2
    prev = [[1] * (m + 1) for _ in range(n + 1)]
    for t in range(1, k + 1):
        Bt = [[0] * (m + 1) for _ in range(n + 1)]
        for r in range(t, n + 1):
            for c in range(t, m + 1):
                v = lbda * Bt[r - 1][c] + lbda * Bt[r][c - 1] - lam2 * Bt[r - 1][c - 1]
                v = v + (lam2 * prev[r - 1][c - 1] if x[r - 1] == y[c - 1] else 0)
                Bt[r][c] = v
        prev = Bt
    return prev[n][m]


def substring(codes, lens, lbda, k):
    """get_string_K (kernels.py:367-382)."""
    seqs = [list(map(int, s)) for s in _codes_list(codes, lens)]
    n = len(seqs)
    K = np.zeros((n, n))
    for i in range(n):
        for j in range(i, n):
            K[i, j] = K[j, i] = ss_pair(seqs[i], seqs[j], lbda, k)
    return K


# --------------------------------------------------------------------- others
def local_alignment_reference(n):
    """get_LA_K as the reference computes it: M,X,Y,X2,Y2 alias one array
    (kernels.py:238,262) and cell [n_x, n_y] is never written, so every entry is
    (1/beta)*log(1+0) = 0.0; the function returns K, not K1 (kernels.py:302)."""
    return np.zeros((n, n))


# substitution matrix of the LA kernel (kernels.py:223, rows/columns A, C, G, T)
LA_S = np.array([[4, 0, 0, 0], [0, 9, -3, -1], [0, -3, 6, 2], [0, -1, -2, 5]])


def la_intended_pair(x, y, e, d, beta, smith):
    """The LA kernel value the reference means (affine_align / Smith_Waterman,
    kernels.py:226-270) with its three defects removed — parity unpinned, the reference
    never produces it:
      * M, X, Y, X2, Y2 are five arrays (the reference aliases one, kernels.py:238, 262);
      * cells (i, j) for i in 1..n_x, j in 1..n_y read x[i-1], y[j-1] (the reference's
        range(1, n) never reaches [n_x, n_y] and skips x[0]);
      * gaps cost what the docstring says, g(n) = e + d(n-1) with e the opening and d the
        extension penalty: opening factor exp(-beta e), extension exp(-beta d) (the
        reference multiplies by exp(+beta d) and exp(+beta e)).
    Same recurrences and the same evaluation order otherwise (sum form, or max for
    smith=1); returns (1/beta) log(1 + X2 + Y2 + M) at [n_x, n_y].  Pure Python floats
    (IEEE double, no fused multiply-add), small cases only."""
    import math  # libm exp / log (the device path computes its table with the same libm)
    es = [[math.exp(beta * float(v)) for v in row] for row in LA_S]
    eo, ee = math.exp(-beta * e), math.exp(-beta * d)
    nx, ny = len(x), len(y)
    z = [0.0] * (ny + 1)
    M, X, Y, X2, Y2 = list(z), list(z), list(z), list(z), list(z)  # row i-1
    for i in range(1, nx + 1):
        m, xx, yy, x2, y2 = [0.0], [0.0], [0.0], [0.0], [0.0]  # row i, column 0
        xi = int(x[i - 1])
        for j in range(1, ny + 1):
            sub = es[xi][int(y[j - 1])]
            if smith:
                m.append(sub * max(1.0, X[j - 1], Y[j - 1], M[j - 1]))
                xx.append(max(eo * M[j], ee * X[j]))
                yy.append(max(eo * m[j - 1], eo * xx[j - 1], ee * yy[j - 1]))
                x2.append(max(M[j], X2[j]))
                y2.append(max(m[j - 1], x2[j - 1], y2[j - 1]))
            else:
                m.append(sub * (1.0 + X[j - 1] + Y[j - 1] + M[j - 1]))
                xx.append(eo * M[j] + ee * X[j])
                yy.append(eo * (m[j - 1] + xx[j - 1]) + ee * yy[j - 1])
                x2.append(M[j] + X2[j])
                y2.append(m[j - 1] + x2[j - 1] + y2[j - 1])
        M, X, Y, X2, Y2 = m, xx, yy, x2, y2
    v = max(1.0, X2[ny], Y2[ny], M[ny]) if smith else 1.0 + X2[ny] + Y2[ny] + M[ny]
    return (1 / beta) * math.log(v)


def la_intended(codes, lens, e=11, d=1, beta=0.5, smith=0):
    """get_LA_K with the intended recurrence: K[i, j] = K[j, i] = la_intended_pair(x_i,
    x_j) for j >= i (the reference's fill order, kernels.py:293-297)."""
    seqs = _codes_list(codes, lens)
    n = len(seqs)
    K = np.zeros((n, n))
    for i in range(n):
        for j in range(i, n):
            K[i, j] = K[j, i] = la_intended_pair(seqs[i], seqs[j], e, d, beta, smith)
    return K


def gappy_k1g0(codes, lens, window=101):
    """get_gappy_K(X, 1, 0): phi_c = [letter c occurs in x[:window]] (kernels.py:420-433)."""
    seqs = _codes_list(codes, lens)
    Phi = np.zeros((len(seqs), 4))
    for i, s in enumerate(seqs):
        for c in set(int(v) for v in s[:window]):
            Phi[i, c] = 1
    return normalize(Phi @ Phi.T)


def gappy_intended_phi(codes, lens, k, g, window=101):
    """Binary presence features of the intended gappy kernel (kernels.py:420-433 with the
    betas over (k-g)-mers, as report §3.7 describes it): phi[i, b] = 1 if the (k-g)-mer b
    (base-4 code, first letter most significant) is itertools.combinations(x[a:a+k], k-g)
    of some window a in range(window - k + 1).  Parity unpinned (the reference raises)."""
    from itertools import combinations
    seqs = _codes_list(codes, lens)
    kk = k - g
    Phi = np.zeros((len(seqs), 4 ** kk), dtype=np.int64)
    for i, s in enumerate(seqs):
        seen = set()
        for a in range(window - k + 1):
            for sub in combinations(s[a:a + k], kk):
                if len(sub) == kk and all(v < 4 for v in sub):
                    c = 0
                    for v in sub:
                        c = c * 4 + int(v)
                    seen.add(c)
        Phi[i, sorted(seen)] = 1
    return Phi


def gappy_intended(codes, lens, k, g, window=101):
    """get_gappy_K intended: normalize_K(Phi Phi^T) (kernels.py:449-454)."""
    Phi = gappy_intended_phi(codes, lens, k, g, window)
    return normalize((Phi @ Phi.T).astype(np.float64))


def center(K):
    """center_K (kernels.py:387-395)."""
    n = K.shape[0]
    B = np.eye(n) - np.ones((n, n)) / n
    return np.linalg.multi_dot([B, K, B])


# --------------------------------------------------------------------- combination consumers
def nlck_combine(kernels, u, degree):
    """NLCK.svm_step / get_K (NLCKernels.py:52, 97): np.sum(kernels * u[:, None, None],
    axis=0) ** degree."""
    return np.sum(np.asarray(kernels) * np.asarray(u)[:, None, None], axis=0) ** degree


def nlck_grad(kernels_fit, u, degree, alpha):
    """NLCK.grad (NLCKernels.py:61-66)."""
    K_t = np.sum(np.asarray(kernels_fit) * np.asarray(u)[:, None, None], axis=0) ** (degree - 1)
    grad = np.zeros(len(kernels_fit))
    for m, Km in enumerate(kernels_fit):
        grad[m] = alpha.T.dot(K_t * Km).dot(alpha)
    return -degree * grad


def alignf_stats(kernels_fit, y):
    """ALIGNF.get_a / get_M (ALIGNF.py:43-58) on center_K (kernels.py:387-395)."""
    Y = np.outer(y, y)
    Kc = [center(K) for K in kernels_fit]
    p = len(Kc)
    a = np.array([(K * Y).sum() for K in Kc])
    M = np.zeros((p, p))
    for i in range(p):
        for j in range(i, p):
            M[i, j] = M[j, i] = (Kc[i] * Kc[j]).sum()
    return a, M


# --------------------------------------------------------------------- sparse CPU comparator
def _kmer_matrix(codes, lens, k, P):
    km = np.zeros((codes.shape[0], P), dtype=np.int64)
    for q in range(k):
        km = km * 4 + (codes[:, q:q + P] & 3)
    return km


def spectrum_phi(codes, lens, k):
    """Phi of get_phi_u (kernels.py:12-25) as a CSR count matrix (N x 4^k); windows
    range(len(x)-k+1), windows holding a non-ACGT symbol dropped."""
    n = len(lens)
    P = int(lens.max()) - k + 1 if n else 0
    if P <= 0:
        return sp.csr_matrix((n, 4 ** k), dtype=np.int32)
    km = _kmer_matrix(codes, lens, k, P)
    bad = np.zeros(km.shape, dtype=bool)
    for q in range(k):
        bad |= codes[:, q:q + P] >= 4
    valid = (np.arange(P)[None, :] <= (lens[:, None] - k)) & ~bad
    r, c = np.nonzero(valid)
    return sp.csr_matrix((np.ones(r.size, dtype=np.int32), (r, km[r, c])), shape=(n, 4 ** k))


def phi_u(x, k, betas):
    """get_phi_u (kernels.py:12-25) for one string: phi[j] = #{i : x[i:i+k] == betas[j]}."""
    from collections import Counter
    cnt = Counter(x[i:i + k] for i in range(len(x) - k + 1))
    return np.array([float(cnt.get(b, 0)) for b in betas])


def phi_km(x, k, m, betas):
    """get_phi_km (kernels.py:161-175) for one format()ed row: phi[j] = #{i < 101-k+1 :
    #(x[i:i+k] != betas[j]) <= m}.  A row shorter than 101 (kernels.py:171 still walks 101-k+1
    windows) compares its short k-mers as numpy does: one symbol broadcasts against every
    letter of the beta, none (k = 1) sums to 0 mismatches, and any other length raises."""
    x = np.asarray(x).reshape(-1)
    B = np.asarray(betas).reshape(len(betas), -1)
    if len(x) >= 101:
        W = np.stack([x[i:i + k] for i in range(101 - k + 1)])       # windows x k
        H = (W[:, None, :] != B[None, :, :]).sum(axis=2)                # windows x betas
        return (H <= m).sum(axis=0).astype(np.float64)
    out = np.zeros(len(B))
    for i in range(101 - k + 1):
        kmer = x[i:i + k]
        for j, b in enumerate(B):
            out[j] += (np.sum(kmer != b) <= m)
    return out


def gappy1_phi(x, betas):
    """gappy_k(x, 1, 0, betas) (kernels.py:420-433): 1.0 where the letter occurs in x[0:101]."""
    present = set(int(v) for v in np.asarray(x).reshape(-1)[:101])
    return np.array([1.0 if int(np.asarray(b).reshape(-1)[0]) in present else 0.0 for b in betas])


def neighbour_masks(k, m):
    """xor masks of every k-mer within Hamming distance m of a k-mer (2-bit letters)."""
    from itertools import combinations, product
    masks = [0]
    for t in range(1, min(m, k) + 1):
        for pos in combinations(range(k), t):
            for letters in product((1, 2, 3), repeat=t):
                v = 0
                for p_, x in zip(pos, letters):
                    v |= x << (2 * p_)
                masks.append(v)
    return np.array(masks, dtype=np.int64)


def mismatch_phi(codes, lens, k, m, window=101):
    """Phi_km of get_phi_km (kernels.py:161-175) as a CSR count matrix: each window a adds
    1 to every k-mer within Hamming distance m of x[a:a+k] (ACGT input, length >= window)."""
    n = len(lens)
    P = window - k + 1
    km = _kmer_matrix(codes, lens, k, P)
    masks = neighbour_masks(k, m)
    cols = (km[:, :, None] ^ masks[None, None, :]).reshape(n, -1)
    rows = np.repeat(np.arange(n), cols.shape[1])
    return sp.csr_matrix((np.ones(rows.size, dtype=np.int32), (rows, cols.ravel())),
                         shape=(n, 4 ** k))


# --------------------------------------------------------------------- dense learners on K
def krr_alpha(K_fit, y, lbda):
    """KRR.fit's solve (KRR.py:33): inv(K_fit + lbda * n * I) . y, with np.linalg.inv."""
    n = K_fit.shape[0]
    return np.dot(np.linalg.inv(K_fit + lbda * n * np.eye(n)), y)


def _sig(x):
    return 1 / (1 + np.exp(-x))


def klr_alpha(K_fit, y, lbda, tol=1e-5, maxiter=50):
    """KLR.fit's IRLS (KLR.py:30-75): from alpha = 0, m = K alpha, W = s(m) s(-m),
    z = m + y / s(-y m), alpha = Ws inv(Ws K Ws + n lbda I) Ws z while the step's 2-norm
    exceeds tol, at most maxiter steps.  Returns (alpha, steps)."""
    n = K_fit.shape[0]
    prev = np.zeros(n)
    diff, steps = np.inf, 0
    for _ in range(maxiter):
        if not diff > tol:
            continue
        m = K_fit @ prev
        W = _sig(m) * _sig(-m)
        z = m + y / _sig(-y * m)
        s = np.sqrt(W)
        A = s[:, None] * K_fit * s[None, :] + n * lbda * np.eye(n)
        alpha = s * (np.linalg.inv(A) @ (s * z))
        diff = np.linalg.norm(alpha - prev, ord=2)
        prev = alpha
        steps += 1
    return prev, steps


def svm_dual(K_fit, y, C, tol=1e-10, maxiter=100):
    """C_SVM.fit's QP (SVM.py:78-89): cvxopt.solvers.qp(P=K, q=-y, G=[diag(y); -diag(y)],
    h=[C; 0]), i.e. min 1/2 a'Ka - y'a s.t. 0 <= y_i a_i <= C.  cvxopt is not installed
    here, so this restates the problem and solves it with a Mehrotra predictor-corrector
    primal-dual interior-point method in x = y o a (box 0 <= x <= C, Q = YKY), the
    algorithm family of cvxopt.solvers.qp.  Returns (a, steps, objective).  Pinned against
    scipy's L-BFGS-B on the reference's own 'BFGS' formulation (SVM.py:70-76) in
    tests/test_learners_cpu.py; cvxopt's own numbers are unavailable (parity unpinned)."""
    K_fit = np.asarray(K_fit, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    n = K_fit.shape[0]
    Q = y[:, None] * K_fit * y[None, :]
    x = np.full(n, 0.5 * C)
    z1 = np.ones(n)
    z2 = np.ones(n)

    def step_to_boundary(x, dx, z1, dz1, z2, dz2):
        t = np.inf
        for v, d in ((x, dx), (C - x, -dx), (z1, dz1), (z2, dz2)):
            neg = d < 0  # v + t d >= 0 needs t <= -v / d
            if neg.any():
                t = min(t, np.min(-v[neg] / d[neg]))
        return t

    steps = 0
    for steps in range(maxiter + 1):
        s2 = C - x
        qx = Q @ x
        rd = qx - 1.0 - z1 + z2
        mu = (x @ z1 + s2 @ z2) / (2 * n)
        obj = 0.5 * x @ qx - x.sum()
        if (2 * n * mu <= tol * max(1.0, abs(obj)) and np.max(np.abs(rd)) <= tol) or steps == maxiter:
            break
        M = Q + np.diag(z1 / x + z2 / s2)
        L = np.linalg.cholesky(M)

        def solve(r):
            return np.linalg.solve(L.T, np.linalg.solve(L, r))

        dxa = solve(-rd - z1 + z2)
        dz1a = (-x * z1 - z1 * dxa) / x
        dz2a = (-s2 * z2 + z2 * dxa) / s2
        ta = min(1.0, step_to_boundary(x, dxa, z1, dz1a, z2, dz2a))
        mu_aff = ((x + ta * dxa) @ (z1 + ta * dz1a) + (s2 - ta * dxa) @ (z2 + ta * dz2a)) / (2 * n)
        smu = (mu_aff / mu) ** 3 * mu
        t1 = smu - x * z1 - dxa * dz1a
        t2 = smu - s2 * z2 + dxa * dz2a
        dx = solve(-rd + t1 / x - t2 / s2)
        dz1 = (t1 - z1 * dx) / x
        dz2 = (t2 + z2 * dx) / s2
        t = min(1.0, 0.99 * step_to_boundary(x, dx, z1, dz1, z2, dz2))
        x, z1, z2 = x + t * dx, z1 + t * dz1, z2 + t * dz2
    return y * x, steps, obj
