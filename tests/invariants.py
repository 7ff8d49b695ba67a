"""Size-independent checks of whole Gram matrices (test infrastructure): exact integer
row sums of the spectrum and mismatch (k, 1) kernels, computed on the host from k-mer
histograms without forming the 4^k-wide feature maps of kernels.py:12-25 / 161-175."""
import numpy as np


def kmers(codes, k, window=None):
    """int64 [n, P] k-mer codes (first letter most significant) of windows 0..L-k, all ACGT."""
    L = codes.shape[1] if window is None else window
    P = L - k + 1
    km = np.zeros((codes.shape[0], P), dtype=np.int64)
    for q in range(k):
        km = km * 4 + codes[:, q:q + P]
    return km


def spectrum_row_sums(codes, k, rows=None):
    """sum_j K_ij = sum_u phi_i(u) * T(u), T = total count of u over all sequences
    (full-length ACGT rows)."""
    km = kmers(codes, k)
    T = np.bincount(km.ravel(), minlength=4 ** k)
    sub = km if rows is None else km[rows[0]:rows[1]]
    return T[sub].sum(axis=1)


def mismatch1_row_sums(codes, k, window=101, rows=None, cols=None):
    """Raw mismatch (k, m=1) row sums: sum_j K_ij = <Phi_i, C> with C = sum_j Phi_j the
    column sums of the neighbour-count map, C(b) = sum_{v: ham(v, b) <= 1} T(v), and
    Phi_i = sum_a 1[B_1(u_a)], so sum_j K_ij = sum_a sum_{b in B_1(u_a)} C(b).
    cols = (c0, c1): the sums over the columns [c0, c1) only (T from those sequences), i.e.
    the row sums of a column block K[:, c0:c1]."""
    km = kmers(codes, k, window)
    tk = km if cols is None else km[cols[0]:cols[1]]
    T = np.bincount(tk.ravel(), minlength=4 ** k).astype(np.int64)
    b = np.arange(4 ** k, dtype=np.int64)
    flips = [d << (2 * (k - 1 - p)) for p in range(k) for d in (1, 2, 3)]
    C = T.copy()
    for f in flips:
        C += T[b ^ f]
    sub = km if rows is None else km[rows[0]:rows[1]]
    s = C[sub].sum(axis=1)
    for f in flips:
        s += C[sub ^ f].sum(axis=1)
    return s
