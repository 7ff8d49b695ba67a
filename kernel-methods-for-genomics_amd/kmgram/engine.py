"""GramEngine: host orchestration of the device Gram kernels (one HIP device).

Each method takes a list of sequences (str) and returns the full symmetric
``np.ndarray (n, n) float64`` the matching reference function returns
(kernels.py:28-455).  All arithmetic runs in libkmgram.so on the GPU; the host only
encodes sequences, validates reference-visible error cases and copies results back.
"""
import os
import threading

import numpy as np

from . import _lib as L
from . import encode as E
from . import params as P


class GramEngine:
    def __init__(self, device=None):
        if device is None:
            device = int(os.environ.get("KMG_DEVICE", "0"))
        self.device = device
        self._ctx = None
        self._lock = threading.Lock()

    @property
    def ctx(self):
        with self._lock:
            if self._ctx is None:
                self._ctx = L.Context(self.device)
            return self._ctx

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    # ------------------------------------------------------------------ helpers
    def _run(self, params, seqs, out_dtype=L.KMG_F64):
        codes, lens = E.encode(seqs)
        n = len(lens)
        if n == 0:
            return np.zeros((0, 0), dtype=L.DTYPES[out_dtype])
        return self.ctx.gram(params, codes, lens, out_dtype)

    @staticmethod
    def _require_acgt(seqs):
        """format() maps A,C,G,T -> 1..4 and int()s every character (kernels.py:184,193):
        any other character raises ValueError there; so do we."""
        for s in seqs:
            bad = set(s) - set(E.ACGT)
            if bad:
                ch = sorted(bad)[0]
                raise ValueError(f"invalid literal for int() with base 10: '{ch}'")

    # ------------------------------------------------------------------ kernels
    def spectrum(self, seqs, k, out_dtype=L.KMG_F64):
        """get_spectrum_K (kernels.py:28-47): K_ij = <phi_i, phi_j>, integer counts."""
        k = int(k)
        if k < 1:
            raise ValueError("k must be >= 1")
        return self._run(P.make(L.KMG_SPECTRUM, k=k), seqs, out_dtype)

    def mismatch(self, seqs, k, m, normalize=True, window=101, out_dtype=L.KMG_F64):
        """get_mismatch_K (kernels.py:196-217): <Phi_i, Phi_j> then normalize_K."""
        seqs = list(seqs)
        self._require_acgt(seqs)
        short = [len(s) for s in seqs if len(s) < window]
        if short:
            # get_phi_km slices windows up to 101 (kernels.py:171): a shorter sequence
            # yields k-mers of the wrong shape and numpy raises while comparing them.
            raise ValueError(f"operands could not be broadcast together (sequence of length "
                             f"{short[0]} < {window})")
        p = P.make(L.KMG_MISMATCH, k=int(k), m=int(m), window=window,
                   normalize=1 if normalize else 0)
        return self._run(p, seqs, out_dtype)

    def wd(self, seqs, d):
        """get_WD_K (kernels.py:84-101)."""
        return self._run(P.make(L.KMG_WD, d=int(d)), seqs)

    def wds(self, seqs, d, S):
        """get_WDShifts_K (kernels.py:138-155); rows of any lengths (the clipped-slice
        suffix matches of kernels.py:133 are counted on the device)."""
        return self._run(P.make(L.KMG_WDS, d=int(d), S=int(S)), seqs)

    @staticmethod
    def _pair_codes(x, y, length):
        """x and y cut or padded to ``length`` symbols with a code neither uses.  Slices of
        the padded strings that end inside them compare exactly like the reference's
        clipped slices: two clipped slices are equal iff they have the same length and
        symbols, and the padded ones iff they hold the same symbols and pad positions."""
        codes, lens = E.encode([x, y])
        used = set(np.unique(codes[0, :lens[0]]).tolist()) | set(np.unique(codes[1, :lens[1]]).tolist())
        pad = next((c for c in range(4, 255) if c not in used), None)
        if pad is None:
            raise ValueError("no free symbol code to pad the pair with")
        ldc = max(4, -(-length // 4) * 4)
        out = np.full((2, ldc), 255, dtype=np.uint8)
        for r in range(2):
            m = min(int(lens[r]), length)
            out[r, :m] = codes[r, :m]
            out[r, m:length] = pad
        return out, np.full(2, length, dtype=np.int32)

    def _pair_value(self, params, codes, lens):
        return float(self.ctx.gram(params, codes, lens, L.KMG_F64)[0, 1])

    def wd_pair(self, x, y, d, span):
        """get_WD_d(x, y, d, L=span) (kernels.py:64-81) for any L: windows end at or before
        L, so x and y padded to L symbols give every clipped comparison."""
        span = int(span)
        if span <= 1:
            return 0.0  # range(1, L - k + 1) is empty for every k
        codes, lens = self._pair_codes(x, y, span)
        return self._pair_value(P.make(L.KMG_WD, d=int(d), span=span), codes, lens)

    def wds_pair(self, x, y, d, S, span):
        """get_WDShifts_d(x, y, d, S, L=span) (kernels.py:115-135) for any L: windows end
        at or before L + S, so the pair is padded to L + S symbols and the sums run to L."""
        span, S = int(span), int(S)
        if span <= 1:
            return 0.0
        codes, lens = self._pair_codes(x, y, span + S)
        return self._pair_value(P.make(L.KMG_WDS, d=int(d), S=S, span=span), codes, lens)

    def substring(self, seqs, lbda, k):
        """get_string_K (kernels.py:367-382)."""
        return self._run(P.make(L.KMG_SUBSTRING, k=int(k), lbda=lbda), seqs)

    def local_alignment(self, seqs, e=11, d=1, beta=0.5, smith=0, eig=1, intended=False):
        """get_LA_K (kernels.py:273-302), reference semantics (the reference
        always returns an all-zero K, and raises ArpackError for eig=1, n >= 8).

        intended=True: the local-alignment kernel the reference means — five DP arrays
        instead of one aliased array, every cell up to [n_x, n_y], gap opening / extension
        factors exp(-beta e) / exp(-beta d) (g(n) = e + d(n-1), the docstring's affine
        gap) — computed on the device (gram_la_kernel; parity unpinned: the reference
        never produces it).  Like the reference, K itself is returned (its eig step only
        builds K1, kernels.py:288-302)."""
        seqs = list(seqs)
        self._require_acgt(seqs)
        n = len(seqs)
        if intended:
            if not beta > 0:
                raise ValueError("LA kernel needs beta > 0")
            p = P.make(L.KMG_LOCALALIGN, smith=int(smith), la_mode=L.KMG_LA_INTENDED,
                       la_e=e, la_d=d, la_beta=beta)
            return self._run(p, seqs)
        if eig == 1 and n >= 8:
            # eigs(K1) on the all-zero K: ARPACK info=-9 (kernels.py:294)
            from scipy.sparse.linalg import ArpackError
            raise ArpackError(-9)
        p = P.make(L.KMG_LOCALALIGN, smith=int(smith), la_mode=L.KMG_LA_REFERENCE,
                   la_e=e, la_d=d, la_beta=beta)
        return self._run(p, seqs)

    def gappy(self, seqs, k, g, intended=False):
        """get_gappy_K (kernels.py:436-455).

        intended=True: the kernel the reference means to compute (report §3.7) instead of
        its numpy-2 failure: phi_b(x) = [the (k-g)-mer b is an order-preserving
        subsequence of some window x[a:a+k], a in range(101 - k + 1)], K = normalize_K of
        the feature inner products (parity unpinned: the reference never produces it)."""
        seqs = list(seqs)
        self._require_acgt(seqs)
        k, g = int(k), int(g)
        if intended:
            if not (0 <= g < k):
                raise ValueError("intended gappy kernel needs 0 <= g < k")
            short = [len(s) for s in seqs if len(s) < 101]
            if short:
                raise ValueError(f"sequence of length {short[0]} shorter than the 101 window")
            p = P.make(L.KMG_GAPPY, k=k, g=g, window=101, normalize=1,
                       la_mode=L.KMG_MODE_INTENDED)
            return self._run(p, seqs)
        for s in seqs:
            gappy_reference_errors(len(s), k, g)
        return self._run(P.make(L.KMG_GAPPY, k=k, g=g, window=101), seqs)

    # ------------------------------------------------------------------ feature maps
    def features(self, kind, seqs, k, cols, m=0, g=0):
        """float64 [len(seqs), len(cols)]: the reference's per-sequence feature map of each
        sequence at the k-mer codes cols (uint32, base 4, first letter most significant;
        0xFFFFFFFF = a beta no window can equal), on the device (kmg_features):
        KMG_SPECTRUM get_phi_u (kernels.py:12-25), KMG_MISMATCH get_phi_km (161-175),
        KMG_GAPPY gappy_k at k=1, g=0 (420-433)."""
        codes, lens = E.encode(seqs)
        p = P.make(kind, k=int(k), m=int(m), g=int(g), window=101)
        return self.ctx.features(p, codes, lens, cols)

    def features_sym(self, kind, codes, lens, k, col_syms, m=0, bcast=False):
        """float64 [n, len(col_syms)] over symbol columns (kmg_features_sym): codes / lens are
        the rows in the caller's symbol code space, col_syms uint8 [ncols, 16] the betas' codes
        in the same space; bcast: get_phi_km's numpy broadcast of short k-mers (rows shorter
        than the 101 window)."""
        p = P.make(kind, k=int(k), m=int(m), window=101)
        return self.ctx.features_sym(p, codes, lens, col_syms,
                                     L.KMG_FEATURES_BCAST if bcast else 0)

    def substring_b_pair(self, x, y, lbda, k):
        """B_k(lbda, k, x, y) of the substring kernel's recursion (kernels.py:322-342) at the
        full strings, from the device sweep (la_mode KMG_MODE_SS_B)."""
        p = P.make(L.KMG_SUBSTRING, k=int(k), lbda=lbda, la_mode=L.KMG_MODE_SS_B)
        return float(self._run(p, [x, y])[0, 1])

    def normalize(self, K):
        """normalize_K (kernels.py:398-415) in place on a float64 C-contiguous matrix."""
        return self.ctx.normalize(K)

    def center(self, K):
        """center_K (kernels.py:387-395)."""
        return self.ctx.center(np.ascontiguousarray(K, dtype=np.float64))


def gappy_reference_errors(n_x, k, g, window=101):
    """Raise what gappy_k (kernels.py:420-433) raises under numpy 2 for a sequence of
    length n_x, before any work: combinations(x[i:i+k], k-g) refuses r = k-g < 0 once a
    window exists, and `b in gap_set` compares a length-k beta array with each (k-g)-tuple:
    the shapes (k,) and (r,) broadcast only when r == k, r == 1 or k == 1, and the result's
    truth value is defined only for one element.  Returns quietly when gap_set is empty
    (nothing is compared) or k=1, g=0."""
    r = k - g
    if window - k + 1 <= 0:
        return  # no window: gap_set = []
    if r < 0:
        raise ValueError("r must be non-negative")
    # the longest slice x[0:k] holds min(n_x, k) symbols: gap_set is non-empty iff r fits
    if min(n_x, k) < r:
        return
    if r in (k, 1) or k == 1:
        size = 0 if r == 0 else max(r, k)
        if size == 1:
            return
        if size == 0 or r == 0:
            raise ValueError("The truth value of an empty array is ambiguous. Use "
                             "`array.size > 0` to check that an array is not empty.")
        raise ValueError("The truth value of an array with more than one element is "
                         "ambiguous. Use a.any() or a.all()")
    raise ValueError(f"operands could not be broadcast together with shapes ({k},) ({r},) ")


_default = None
_default_lock = threading.Lock()


def default_engine():
    global _default
    with _default_lock:
        if _default is None:
            _default = GramEngine()
        return _default
