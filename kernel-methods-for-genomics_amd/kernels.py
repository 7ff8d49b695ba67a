"""Drop-in replacement of afiliot/Kernel-Methods-For-Genomics ``kernels.py``.

Same module name, same public functions and signatures, same return contract
(fresh C-contiguous ``np.ndarray (n, n) float64``; ``normalize_K`` mutates in place),
same method-string grammar in ``select_method`` (kernels.py:461-505) — but every
Gram matrix is computed on an AMD MI355X by libkmgram.so (hand-written HIP kernels
for gfx950).  Put this directory on ``sys.path`` ahead of the reference and
``import kernels as km`` in utils.py / run.py keeps working unchanged.

There is no CPU fallback: without the built library or a visible HIP device every
Gram call raises.
"""
import functools

import numpy as np

from kmgram import _lib as _L
from kmgram import engine as _engine
from kmgram.encode import as_sequence_list as _seqs
from kmgram.params import beta, delta  # noqa: F401  (reference helpers, kernels.py:53,106)

__all__ = [
    "get_spectrum_K", "get_WD_K", "get_WDShifts_K", "get_mismatch_K", "get_LA_K",
    "get_string_K", "get_gappy_K", "center_K", "normalize_K", "select_method", "beta",
    "delta", "letter_to_num", "format", "S", "get_WD_d", "get_WDShifts_d", "K_k",
    "affine_align", "Smith_Waterman", "get_phi_u", "get_phi_km", "gappy_k", "B_k", "rec",
]

# substitution matrix extracted from BLOSUM62 (kernels.py:223)
S = np.array([[4, 0, 0, 0], [0, 9, -3, -1], [0, -3, 6, 2], [0, -1, -2, 5]])


def _eng():
    return _engine.default_engine()


# ----------------------------------------------------------------------- Gram family
def get_spectrum_K(X, k):
    """Spectrum kernel SP(k) (kernels.py:28-47)."""
    return _eng().spectrum(_seqs(X), k)


def get_WD_K(X, d):
    """Weighted degree kernel WD(d) (kernels.py:84-101)."""
    return _eng().wd(_seqs(X), d)


def get_WDShifts_K(X, d, S):
    """Weighted degree kernel with shifts WDS(d, S) (kernels.py:138-155)."""
    return _eng().wds(_seqs(X), d, S)


def get_mismatch_K(X, k, m):
    """Mismatch kernel (k, m), normalised (kernels.py:196-217)."""
    return _eng().mismatch(_seqs(X), k, m)


def get_LA_K(X, e=11, d=1, beta=0.5, smith=0, eig=1):
    """Local alignment kernel (kernels.py:273-302), reference semantics."""
    return _eng().local_alignment(_seqs(X), e, d, beta, smith, eig)


def get_string_K(X, lbda, k):
    """Substring kernel SS(lambda, k) (kernels.py:367-382)."""
    return _eng().substring(_seqs(X), lbda, k)


def get_gappy_K(X, k, g):
    """Gappy kernel GP(k, g) (kernels.py:436-455)."""
    return _eng().gappy(_seqs(X), k, g)


# ----------------------------------------------------------------------- helpers
def center_K(K):
    """(I - 11^T/n) K (I - 11^T/n) (kernels.py:387-395)."""
    return _eng().center(np.asarray(K))


def normalize_K(K):
    """In place: K_ij /= sqrt(K_ii) sqrt(K_jj), diagonal := 1; unchanged if K[0,0] == 1
    (kernels.py:398-415).  Returns the same object."""
    if K[0, 0] == 1:
        print('Kernel already normalized')
        return K
    if K.dtype == np.float64 and K.flags.c_contiguous:
        _eng().normalize(K)
        return K
    work = np.array(K, dtype=np.float64, order="C")
    _eng().normalize(work)
    K[...] = work  # same cast the reference's element-wise `K[i, j] /= ...` applies
    return K


def letter_to_num(x):
    """'A'->'1', 'C'->'2', 'G'->'3', 'T'->'4' (kernels.py:178-184)."""
    return x.replace('A', '1').replace('C', '2').replace('G', '3').replace('T', '4')


def format(x):  # noqa: A001  (reference name, kernels.py:187-193)
    """'AGCT' -> array([1, 3, 2, 4])."""
    return np.array(list(letter_to_num(x))).astype(int)


# ----------------------------------------------------------------------- pair helpers
def _pair(fn, x, y):
    K = fn([x, y])
    return K[0, 1]


def get_WD_d(x, y, d, L):
    """WD value of one pair (kernels.py:64-81), any L (slices clip as Python's do)."""
    return _eng().wd_pair(x, y, d, L)


def get_WDShifts_d(x, y, d, S, L):
    """WDS value of one pair (kernels.py:115-135), any L."""
    return _eng().wds_pair(x, y, d, S, L)


def K_k(lbda, k, x, y):
    """Substring kernel of one pair (kernels.py:344-364)."""
    return _pair(lambda s: _eng().substring(s, lbda, k), x, y)


def affine_align(x, y, e, d, beta):
    """Reference LA value of one pair: always 0.0 (kernels.py:226-246)."""
    _engine.GramEngine._require_acgt([x, y])
    return 0.0


def Smith_Waterman(x, y, e=11, d=1, beta=0.5):
    """Reference Smith-Waterman LA value of one pair: always 0.0 (kernels.py:249-270)."""
    _engine.GramEngine._require_acgt([x, y])
    return 0.0


# ----------------------------------------------------------------------- feature maps
# The reference's per-sequence feature maps, evaluated on the device (kmg_features): the
# host only maps each beta to its base-4 k-mer code (the column the device scores).
_NO_MATCH = 0xFFFFFFFF
_ACGT_CODE = np.full(256, 255, dtype=np.uint8)
for _i, _c in enumerate(b"ACGT"):
    _ACGT_CODE[_c] = _i


def _codes_of_rows(rows, k):
    """int letter rows (values 0..3) [nb, k] -> base-4 codes, first letter most significant."""
    out = np.zeros(rows.shape[0], dtype=np.uint64)
    for q in range(k):
        out = out * np.uint64(4) + rows[:, q].astype(np.uint64)
    return out.astype(np.uint32)


def _string_beta_cols(betas, k):
    """get_phi_u's string betas -> column codes, or None when a beta of length k holds a
    letter outside A/C/G/T (those take the symbol columns).  A beta of another length than k
    equals no window (x[i:i+k] always holds k symbols)."""
    if not all(isinstance(b, str) for b in betas):
        raise TypeError("get_phi_u: betas must be strings (kernels.py:37)")
    cols = np.full(len(betas), _NO_MATCH, dtype=np.uint32)
    sel = np.fromiter((len(b) == k for b in betas), dtype=bool, count=len(betas))
    if sel.any():
        try:
            raw = "".join(b for b, t in zip(betas, sel) if t).encode("ascii")
        except UnicodeEncodeError:
            return None
        letters = _ACGT_CODE[np.frombuffer(raw, dtype=np.uint8)]
        if (letters > 3).any():
            return None
        cols[sel] = _codes_of_rows(letters.reshape(-1, k), k)
    return cols


# ---- symbol columns: any letter / value compares by identity (kmg_features_sym)
_PAD = 255  # the code no window holds


def _symbol_codes(keys):
    """A code per distinct key: A/C/G/T (or format()ed 1..4) -> 0..3 in the reference's beta
    order, every other key its own code from 4 (< 255: the padding code)."""
    table = {}
    for key in keys:
        if key not in table:
            table[key] = None
    out, nxt = {}, 4
    for key in table:
        fixed = _FIXED_CODE.get(key)
        if fixed is not None:
            out[key] = fixed
        else:
            out[key] = nxt
            nxt += 1
    if nxt > _PAD:
        raise NotImplementedError("feature maps: more than 251 distinct symbols outside A/C/G/T")
    return out


_FIXED_CODE = {"A": 0, "C": 1, "G": 2, "T": 3, 1: 0, 2: 1, 3: 2, 4: 3}


def _sym_columns(rows, k, code):
    """Beta symbol lists -> uint8 [len(rows), 16] columns (None: a beta no window equals)."""
    cols = np.zeros((len(rows), 16), dtype=np.uint8)
    for j, r in enumerate(rows):
        if r is None:
            cols[j, :k] = _PAD
        else:
            cols[j, :k] = [code[s] for s in r]
    return cols


def _phi_u_symbols(x, k, betas):
    """get_phi_u with betas outside A/C/G/T: x and the betas in one symbol code space, string
    equality by code identity on the device."""
    code = _symbol_codes(list(x) + [c for b in betas if len(b) == k for c in b])
    xc = np.array([[code[c] for c in x]], dtype=np.uint8).reshape(1, -1)
    codes = np.full((1, max(4, -(-len(x) // 4) * 4)), _PAD, dtype=np.uint8)
    codes[0, :len(x)] = xc
    rows = [list(b) if len(b) == k else None for b in betas]
    return _eng().features_sym(_L.KMG_SPECTRUM, codes, np.array([len(x)], dtype=np.int32), k,
                               _sym_columns(rows, k, code))[0]


def _phi_km_symbols(xa, k, m, B, bcast):
    """get_phi_km over format()ed values outside 1..4 (in x or in the betas) or with numpy's
    broadcast of short k-mers: integer equality by code identity on the device."""
    xs = [v.item() if hasattr(v, "item") else v for v in xa.reshape(-1)]
    bs = [[v.item() if hasattr(v, "item") else v for v in row] for row in B]
    code = _symbol_codes(xs + [v for row in bs for v in row])
    codes = np.full((1, max(4, -(-len(xs) // 4) * 4)), _PAD, dtype=np.uint8)
    codes[0, :len(xs)] = [code[v] for v in xs]
    return _eng().features_sym(_L.KMG_MISMATCH, codes, np.array([len(xs)], dtype=np.int32), k,
                               _sym_columns(bs, k, code), m=m, bcast=bcast)[0]


def _format_rows(a):
    """format()ed letters (1..4 for A, C, G, T) -> 0..3; anything else -> 4 (a symbol that
    mismatches every letter, as an integer outside 1..4 compares in kernels.py:174)."""
    a = np.asarray(a)
    ok = (a >= 1) & (a <= 4)
    return np.where(ok, a - 1, 4).astype(np.uint8), bool(ok.all())


def _formatted(x):
    """x as get_phi_km / gappy_k receive it, format(x) (kernels.py:209, 448); a str is
    format()ed here first (the reference's own callers always pass format(x))."""
    return format(x) if isinstance(x, str) else np.asarray(x)


def _decoded(x):
    """format()ed integer letters back to the sequence string the encoder takes; symbols
    outside 1..4 become 'N' (they equal no letter of a beta)."""
    codes, _ = _format_rows(x)
    return "".join("ACGTN"[c] for c in codes.reshape(-1))


def _formatted_beta_cols(betas, k, who):
    B = np.asarray(betas)
    if B.ndim == 1 and k == 1:
        B = B.reshape(-1, 1)
    if B.size == 0:
        return np.zeros(len(betas), dtype=np.uint32)
    if B.ndim != 2 or B.shape[1] != k:
        raise NotImplementedError(f"{who}: betas must be format()ed {k}-mers")
    rows, ok = _format_rows(B)
    if not ok:
        raise NotImplementedError(f"{who}: betas outside the A/C/G/T alphabet")
    return _codes_of_rows(rows, k)


def get_phi_u(x, k, betas):
    """Spectrum feature vector of x (kernels.py:12-25): phi[j] = #{i < len(x)-k+1 :
    x[i:i+k] == betas[j]}, float64[len(betas)].  Computed on the device."""
    k = int(k)
    if k < 1:
        raise ValueError("k must be >= 1")
    if not isinstance(x, str):
        raise TypeError("get_phi_u: x must be a DNA string (kernels.py:39-40)")
    betas = list(betas)
    if not betas:
        return np.zeros(0)
    if k > 16:
        raise NotImplementedError("get_phi_u: k > 16")
    cols = _string_beta_cols(betas, k)
    if cols is None:
        return _phi_u_symbols(x, k, betas)
    return _eng().features(_L.KMG_SPECTRUM, [x], k, cols)[0]


def get_phi_km(x, k, m, betas):
    """Mismatch feature vector of format(x) (kernels.py:161-175): phi[j] = #{i < 101-k+1 :
    sum(x[i:i+k] != betas[j]) <= m}, float64[len(betas)].  Computed on the device.  A row
    shorter than the 101 window raises the ValueError numpy raises comparing its first
    short k-mer (kernels.py:174)."""
    k, m = int(k), int(m)
    if k < 1:
        raise ValueError("k must be >= 1")
    xa = _formatted(x).reshape(-1)
    n_x = len(xa)
    if len(betas) == 0:
        return np.zeros(0)
    quirk = False
    if n_x < 101:
        # window lengths min(k, n_x - i), i in range(101 - k + 1): numpy broadcasts a
        # short k-mer of 1 symbol (or 0 at k = 1) against the beta and raises for others
        for i in range(101 - k + 1):
            ln = max(0, min(k, n_x - i))
            if ln == k:
                continue
            if ln == 1 or k == 1:
                quirk = True
                continue
            raise ValueError(f"operands could not be broadcast together with shapes ({ln},) "
                             f"({k},) ")
    if k > 16:
        raise NotImplementedError("get_phi_km: k > 16")
    B = np.asarray(betas)
    if B.ndim == 1 and k == 1:
        B = B.reshape(-1, 1)
    if B.ndim != 2 or B.shape[1] != k:
        raise NotImplementedError(f"get_phi_km: betas must be format()ed {k}-mers")
    _, x_ok = _format_rows(xa)
    _, b_ok = _format_rows(B)
    if quirk or not x_ok or not b_ok:
        return _phi_km_symbols(xa, k, m, B, quirk)
    cols = _codes_of_rows(_format_rows(B)[0], k)
    return _eng().features(_L.KMG_MISMATCH, [_decoded(xa)], k, cols, m=m)[0]


def gappy_k(x, k, g, betas):
    """Gappy feature vector of format(x) (kernels.py:420-433): phi[j] = [betas[j] in
    gap_set], gap_set = the (k-g)-combinations of every window x[i:i+k], i < 101-k+1.
    Under numpy 2 `b in gap_set` compares a length-k array with (k-g)-tuples, which raises
    for every (k, g) but k=1, g=0 once gap_set is non-empty (engine.gappy_reference_errors,
    pinned to the reference's own failures); k=1, g=0 (letter presence in x[0:101]) is
    computed on the device."""
    k, g = int(k), int(g)
    xa = _formatted(x).reshape(-1)
    if k - g < 0 or len(betas) > 0:
        _engine.gappy_reference_errors(len(xa), k, g)
    if len(betas) == 0:
        return np.zeros(0)
    if not (k == 1 and g == 0):
        return np.zeros(len(betas))  # gap_set is empty (no error above): no beta is in it
    cols = _formatted_beta_cols(betas, 1, "gappy_k")
    return _eng().features(_L.KMG_GAPPY, [_decoded(xa)], 1, cols, g=0)[0]


def rec(func):
    """Memoise ``func`` on the printed form of its arguments, '[a]-[b]-...' (the key of
    kernels.py:308-319): calls whose arguments print alike share one result."""
    memo = {}

    @functools.wraps(func)
    def recd(*args):
        key = "-".join("[%s]" % a for a in args)  # (a tuple argument formats as the reference's)
        if key not in memo:
            memo[key] = func(*args)
        return memo[key]
    return recd


@rec
def B_k(lbda, k, x, y):
    """Auxiliary B_k(x, y) of the substring kernel's recursion (kernels.py:322-342), read
    off the device sweep (KMG_MODE_SS_B): 1 for k = 0, 0 when a string is shorter than k
    (the reference's integer base cases), else the float64 recursion value."""
    k = int(k)
    if k == 0:
        return 1
    if len(x) < k or len(y) < k:
        return 0
    return _eng().substring_b_pair(x, y, lbda, k)


# ----------------------------------------------------------------------- dispatch
def select_method(X, method):
    """Compute the kernel named by ``method`` (grammar of kernels.py:461-505):
    SP_k{k}, WD_d{d}, WDS_d{d}_s{S}, MM_k{k}_m{m}, LA_e{e}_d{d}_b{beta}_smith{0/1}_eig{0/1},
    SS_l{lambda}_k{k}, GP_k{k}_g{g}.  Field values are read as ``int(tok[1:])`` /
    ``float(tok[1:])`` exactly like the reference, and an unknown method fails the way
    the reference does (UnboundLocalError on ``K``)."""
    m = method.split('_')
    if method[:2] == 'SP':
        k = int(m[1][1:])
        K = get_spectrum_K(X, k)
    elif method[:2] == 'WD' and method[2] != 'S':
        print(m)
        d = int(m[1][1:])
        K = get_WD_K(X, d)
    elif method[:2] == 'MM':
        k, m = int(m[1][1:]), int(m[2][1:])
        K = get_mismatch_K(X, k, m)
    elif method[:2] == 'LA':
        e, d, beta_ = [float(m[i][1:]) for i in range(1, 4)]
        smith, eig = int(m[4][5:]), int(m[5][3:])
        K = get_LA_K(X, e, d, beta_, smith, eig)
    elif method[:3] == 'WDS':
        d, S_ = int(m[1][1:]), int(m[2][1:])
        K = get_WDShifts_K(X, d, S_)
    elif method[:2] == 'SS':
        lbda, k = float(m[1][1:]), int(m[2][1:])
        K = get_string_K(X, lbda, k)
    elif method[:2] == 'GP':
        k, g = int(m[1][1:]), int(m[2][1:])
        K = get_gappy_K(X, k, g)
    else:
        NotImplementedError('Method not implemented. Please refer to the documentation for '
                            'choosing among available methods')
    return K  # noqa: F821  (UnboundLocalError for unknown methods, as in the reference)
