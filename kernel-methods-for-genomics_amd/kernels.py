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
import numpy as np

from kmgram import engine as _engine
from kmgram.encode import as_sequence_list as _seqs
from kmgram.params import beta, delta  # noqa: F401  (reference helpers, kernels.py:53,106)

__all__ = [
    "get_spectrum_K", "get_WD_K", "get_WDShifts_K", "get_mismatch_K", "get_LA_K",
    "get_string_K", "get_gappy_K", "center_K", "normalize_K", "select_method", "beta",
    "delta", "letter_to_num", "format", "S", "get_WD_d", "get_WDShifts_d", "K_k",
    "affine_align", "Smith_Waterman",
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
