"""CPU tests: the C-ABI library loads and exports every declared symbol; host logic
(encoding, weights, method grammar, reference-visible error paths) without a GPU."""
import ctypes
import os
import re

import numpy as np
import pandas as pd
import pytest

from conftest import ROOT
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P
import cpu_ref

HEADER = os.path.join(ROOT, "include", "kmgram.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(kmg_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding():
    assert declared_functions() == sorted(L.EXPORTS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(L.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert L.load().kmg_version() == 1


def test_params_struct_layout():
    # kmg_params: 16 int32 + 5 double + 2*64 double + 1 double
    assert ctypes.sizeof(L.KmgParams) == 16 * 4 + 5 * 8 + 128 * 8 + 8


def test_no_device_fails_loudly():
    if L.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(L.KmgError):
        L.Context(0)
    import kernels
    with pytest.raises(L.KmgError):
        kernels.get_spectrum_K(pd.DataFrame({"seq": ["ACGTACGT", "ACGA"]}), 3)


def test_encode_roundtrip():
    seqs = ["ACGT", "", "NNACGTxx", "TTTT", "ACGTACGTAC"]
    codes, lens = E.encode(seqs)
    assert lens.tolist() == [4, 0, 8, 4, 10]
    assert codes[0, :4].tolist() == [0, 1, 2, 3]
    assert codes[2, 0] == codes[2, 1] >= 4 and codes[2, 6] == codes[2, 7] >= 4
    assert codes[2, 0] != codes[2, 6]  # 'N' != 'x'
    assert codes.shape[1] % 4 == 0
    u = ["AĀCGT", "ĀĀ"]
    c2, l2 = E.encode(u)
    assert c2[0, 1] == c2[1, 0] >= 132


def test_encode_non_ascii_cap():
    """123 distinct non-ASCII characters take codes 132..254 (255 stays the padding code);
    a 124th is refused."""
    chars = [chr(0x100 + t) for t in range(123)]
    codes, lens = E.encode(["".join(chars), "A"])
    assert sorted(set(codes[0, :123].tolist())) == list(range(132, 255))
    assert codes[1, 1] == 255  # padding
    with pytest.raises(ValueError):
        E.encode(["".join(chars) + chr(0x100 + 123)])


def test_synthetic_generator_matches_survey():
    codes, lens = E.synthetic(4, 101, seed=20261015)
    assert "".join("ACGT"[c] for c in codes[0, :16]) == "GACTCCTCGGACGGCG"


@pytest.mark.parametrize("k,m", [(1, 1), (3, 1), (5, 2), (9, 1), (12, 3), (16, 5)])
def test_mismatch_weights(k, m):
    w = P.mismatch_weights(k, m)
    assert w == cpu_ref.mismatch_weights(k, m).tolist()
    if m == 1 and k >= 2:
        assert w[:3] == [1 + 3 * k, 4, 2] and all(v == 0 for v in w[3:])


def test_beta_delta_bits():
    # same expression order as kernels.py:61 and :112
    assert P.beta(10, 3) == 2 * (10 - 3 + 1) / 10 / (10 + 1)
    assert P.delta(2) == 1 / 2 / 3
    p = P.make(L.KMG_WDS, d=5, S=3)
    assert list(p.coef_a[:5]) == [P.beta(5, k) for k in range(1, 6)]
    assert list(p.coef_b[:4]) == [P.delta(s) for s in range(4)]
    s = P.make(L.KMG_SUBSTRING, k=3, lbda=0.7)
    assert s.lambda2 == 0.7 ** 2


def _X(seqs):
    return pd.DataFrame({"Id": range(len(seqs)), "seq": seqs})


def test_select_method_unknown_raises_unbound():
    import kernels
    with pytest.raises(UnboundLocalError):
        kernels.select_method(_X(["ACGT"]), "XX_k3")


def test_select_method_bare_wd_indexerror():
    import kernels
    with pytest.raises(IndexError):
        kernels.select_method(_X(["ACGT"]), "WD")


def test_mismatch_error_paths():
    import kernels
    with pytest.raises(ValueError):
        kernels.get_mismatch_K(_X(["ACGT" * 30, "ACGN" * 30]), 3, 1)  # format() ValueError
    with pytest.raises(ValueError):
        kernels.get_mismatch_K(_X(["ACGT" * 30, "ACGT" * 10]), 3, 1)  # length < 101


def test_la_error_paths():
    import kernels
    from scipy.sparse.linalg import ArpackError
    with pytest.raises(ArpackError):
        kernels.get_LA_K(_X(["ACGT" * 25] * 8))
    with pytest.raises(ValueError):
        kernels.get_LA_K(_X(["ACGN"] * 3), eig=0)


def test_gappy_error_paths():
    import kernels
    for k, g in [(3, 1), (3, 0), (2, 1), (1, 1), (2, 0)]:
        with pytest.raises(ValueError):
            kernels.get_gappy_K(_X(["ACGT" * 26] * 3), k, g)


def test_kernel_class_repr():
    from kmgram import Kernel
    assert repr(Kernel("SP_k4")) == "Kernel('SP_k4')"
