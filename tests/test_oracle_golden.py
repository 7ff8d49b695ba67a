"""Pin the oracle (oracle/cpu_ref.py and oracle/kmg_oracle.c) against the golden vectors
produced by the unmodified reference kernels.py (tests/golden/make_golden.py).
CPU only; bit-exact for every integer and float64 fixture."""
import numpy as np
import pytest

import cpu_ref
import cref
from golden_io import load_xtr0, sha256_f64
from kmgram.encode import encode


def _enc(golden, name):
    return encode(golden.seqs(name))


@pytest.mark.parametrize("k", range(1, 9))
def test_spectrum_xtr0(golden, k):
    name = f"SP_k{k}_xtr0_n48"
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    assert np.array_equal(cpu_ref.spectrum(codes, lens, k).astype(np.float64), ref)
    assert np.array_equal(cref.spectrum(codes, lens, k).astype(np.float64), ref)


@pytest.mark.parametrize("name,k", [("SP_k3_ragged", 3), ("SP_k5_ragged", 5), ("SP_k8_stress", 8)])
def test_spectrum_ragged_and_stress(golden, name, k):
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    assert np.array_equal(cpu_ref.spectrum(codes, lens, k).astype(np.float64), ref)
    assert np.array_equal(cref.spectrum(codes, lens, k).astype(np.float64), ref)


def test_spectrum_config1_sha(golden):
    """BASELINE configs[0]: SP k=6 on all of Xtr0 (N=2000), SHA-256 of the float64 K."""
    codes, lens = load_xtr0()
    e = golden.entry("SP_k6_xtr0_full")
    K = cref.spectrum(codes, lens, 6)
    assert [int(v) for v in K.sum(axis=1)] == e["row_sums"]
    assert np.array_equal(K[:64, :64], golden.K("SP_k6_xtr0_full__block"))
    assert sha256_f64(K) == e["sha256_f64"]


@pytest.mark.parametrize("name", ["MM_k3_m1_xtr0_n32", "MM_k4_m1_xtr0_n32", "MM_k5_m1_xtr0_n32",
                                  "MM_k6_m1_xtr0_n32", "MM_k5_m1_stress", "MM_k5_m0_xtr0_n16",
                                  "MM_k5_m2_xtr0_n16", "MM_k4_m3_xtr0_n12"])
def test_mismatch(golden, name):
    e = golden.entry(name)
    k, m = e["kwargs"]["k"], e["kwargs"]["m"]
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    assert np.array_equal(cref.mismatch_rows(codes, lens, k, m), ref)
    if len(lens) <= 16:
        assert np.array_equal(cpu_ref.mismatch(codes, lens, k, m), ref)


def test_mismatch_k9_sha(golden):
    name = "MM_k9_m1_xtr0_n8"
    codes, lens = _enc(golden, name)
    K = cref.mismatch_rows(codes, lens, 9, 1)
    assert np.array_equal(K, golden.K(name))
    assert sha256_f64(K) == golden.entry(name)["sha256_f64"]
    # survey-recorded raw integers
    raw = cref.mismatch_raw(codes, lens, 9, 1)
    assert raw[0].tolist() == [2628, 128, 56, 40, 554, 28, 28, 10]


@pytest.mark.parametrize("k,m", [(2, 1), (3, 1), (3, 2), (2, 0), (3, 3)])
def test_mismatch_closed_form_vs_phi(golden, k, m):
    """sum_{a,b} w_m[ham] equals the literal Phi Phi^T over all 4^k betas."""
    codes, lens = _enc(golden, "MM_k4_m3_xtr0_n12")
    codes, lens = codes[:5], lens[:5]
    a = cpu_ref.mismatch_phi_bruteforce(codes, lens, k, m)
    b = cpu_ref.mismatch_raw(codes, lens, k, m)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("d", [1, 2, 4, 5, 10])
def test_wd(golden, d):
    name = f"WD_d{d}_xtr0_n64"
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    assert np.array_equal(cref.wd(codes, lens, d), ref)
    if d in (1, 4):
        assert np.array_equal(cpu_ref.wd(codes[:20], lens[:20], d), ref[:20, :20])


def test_wd_stress(golden):
    codes, lens = _enc(golden, "WD_d5_stress")
    assert np.array_equal(cref.wd(codes, lens, 5), golden.K("WD_d5_stress"))


@pytest.mark.parametrize("d,S", [(1, 0), (3, 1), (5, 3), (10, 5)])
def test_wds(golden, d, S):
    name = f"WDS_d{d}_s{S}_xtr0_n24"
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    assert np.array_equal(cref.wds(codes, lens, d, S), ref)
    if d <= 3:
        assert np.array_equal(cpu_ref.wds(codes[:8], lens[:8], d, S), ref[:8, :8])


def test_wds_stress(golden):
    codes, lens = _enc(golden, "WDS_d5_s3_stress")
    assert np.array_equal(cref.wds(codes, lens, 5, 3), golden.K("WDS_d5_s3_stress"))


@pytest.mark.parametrize("name", ["WD_d5_ragged", "WD_d1_ragged", "WDS_d1_s1_ragged",
                                  "WDS_d3_s2_ragged", "WDS_d5_s3_ragged", "WDS_d4_s7_ragged"])
def test_wd_wds_ragged(golden, name):
    """Rows of different lengths: slices clip and compare as strings (kernels.py:79,133)."""
    e = golden.entry(name)
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    kw = e["kwargs"]
    if name.startswith("WDS"):
        assert np.array_equal(cref.wds(codes, lens, kw["d"], kw["S"]), ref)
        assert np.array_equal(cpu_ref.wds(codes[:6], lens[:6], kw["d"], kw["S"]), ref[:6, :6])
    else:
        assert np.array_equal(cref.wd(codes, lens, kw["d"]), ref)
        assert np.array_equal(cpu_ref.wd(codes[:6], lens[:6], kw["d"]), ref[:6, :6])


def test_wd_pair_any_L(golden):
    """get_WD_d / get_WDShifts_d with L != len(x) (kernels.py:64-81, 115-135)."""
    names = golden.names("WDd_p") + golden.names("WDSd_p")
    assert len(names) >= 40
    for name in names:
        e = golden.entry(name)
        x, y = golden.seqs(name)
        kw = e["kwargs"]
        if name.startswith("WDSd"):
            v = cpu_ref.wds_pair(x, y, kw["d"], kw["S"], kw["L"])
        else:
            v = cpu_ref.wd_pair(x, y, kw["d"], kw["L"])
        assert v == golden.K(name)[0], name


@pytest.mark.parametrize("lb,k", [(0.5, 3), (1.0, 3), (0.7, 5), (0.3, 2), (0.5, 1)])
def test_substring(golden, lb, k):
    name = f"SS_l{lb}_k{k}_xtr0_n10"
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    assert np.array_equal(cref.ss(codes, lens, lb, k), ref)
    if k <= 3:
        assert np.array_equal(cpu_ref.substring(codes[:4], lens[:4], lb, k), ref[:4, :4])


def test_substring_short(golden):
    name = "SS_l0.5_k3_short"
    codes, lens = _enc(golden, name)
    ref = golden.K(name)
    assert np.array_equal(cref.ss(codes, lens, 0.5, 3), ref)
    assert np.array_equal(cpu_ref.substring(codes, lens, 0.5, 3), ref)


@pytest.mark.parametrize("name", ["LA_smith0_eig0_n6", "LA_smith1_eig0_n6", "LA_smith0_eig1_n6"])
def test_local_alignment_zero(golden, name):
    ref = golden.K(name)
    assert np.array_equal(cpu_ref.local_alignment_reference(ref.shape[0]), ref)


def test_recorded_errors(golden):
    assert golden.entry("LA_smith0_eig1_n8")["error"] == "ArpackError"
    assert golden.entry("GP_k3_g1_n4")["error"] == "ValueError"
    assert golden.entry("GP_k3_g0_n4")["error"] == "ValueError"
    assert golden.entry("select_XX_k3_n6")["error"] == "UnboundLocalError"


def test_select_grammar_goldens(golden):
    """select_method's parsing (kernels.py:479-502), against the direct fixtures."""
    seqs6 = golden.seqs("select_SP_k4_n6")
    codes, lens = encode(seqs6)
    assert np.array_equal(golden.K("select_SP_k4_n6"), cpu_ref.spectrum(codes, lens, 4))
    assert np.array_equal(golden.K("select_WD_k5_n6"), cref.wd(codes, lens, 5))
    assert np.array_equal(golden.K("select_WD_d4_n6"), cref.wd(codes, lens, 4))
    assert np.array_equal(golden.K("select_MM_k4_m1_n6"), cref.mismatch_rows(codes, lens, 4, 1))
    assert np.array_equal(golden.K("select_WDS_d3_s1_n6"), cref.wds(codes, lens, 3, 1))
    assert np.array_equal(golden.K("select_SS_l0.5_k2_n6"), cref.ss(codes, lens, 0.5, 2))
    assert np.array_equal(golden.K("select_LA_e11_d1_b0.5_smith0_eig0_n6"), np.zeros((6, 6)))


def test_center_restatement():
    rng = np.random.default_rng(0)
    A = rng.standard_normal((7, 7))
    K = A @ A.T
    n = 7
    B = np.eye(n) - np.ones((n, n)) / n
    assert np.allclose(cpu_ref.center(K), B @ K @ B)
