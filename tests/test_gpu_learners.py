"""GPU parity of the dense learners on K (kmg_krr_solve / kmg_klr_fit: the blocked Cholesky
of csrc/kmg_solve.hip -- or rocSOLVER potrf with KMG_CHOL=0 --, rocSOLVER LU fallback, HIP IRLS
kernels) through the drop-in KRR.py / KLR.py.

Pinned by golden vectors from the unmodified reference KRR.py / KLR.py
(tests/golden/make_learner_golden.py).  The reference inverts with np.linalg.inv; the device
factorises and solves, so alpha agrees to rounding scaled by the system's condition number:
rtol 1e-8 below (kappa <= ~1e3 for these systems), support-vector sets and predictions exact.
"""
import numpy as np
import pandas as pd
import pytest

import cpu_ref
import learner_cases as LC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def case_data():
    return LC.load()


@pytest.mark.parametrize("case", range(4))
def test_dropin_learner_matches_reference(engine, case_data, case):
    from KRR import KRR
    from KLR import KLR
    K, labels, meta, arr = case_data
    m = meta[f"case{case}"]
    ID = np.arange(LC.N_ALL)
    cls = KRR if m["learner"] == "KRR" else KLR
    model = cls(K, ID, **m["kwargs"])
    model.fit(pd.DataFrame({"Id": ID[:LC.N_FIT]}),
              pd.DataFrame({"Id": ID[:LC.N_FIT], "Bound": labels[:LC.N_FIT]}))
    pred = model.predict(pd.DataFrame({"Id": ID[LC.N_FIT:]}))
    tag = f"case{case}"
    assert np.array_equal(model.idx_sv, arr[f"{tag}_idx_sv"])
    np.testing.assert_allclose(model.a, arr[f"{tag}_a"], rtol=1e-8, atol=1e-10)
    assert model.b == pytest.approx(m["b"], rel=1e-7, abs=1e-9)
    assert np.array_equal(pred, arr[f"{tag}_pred"])
    assert model.score(pred, labels[LC.N_FIT:]) == pytest.approx(m["score"])


def _psd(n, r, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((n, r))
    return cpu_ref.normalize(A @ A.T + 1e-3 * np.eye(n))


@pytest.mark.parametrize("n", [1, 7, 64, 513, 2000])
def test_krr_solve_vs_oracle(ctx, n):
    K = _psd(n, max(1, n // 2), n)
    y = np.where(np.random.default_rng(n + 1).random(n) > 0.5, 1.0, -1.0)
    got = ctx.krr_solve(K, y, 0.05)
    ref = cpu_ref.krr_alpha(K, y, 0.05)
    np.testing.assert_allclose(got, ref, rtol=1e-9, atol=1e-12)


def test_krr_solve_strided_view(ctx):
    """A sub-block of a larger K (row stride ld > n) is read in place."""
    K = _psd(300, 100, 3)
    y = np.ones(200)
    sub = K[:200, :200]
    np.testing.assert_allclose(ctx.krr_solve(sub, y, 0.1), cpu_ref.krr_alpha(sub, y, 0.1),
                               rtol=1e-9, atol=1e-12)


def test_krr_indefinite_uses_lu(ctx):
    """Not positive definite (Cholesky fails) but non-singular: inv() succeeds in the
    reference, so the device falls back to LU and must agree."""
    rng = np.random.default_rng(11)
    B = rng.standard_normal((150, 150))
    K = (B + B.T) / 2  # symmetric indefinite
    y = rng.standard_normal(150)
    np.testing.assert_allclose(ctx.krr_solve(K, y, 0.0), cpu_ref.krr_alpha(K, y, 0.0),
                               rtol=1e-7, atol=1e-9)


def test_krr_singular_raises_linalgerror(ctx):
    K = np.zeros((5, 5))
    with pytest.raises(np.linalg.LinAlgError):
        ctx.krr_solve(K, np.ones(5), 0.0)
    with pytest.raises(np.linalg.LinAlgError):
        cpu_ref.krr_alpha(K, np.ones(5), 0.0)


@pytest.mark.parametrize("n,lbda,tol,maxiter", [(50, 0.1, 1e-5, 50), (800, 0.01, 1e-8, 30),
                                                (300, 1.0, 1e-5, 1), (200, 0.1, np.inf, 5)])
def test_klr_fit_vs_oracle(ctx, n, lbda, tol, maxiter):
    K = _psd(n, n // 3 + 1, n + 5)
    y = np.where(np.random.default_rng(n).random(n) > 0.4, 1.0, -1.0)
    got, it = ctx.klr_fit(K, y, lbda, tol, maxiter)
    ref, steps = cpu_ref.klr_alpha(K, y, lbda, tol, maxiter)
    assert it == steps
    np.testing.assert_allclose(got, ref, rtol=1e-8, atol=1e-11)


def test_learner_empty(ctx):
    assert ctx.krr_solve(np.zeros((0, 0)), np.zeros(0), 0.1).shape == (0,)
    a, it = ctx.klr_fit(np.zeros((0, 0)), np.zeros(0), 0.1, 1e-5, 10)
    assert a.shape == (0,) and it == 0


# ---------------------------------------------------------------- C_SVM (SVM.py:78-89)
# cvxopt is not installed, so the reference's own numbers cannot be produced here (parity
# unpinned to cvxopt); the device interior point is checked against the oracle's
# (oracle/cpu_ref.svm_dual, itself checked against L-BFGS-B in test_learners_cpu.py):
# same optimum to 1e-9 relative in the objective, alpha within 1e-5 * C.
@pytest.mark.parametrize("n,C", [(1, 1.0), (40, 0.1), (300, 1.0), (300, 10.0), (2000, 2.0)])
def test_svm_fit_vs_oracle(ctx, n, C):
    K = _psd(n, max(1, n // 4), 3 * n + 1)
    y = np.where(np.random.default_rng(n).random(n) > 0.5, 1.0, -1.0)
    a, steps, obj = ctx.svm_fit(K, y, C)
    ra, rsteps, robj = cpu_ref.svm_dual(K, y, C)
    assert steps < 100
    assert obj == pytest.approx(robj, rel=1e-9, abs=1e-12)
    np.testing.assert_allclose(a, ra, atol=1e-5 * C, rtol=0)
    x = y * a
    assert np.all(x >= 0) and np.all(x <= C)


@pytest.mark.parametrize("C", [0.5, 1.9])
def test_dropin_csvm_on_xtr0(engine, C):
    """run.py's learner (C_SVM(K, ID, C=...), run.py:15) through the drop-in SVM.py on the
    normalised SP k=6 Gram of Xtr0 rows 0..399: predictions equal the oracle's."""
    from SVM import C_SVM
    K, labels, _, _ = LC.load()
    ID = np.arange(LC.N_ALL)
    svm = C_SVM(K, ID, C=C, print_callbacks=False)
    svm.fit(pd.DataFrame({"Id": ID[:LC.N_FIT]}),
            pd.DataFrame({"Id": ID[:LC.N_FIT], "Bound": labels[:LC.N_FIT]}))
    pred = svm.predict(pd.DataFrame({"Id": ID[LC.N_FIT:]}))
    idx_fit = np.arange(LC.N_FIT)
    ra, _, robj = cpu_ref.svm_dual(K[:LC.N_FIT, :LC.N_FIT], labels[:LC.N_FIT].astype(float), C)
    _, _, rb, rpred = LC.bookkeeping(K, ra, idx_fit, labels[:LC.N_FIT], 1e-5,
                                     np.arange(LC.N_FIT, LC.N_ALL))
    assert svm.objective == pytest.approx(robj, rel=1e-9)
    assert svm.b == pytest.approx(rb, rel=1e-4, abs=1e-6)
    assert np.array_equal(pred, rpred)
    assert 0.0 <= svm.score(pred, labels[LC.N_FIT:]) <= 1.0


def test_svm_bad_arguments(ctx):
    K = np.eye(3)
    with pytest.raises(Exception):
        ctx.svm_fit(K, np.array([1.0, -1.0, 1.0]), 0.0)
    with pytest.raises(Exception):
        ctx.svm_fit(K, np.array([1.0, 0.0, 1.0]), 1.0)


def test_krr_klr_asymmetric_K_match_inv(ctx):
    """A K that is not exactly symmetric (the reference inverts whatever it is given,
    KRR.py:33 / KLR.py:55): the device solves the full system (LU), not one triangle."""
    rng = np.random.default_rng(13)
    n = 300
    A = rng.standard_normal((n, 40))
    K = A @ A.T / 40 + 0.5 * np.eye(n)
    K[3, 7] += 1e-3  # asymmetric by one entry
    K[200, 11] -= 2e-3
    y = np.where(rng.random(n) > 0.5, 1.0, -1.0)
    lb = 0.05
    ref = np.linalg.inv(K + lb * n * np.eye(n)) @ y
    got = ctx.krr_solve(K, y, lb)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12)
    sym = ctx.krr_solve((K + K.T) / 2, y, lb)
    assert not np.allclose(sym, got, rtol=1e-9, atol=0)  # the triangle read would differ


def test_engine_gram_takes_cholesky(ctx):
    """Every Gram kmg_gram returns is bitwise symmetric, so KRR / KLR on it factorise by
    Cholesky (rocSOLVER dpotrf), never by the per-column LU of an asymmetric K."""
    from kmgram import _lib as L, encode as E, params as P
    codes, lens = E.synthetic(700, 101, seed=17)
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), codes, lens,
                 L.KMG_F64)
    assert np.array_equal(K, K.T)
    y = np.where(np.random.default_rng(3).random(700) > 0.5, 1.0, -1.0)
    got = ctx.krr_solve(K, y, 0.01)
    assert ctx.last_factorisation() == "cholesky"
    np.testing.assert_allclose(got, cpu_ref.krr_alpha(K, y, 0.01), rtol=1e-9, atol=1e-12)
    ctx.klr_fit(K, y, 0.01, 1e-5, 3)
    assert ctx.last_factorisation() == "cholesky"


def test_factorisation_branches_reported(ctx):
    """The three branches of the solve (Cholesky, LU of an asymmetric K, LU after a failed
    Cholesky) are what kmg_last_factorisation reports."""
    rng = np.random.default_rng(21)
    n = 120
    A = rng.standard_normal((n, 30))
    K = A @ A.T / 30 + 0.5 * np.eye(n)
    y = rng.standard_normal(n)
    ctx.krr_solve(K, y, 0.1)
    assert ctx.last_factorisation() == "cholesky"
    Ka = K.copy()
    Ka[5, 9] += 1e-12
    ctx.krr_solve(Ka, y, 0.1)
    assert ctx.last_factorisation() == "lu_asymmetric"
    B = rng.standard_normal((n, n))
    ctx.krr_solve((B + B.T) / 2, y, 0.0)
    assert ctx.last_factorisation() == "lu_indefinite"


@pytest.mark.parametrize("chol", ["1", "0"])
@pytest.mark.parametrize("n", [127, 128, 129, 256, 385])
def test_krr_block_edges_both_factorisations(ctx, tune, chol, n):
    """The blocked Cholesky (KMG_CHOL=1: LDS diagonal blocks of 128, inverse-block GEMM
    panels, one-launch-a-block substitution sweeps) and rocSOLVER potrf/potrs (KMG_CHOL=0)
    at sizes on and around the 128-column block edges."""
    tune(KMG_CHOL=chol)
    K = _psd(n, max(1, n // 3), 7 * n)
    y = np.where(np.random.default_rng(n + 3).random(n) > 0.5, 1.0, -1.0)
    got = ctx.krr_solve(K, y, 0.02)
    assert ctx.last_factorisation() == "cholesky"
    np.testing.assert_allclose(got, cpu_ref.krr_alpha(K, y, 0.02), rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("chol", ["1", "0"])
def test_indefinite_pivot_in_later_block_falls_back(ctx, tune, chol):
    """A pivot that fails in the third diagonal block (column ~300) of the blocked path:
    every later block returns at once, the system is rebuilt and LU agrees with inv()."""
    tune(KMG_CHOL=chol)
    n = 400
    K = _psd(n, n, 5)
    K[300, 300] = -5.0  # symmetric, not positive definite
    y = np.random.default_rng(6).standard_normal(n)
    got = ctx.krr_solve(K, y, 0.0)
    assert ctx.last_factorisation() == "lu_indefinite"
    np.testing.assert_allclose(got, cpu_ref.krr_alpha(K, y, 0.0), rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("chol", ["1", "0"])
def test_svm_both_factorisations(ctx, tune, chol):
    tune(KMG_CHOL=chol)
    n, C = 700, 1.0
    K = _psd(n, n // 4, 99)
    y = np.where(np.random.default_rng(98).random(n) > 0.5, 1.0, -1.0)
    a, steps, obj = ctx.svm_fit(K, y, C)
    ra, rsteps, robj = cpu_ref.svm_dual(K, y, C)
    assert obj == pytest.approx(robj, rel=1e-9, abs=1e-12)
    np.testing.assert_allclose(a, ra, atol=1e-5 * C, rtol=0)


@pytest.mark.parametrize("panels", ["0", "3", "4"])
@pytest.mark.parametrize("n", [1500, 2101])
def test_krr_trailing_update_panels(ctx, tune, panels, n):
    """The blocked Cholesky's trailing update as KMG_CHOL_PANELS GEMM column panels (taken
    once the trailing triangle is >= 1024 rows: the n = 9000 production path) against one
    dsyrk (0): ragged last panels (n = 2101: 1845 rows in 3 or 4 panels) and the panel
    offsets, against numpy's inv (KRR.py:33)."""
    tune(KMG_CHOL="1", KMG_CHOL_PANELS=panels)
    K = _psd(n, n // 3, 11 * n)
    y = np.where(np.random.default_rng(n + 9).random(n) > 0.5, 1.0, -1.0)
    got = ctx.krr_solve(K, y, 0.02)
    assert ctx.last_factorisation() == "cholesky"
    np.testing.assert_allclose(got, cpu_ref.krr_alpha(K, y, 0.02), rtol=1e-9, atol=1e-12)


def test_svm_panel_path_n1700(ctx, tune):
    """One C-SVM fit (SVM.py:78-89) at a size whose factorisations take the GEMM-panel
    trailing update (KMG_CHOL=1, default panels)."""
    tune(KMG_CHOL="1", KMG_CHOL_PANELS=None)
    n, C = 1700, 1.0
    K = _psd(n, n // 4, 1701)
    y = np.where(np.random.default_rng(1702).random(n) > 0.5, 1.0, -1.0)
    a, steps, obj = ctx.svm_fit(K, y, C)
    ra, rsteps, robj = cpu_ref.svm_dual(K, y, C)
    assert steps < 100
    assert obj == pytest.approx(robj, rel=1e-9, abs=1e-12)
    np.testing.assert_allclose(a, ra, atol=1e-5 * C, rtol=0)


def test_device_lds_allows_in_tree_cholesky():
    """The in-tree factorisation needs ~133 KB of LDS a workgroup (chol_inv_kernel); the
    library uses it only where the device reports that much (use_own_chol, else rocSOLVER).
    On the MI355X it must be taken: the largest of the runtime's LDS attributes >= 133 KB."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    vals = []
    # hipDeviceAttributeMaxSharedMemoryPerBlock, ...SharedMemPerBlockOptin,
    # ...MaxSharedMemoryPerMultiprocessor (ROCm 7.2 hip_runtime_api.h enum values)
    for attr in (74, 75, 10002):
        v = ctypes.c_int(0)
        if hip.hipDeviceGetAttribute(ctypes.byref(v), attr, 0) == 0:
            vals.append(v.value)
    assert max(vals) >= 8 * (128 * 129 + 128), vals
