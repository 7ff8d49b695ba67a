"""GPU parity of the dense learners on K (kmg_krr_solve / kmg_klr_fit: rocSOLVER Cholesky,
LU fallback, HIP IRLS kernels in csrc/kmg_solve.hip) through the drop-in KRR.py / KLR.py.

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
