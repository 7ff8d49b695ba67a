"""Oracle restatements of KRR.fit / KLR.fit (oracle/cpu_ref.py) against the golden vectors
made by the unmodified reference KRR.py / KLR.py (tests/golden/make_learner_golden.py)."""
import numpy as np
import pytest

import cpu_ref
import learner_cases as LC


@pytest.fixture(scope="module")
def case_data():
    return LC.load()


@pytest.mark.parametrize("case", range(4))
def test_oracle_learner_matches_reference(case_data, case):
    K, labels, meta, arr = case_data
    m = meta[f"case{case}"]
    kw = dict(m["kwargs"])
    idx_fit = np.arange(LC.N_FIT)
    K_fit = K[np.ix_(idx_fit, idx_fit)]
    y_fit = labels[:LC.N_FIT]
    if m["learner"] == "KRR":
        alpha = cpu_ref.krr_alpha(K_fit, y_fit, kw["lbda"])
        rtol = 0.0  # same numpy expression as KRR.py:33
    else:
        alpha, _ = cpu_ref.klr_alpha(K_fit, y_fit, kw["lbda"], kw.get("tol", 1e-5),
                                     kw.get("maxiter", 50))
        rtol = 1e-9  # diagonal scalings applied elementwise instead of by np.dot
    a, idx_sv, b, pred = LC.bookkeeping(K, alpha, idx_fit, y_fit, 1e-5,
                                        np.arange(LC.N_FIT, LC.N_ALL))
    tag = f"case{case}"
    assert np.array_equal(idx_sv, arr[f"{tag}_idx_sv"])
    np.testing.assert_allclose(a, arr[f"{tag}_a"], rtol=rtol, atol=1e-12)
    assert b == pytest.approx(m["b"], rel=1e-9, abs=1e-12)
    assert np.array_equal(pred, arr[f"{tag}_pred"])


def test_positions_lookup():
    from kmgram.learners import _positions
    ID = np.array([10, 3, 7, 42])
    assert _positions(ID, [42, 10, 7]).tolist() == [3, 0, 2]
    with pytest.raises(ValueError):
        _positions(ID, [5])


@pytest.mark.parametrize("C", [0.1, 1.0, 10.0])
def test_svm_oracle_optimum_vs_lbfgsb(C):
    """The oracle's interior-point optimum of C_SVM's QP (SVM.py:78-89; cvxopt absent, parity
    to cvxopt's own numbers unpinned) against the reference's other solver for the same QP,
    L-BFGS-B on loss/jac with the same bounds (SVM.py:29-40, 66-76), run to tight tolerance
    from zero (the reference starts from randn)."""
    from scipy.optimize import fmin_l_bfgs_b
    K, labels, _, _ = LC.load()
    n = 120
    K_fit, y = K[:n, :n], labels[:n].astype(np.float64)
    a, steps, obj = cpu_ref.svm_dual(K_fit, y, C)
    assert steps < 40
    loss = lambda v: -(2 * np.dot(v, y) - np.dot(v.T, np.dot(K_fit, v)))  # noqa: E731
    jac = lambda v: -(2 * y - 2 * np.dot(K_fit, v))  # noqa: E731
    bounds = [[-C if yi <= 0 else 0, C if yi >= 0 else 0] for yi in y]
    ref, fval, _ = fmin_l_bfgs_b(loss, np.zeros(n), fprime=jac, bounds=bounds, pgtol=1e-12,
                                 factr=10, maxiter=20000)
    assert obj == pytest.approx(fval / 2, rel=1e-9)
    assert obj <= fval / 2 + 1e-9 * abs(fval)
    np.testing.assert_allclose(a, ref, atol=1e-5 * C)
    # feasibility and KKT of the returned a (x = y o a in the box [0, C])
    x = y * a
    assert np.all(x >= 0) and np.all(x <= C)
    g = y * (K_fit @ a) - 1.0  # gradient in x
    assert np.abs(x - np.clip(x - g, 0, C)).max() < 1e-6 * max(1.0, C)  # projected-gradient KKT
