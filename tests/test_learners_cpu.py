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
