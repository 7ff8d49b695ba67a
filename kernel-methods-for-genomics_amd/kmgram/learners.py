"""Dense learners on a precomputed Gram matrix, solved on the device.

Mirrors of the reference's KRR (KRR.py:4-66), KLR (KLR.py:4-110) and C_SVM
(SVM.py:6-128): same constructor arguments, same ``fit(X, y)`` / ``predict(X)`` /
``score(pred, y)`` contract on pandas frames with ``Id`` and ``Bound`` columns, same fitted
attributes.  The n x n system that the reference inverts with ``np.linalg.inv`` (KRR.py:33,
KLR.py:53-54) is factorised on the MI355X by libkmgram (``kmg_krr_solve`` /
``kmg_klr_fit``: the in-tree blocked Cholesky, rocSOLVER LU as the fallback), and C_SVM's cvxopt QP
(SVM.py:78-89; cvxopt is not installed here) is solved by a device interior-point method
(``kmg_svm_fit``).  The O(n_sv^2) bookkeeping around the solve (support-vector selection,
intercept, decision values) stays on the host as vectorised numpy.  No CPU fallback for
the solve.
"""
import numpy as np

from .engine import default_engine


def _positions(ID, ids):
    """Row of K of every id: the reference's per-id ``np.where(ID == id)[0]`` (KRR.py:29),
    as one hash lookup.  Ids must be unique in ``ID``."""
    where = {v: r for r, v in enumerate(np.asarray(ID).tolist())}
    try:
        return np.array([where[v] for v in np.asarray(ids).tolist()], dtype=np.int64)
    except KeyError as e:
        raise ValueError(f"Id {e.args[0]!r} is not a row of the kernel") from None


def _labels(y):
    return np.asarray(y.loc[:, "Bound"] if hasattr(y, "loc") else y)


class _GramLearner:
    """Shared fit/predict bookkeeping (identical in KRR.py, KLR.py and SVM.py)."""

    def _solve(self, K_fit, y_fit):
        raise NotImplementedError

    def fit(self, X, y):
        self.Id_fit = np.array(X.loc[:, "Id"])
        self.idx_fit = _positions(self.ID, self.Id_fit)
        K = np.asarray(self.K)
        self.K_fit = K[np.ix_(self.idx_fit, self.idx_fit)]
        self.y_fit, self.X_fit = _labels(y), X
        self.n = self.K_fit.shape[0]
        self.a = self._solve(self.K_fit, self.y_fit)
        # support vectors: |alpha| > eps (KRR.py:35, KLR.py:77)
        sv = np.where(np.abs(self.a) > self.eps)
        self.y_fit = self.y_fit[sv]
        self.a = self.a[sv]
        self.idx_sv = self.idx_fit[sv]
        # intercept: mean residual of the support vectors (KRR.py:40-41)
        self.y_hat = self.a @ K[np.ix_(self.idx_sv, self.idx_sv)]
        self.b = np.mean(self.y_fit - self.y_hat)

    def decision_function(self, X):
        self.Id_pred = np.array(X.loc[:, "Id"])
        self.idx_pred = _positions(self.ID, self.Id_pred)
        K = np.asarray(self.K)
        return self.a @ K[np.ix_(self.idx_sv, self.idx_pred)] + self.b

    def predict(self, X):
        """sign(sum_sv a_s K[s, i] + b) for every row of X (KRR.py:43-56)."""
        return np.sign(self.decision_function(X))

    def score(self, pred, y):
        """Accuracy of -1/1 predictions (KRR.py:58-66)."""
        label = y if isinstance(y, np.ndarray) else np.array(y.loc[:, "Bound"])
        assert 0 not in np.unique(label), "Labels must be -1 or 1, not 0 or 1"
        return np.mean(pred == label)


class KRR(_GramLearner):
    """Kernel ridge regression (KRR.py:4-66): alpha = inv(K_fit + lbda * n * I) . y."""

    def __init__(self, K, ID, eps=1e-5, lbda=0.1, solver=None):
        self.K = K
        self.ID = ID
        self.eps = eps
        self.lbda = lbda
        self.solver = solver

    def _solve(self, K_fit, y_fit):
        return default_engine().ctx.krr_solve(K_fit, y_fit, self.lbda)


class KLR(_GramLearner):
    """Kernel logistic regression by IRLS (KLR.py:4-110); the whole IRLS loop runs in one
    device call and ``iterations`` records how many weighted-KRR steps it took."""

    def __init__(self, K, ID, eps=1e-5, lbda=0.1, tol=1e-5, maxiter=50, solver=None):
        self.K = K
        self.ID = ID
        self.eps = eps
        self.lbda = lbda
        self.tol = tol
        self.solver = solver
        self.maxiter = maxiter

    @staticmethod
    def sigmoid(x):
        return 1 / (1 + np.exp(-x))

    def _solve(self, K_fit, y_fit):
        alpha, self.iterations = default_engine().ctx.klr_fit(K_fit, y_fit, self.lbda, self.tol,
                                                               self.maxiter)
        return alpha


class C_SVM(_GramLearner):
    """C-SVM without intercept in the QP (SVM.py:6-128): a = argmin 1/2 a'Ka - y'a with
    0 <= y_i a_i <= C, then the shared support-vector / intercept bookkeeping.  Both of the
    reference's solvers ('CVX': cvxopt.solvers.qp, SVM.py:78-89; 'BFGS': L-BFGS-B from a
    random start, SVM.py:66-76) solve this same convex QP; here both run the device
    interior-point method to a duality gap of ``tol`` (``iterations``, ``objective`` kept)."""

    def __init__(self, K, ID, C=10, eps=1e-5, solver="CVX", print_callbacks=True, tol=1e-10,
                 maxiter=100):
        self.K = K
        self.ID = ID
        self.C = C
        self.eps = eps
        self.solver = solver
        self.print_callbacks = print_callbacks
        self.Nfeval = 1
        self.tol = tol
        self.maxiter = maxiter

    def loss(self, a):
        """a'Ka - 2 a'y, twice the QP objective (SVM.py:29-34; host evaluation)."""
        return -(2 * np.dot(a, self.y_fit) - np.dot(a.T, np.dot(self.K_fit, a)))

    def jac(self, a):
        return -(2 * self.y_fit - 2 * np.dot(self.K_fit, a))

    def _solve(self, K_fit, y_fit):
        if self.solver not in ("CVX", "BFGS"):
            # the reference leaves self.a unset and fails on its next line (SVM.py:91)
            raise AttributeError("'C_SVM' object has no attribute 'a'")
        y = np.asarray(y_fit, dtype=np.float64)
        bad = ~np.isin(y, (-1.0, 1.0))
        if bad.any():
            # the device QP takes labels in {-1, 1}; the reference hands any y to cvxopt /
            # L-BFGS-B (SVM.py:66-89) and so does not reject them
            raise ValueError(f"C_SVM: the Bound column must hold -1 / 1 labels after the "
                             f"fit() mapping (got {np.unique(y[bad])[:5].tolist()})")
        alpha, self.iterations, self.objective = default_engine().ctx.svm_fit(
            K_fit, y, self.C, self.tol, self.maxiter)
        return alpha
