"""Full-size accuracy of the learners' solve (GPU box): KRR at n = 9000 on a normalised
PSD K through the blocked Cholesky (KMG_CHOL=1) and rocSOLVER (KMG_CHOL=0), both against
numpy's LU solve of the same system; relative error and scaled residual per path.
usage: python3 tools/check_solver_n9000.py [n] [lambda ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kernel-methods-for-genomics_amd")]
from kmgram import _lib as L  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 9000
    rng = np.random.default_rng(9000)
    A = rng.standard_normal((n, n // 3))
    K = A @ A.T + 1e-3 * np.eye(n)
    d = np.sqrt(np.diag(K))
    K = K / d[:, None] / d[None, :]
    K = (K + K.T) / 2
    y = np.where(rng.random(n) > 0.5, 1.0, -1.0)
    for lbda in [float(a) for a in sys.argv[2:]] or [1e-3]:
        check(K, y, n, lbda)


def cond_spd(M):
    w = np.linalg.eigvalsh(M)
    return float(w[-1] / w[0])


def check(K, y, n, lbda):
    M = K + lbda * n * np.eye(n)
    ref = np.linalg.solve(M, y)
    out = {"n": n, "lambda": lbda, "cond_2": cond_spd(M)}
    for chol in ("1", "0"):
        os.environ["KMG_CHOL"] = chol
        ctx = L.Context(0)
        try:
            got = ctx.krr_solve(K, y, lbda)
            fac = ctx.last_factorisation()
        finally:
            ctx.close()
        out["chol" + chol] = {
            "factorisation": fac,
            "rel_err_vs_numpy": float(np.linalg.norm(got - ref) / np.linalg.norm(ref)),
            "max_rel_elem": float(np.max(np.abs(got - ref)) / np.max(np.abs(ref))),
            "scaled_residual": float(np.linalg.norm(M @ got - y) / (np.linalg.norm(M, 1) * np.linalg.norm(got))),
        }
    out["numpy_scaled_residual"] = float(np.linalg.norm(M @ ref - y) / (np.linalg.norm(M, 1) * np.linalg.norm(ref)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
