"""Shared inputs of the dense-learner tests (fixtures from tests/golden/make_learner_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
N_FIT, N_ALL, K_SP = 300, 400, 6


def load():
    """(K, labels, meta, arrays): K = normalised SP k=6 Gram of Xtr0 rows 0..399 by the
    pinned oracle, labels Ytr0 (-1/1) of those rows."""
    import cref
    import cpu_ref
    import golden_io
    codes, lens = golden_io.load_xtr0()
    K = cpu_ref.normalize(cref.spectrum(codes[:N_ALL], lens[:N_ALL], K_SP).astype(np.float64))
    z = np.load(os.path.join(GOLDEN, "learners.npz"), allow_pickle=False)
    arrays = {k: z[k] for k in z.files}
    meta = json.load(open(os.path.join(GOLDEN, "learners_meta.json")))
    return K, arrays["labels"], meta, arrays


def bookkeeping(K, alpha, idx_fit, y_fit, eps, idx_pred):
    """Support vectors, intercept and predictions around a solved alpha (KRR.py:35-56)."""
    sv = np.where(np.abs(alpha) > eps)
    a, ys, idx_sv = alpha[sv], y_fit[sv], idx_fit[sv]
    b = np.mean(ys - a @ K[np.ix_(idx_sv, idx_sv)])
    pred = np.sign(a @ K[np.ix_(idx_sv, idx_pred)] + b)
    return a, idx_sv, b, pred
