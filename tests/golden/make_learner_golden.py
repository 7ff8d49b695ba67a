"""Golden vectors for the dense learners on K, made by running the
UNMODIFIED reference ``KRR.py`` and ``KLR.py`` (afiliot/Kernel-Methods-For-Genomics, read-only
at /root/reference; both import only numpy) in the build container.

Test infrastructure, run by hand here only: ``python tests/golden/make_learner_golden.py``.
Input K: the normalised spectrum k=6 Gram of Xtr0 rows 0..399 (oracle/cref.spectrum, itself
pinned bit-exactly to the reference's get_spectrum_K, then normalize_K), labels Ytr0 with
0 -> -1 as utils.py:29 does.  Fit on rows 0..299, predict rows 300..399.
Output: learners.npz (alpha before the support-vector filter is not kept by the reference,
so the fixture holds the fitted a, idx_sv, b and the predictions) + learners_meta.json.
"""
import json
import os
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
N_FIT, N_ALL, K_SP = 300, 400, 6
CASES = [("KRR", {"lbda": 0.1}), ("KRR", {"lbda": 1e-3}), ("KLR", {"lbda": 0.1}),
         ("KLR", {"lbda": 1e-2, "tol": 1e-7, "maxiter": 30})]


def inputs():
    """(K, labels) shared by this script and the tests."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cref
    import cpu_ref
    import golden_io
    codes, lens = golden_io.load_xtr0()
    K = cpu_ref.normalize(cref.spectrum(codes[:N_ALL], lens[:N_ALL], K_SP).astype(np.float64))
    z = np.load(os.path.join(HERE, "learners.npz"), allow_pickle=False) if os.path.exists(
        os.path.join(HERE, "learners.npz")) else None
    labels = z["labels"] if z is not None else None
    return K, labels


def main():
    import pandas as pd
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import KRR as ref_krr  # the reference modules
    import KLR as ref_klr
    K, _ = inputs()
    y = pd.read_csv(os.path.join(REF, "Data", "Ytr0.csv"))
    y["Bound"] = y["Bound"].replace(0, -1)
    labels = np.asarray(y["Bound"][:N_ALL], dtype=np.int64)
    ID = np.arange(N_ALL)
    X_fit = pd.DataFrame({"Id": ID[:N_FIT]})
    y_fit = pd.DataFrame({"Id": ID[:N_FIT], "Bound": labels[:N_FIT]})
    X_te = pd.DataFrame({"Id": ID[N_FIT:]})
    arrays, meta = {"labels": labels}, {}
    for c, (name, kw) in enumerate(CASES):
        cls = ref_krr.KRR if name == "KRR" else ref_klr.KLR
        model = cls(K, ID, **kw)
        model.fit(X_fit, y_fit)
        pred = model.predict(X_te)
        tag = f"case{c}"
        arrays[f"{tag}_a"] = np.asarray(model.a, dtype=np.float64)
        arrays[f"{tag}_idx_sv"] = np.asarray(model.idx_sv, dtype=np.int64)
        arrays[f"{tag}_pred"] = np.asarray(pred, dtype=np.float64)
        meta[tag] = {"learner": name, "kwargs": kw, "b": float(model.b),
                     "score": float(model.score(pred, labels[N_FIT:])),
                     "source": "KRR.py:21-56" if name == "KRR" else "KLR.py:57-98"}
    meta["inputs"] = {"K": f"normalize_K(SP k={K_SP}) of Xtr0 rows 0..{N_ALL - 1}",
                      "fit_rows": [0, N_FIT], "predict_rows": [N_FIT, N_ALL],
                      "labels": "Ytr0 Bound, 0 -> -1 (utils.py:29)"}
    np.savez_compressed(os.path.join(HERE, "learners.npz"), **arrays)
    json.dump(meta, open(os.path.join(HERE, "learners_meta.json"), "w"), indent=1)
    print(json.dumps(meta, indent=1))


if __name__ == "__main__":
    main()
