"""Kernel parameters: the reference's coefficient formulas and the mismatch weights.

Everything here is scalar host arithmetic evaluated exactly as the reference's Python
does it, so that the float64 coefficients handed to the device are the same bits.
"""
from math import comb

from . import _lib as L


def beta(d, k):
    """WD degree weight, kernels.py:53-61: 2 * (d - k + 1) / d / (d + 1)."""
    return 2 * (d - k + 1) / d / (d + 1)


def delta(s):
    """WDS shift weight, kernels.py:106-112: 1/2/(s+1)."""
    return 1 / 2 / (s + 1)


def mismatch_weights(k, m):
    """w_m(h) = #{b : ham(u,b) <= m and ham(v,b) <= m} for two k-mers u, v at Hamming
    distance h.  Then <Phi_x, Phi_y> = sum_{a,b} w_m(ham(x_a, y_b)) where Phi is the
    mismatch feature map of get_phi_km (kernels.py:161-175).  For m=1: (1+3k, 4, 2, 0...).
    """
    w = []
    for h in range(k + 1):
        tot = 0
        for i in range(k - h + 1):  # letters changed where u and v agree
            for a in range(h + 1):  # differing positions where b takes u's letter
                for b in range(h - a + 1):  # ... where b takes v's letter
                    c = h - a - b  # ... where b takes a third letter (2 choices)
                    if i + b + c <= m and i + a + c <= m:
                        tot += comb(k - h, i) * 3 ** i * comb(h, a) * comb(h - a, b) * 2 ** c
        w.append(tot)
    return w


def make(kind, **kw):
    """Fill a KmgParams struct."""
    p = L.KmgParams()
    p.kind = kind
    for name in ("k", "m", "d", "S", "g", "window", "normalize", "smith", "la_mode", "span"):
        if name in kw:
            setattr(p, name, int(kw[name]))
    if "lbda" in kw:
        lbda = kw["lbda"]
        p.lambda_ = float(lbda)
        p.lambda2 = float(lbda ** 2)  # lbda**2 exactly as the reference evaluates it (kernels.py:340)
    for name in ("la_e", "la_d", "la_beta"):
        if name in kw:
            setattr(p, name, float(kw[name]))
    if kind in (L.KMG_WD, L.KMG_WDS):
        d = int(kw["d"])
        if d > L.KMG_MAX_COEF:
            raise L.KmgUnsupported(L.KMG_EUNSUPPORTED, f"d={d} > {L.KMG_MAX_COEF}")
        for k in range(1, d + 1):
            p.coef_a[k - 1] = beta(d, k)
    if kind == L.KMG_WDS:
        S = int(kw["S"])
        if S + 1 > L.KMG_MAX_COEF:
            raise L.KmgUnsupported(L.KMG_EUNSUPPORTED, f"S={S} too large")
        for s in range(S + 1):
            p.coef_b[s] = delta(s)
    p.diag_value = float("nan")
    return p
