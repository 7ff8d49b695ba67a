"""ctypes wrapper of the C oracle (oracle/kmg_oracle.c).  TEST INFRASTRUCTURE ONLY —
importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libkmoracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        D = ctypes.c_double
        lib.kmo_spectrum.argtypes = [P, P, I64, I64, I, I64, I64, P]
        lib.kmo_mismatch_raw.argtypes = [P, P, I64, I64, I, I, P, I64, I64, P]
        lib.kmo_mismatch_diag.argtypes = [P, P, I64, I64, I, I, P, P]
        lib.kmo_wd.argtypes = [P, P, I64, I64, I, P, I64, I64, P]
        lib.kmo_wds.argtypes = [P, P, I64, I64, I, I, P, P, I64, I64, P]
        lib.kmo_ss.argtypes = [P, P, I64, I64, I, D, D, I64, I64, P]
        for f in ("kmo_spectrum", "kmo_mismatch_raw", "kmo_mismatch_diag", "kmo_wd", "kmo_wds",
                  "kmo_ss"):
            getattr(lib, f).restype = ctypes.c_int
        _lib = lib
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _prep(codes, lens):
    return (np.ascontiguousarray(codes, dtype=np.uint8),
            np.ascontiguousarray(lens, dtype=np.int32))


def _rows(n, rows):
    return (0, n) if rows is None else rows


def spectrum(codes, lens, k, rows=None):
    codes, lens = _prep(codes, lens)
    n, ldc = codes.shape
    r0, r1 = _rows(n, rows)
    out = np.zeros((r1 - r0, n), dtype=np.int64)
    rc = load().kmo_spectrum(_p(codes), _p(lens), n, ldc, k, r0, r1, _p(out))
    assert rc == 0, rc
    return out


def mismatch_raw(codes, lens, k, m, window=101, rows=None):
    from cpu_ref import mismatch_weights
    codes, lens = _prep(codes, lens)
    n, ldc = codes.shape
    r0, r1 = _rows(n, rows)
    w = np.zeros(33, dtype=np.int64)
    ww = mismatch_weights(k, m)
    w[: len(ww)] = ww
    out = np.zeros((r1 - r0, n), dtype=np.int64)
    rc = load().kmo_mismatch_raw(_p(codes), _p(lens), n, ldc, k, window, _p(w), r0, r1, _p(out))
    assert rc == 0, rc
    return out


def mismatch_diag(codes, lens, k, m, window=101):
    from cpu_ref import mismatch_weights
    codes, lens = _prep(codes, lens)
    n, ldc = codes.shape
    w = np.zeros(33, dtype=np.int64)
    ww = mismatch_weights(k, m)
    w[: len(ww)] = ww
    out = np.zeros(n, dtype=np.int64)
    rc = load().kmo_mismatch_diag(_p(codes), _p(lens), n, ldc, k, window, _p(w), _p(out))
    assert rc == 0, rc
    return out


def mismatch_rows(codes, lens, k, m, window=101, rows=None):
    """Normalised rows of get_mismatch_K (kernels.py:216, normalize_K 398-415)."""
    n = codes.shape[0]
    r0, r1 = _rows(n, rows)
    raw = mismatch_raw(codes, lens, k, m, window, (r0, r1)).astype(np.float64)
    diag = mismatch_diag(codes, lens, k, m, window).astype(np.float64)
    if diag[0] == 1:
        return raw
    d = np.sqrt(diag)
    out = raw / (d[r0:r1, None] * d[None, :])
    for t, i in enumerate(range(r0, r1)):
        out[t, i] = 1.0
    return out


def wd(codes, lens, d, rows=None):
    codes, lens = _prep(codes, lens)
    n, ldc = codes.shape
    r0, r1 = _rows(n, rows)
    beta = np.array([2 * (d - k + 1) / d / (d + 1) for k in range(1, d + 1)] + [0.0])
    out = np.zeros((r1 - r0, n))
    assert load().kmo_wd(_p(codes), _p(lens), n, ldc, d, _p(beta), r0, r1, _p(out)) == 0
    return out


def wds(codes, lens, d, S, rows=None):
    codes, lens = _prep(codes, lens)
    n, ldc = codes.shape
    r0, r1 = _rows(n, rows)
    beta = np.array([2 * (d - k + 1) / d / (d + 1) for k in range(1, d + 1)] + [0.0])
    delta = np.array([1 / 2 / (s + 1) for s in range(S + 1)])
    out = np.zeros((r1 - r0, n))
    assert load().kmo_wds(_p(codes), _p(lens), n, ldc, d, S, _p(beta), _p(delta), r0, r1,
                          _p(out)) == 0
    return out


def ss(codes, lens, lbda, k, rows=None):
    codes, lens = _prep(codes, lens)
    n, ldc = codes.shape
    r0, r1 = _rows(n, rows)
    out = np.zeros((r1 - r0, n))
    assert load().kmo_ss(_p(codes), _p(lens), n, ldc, k, float(lbda), float(lbda ** 2), r0, r1,
                         _p(out)) == 0
    return out
