"""ctypes binding of libkmgram.so (C ABI: include/kmgram.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
kernel-methods-for-genomics_amd/csrc``).  There is deliberately no fallback: if the
shared object is missing or no HIP device is visible, every compute call raises.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# KMGRAM_LIB: another build of the same ABI (the host-ASan build, tools/asan_tests.sh)
LIB_PATH = os.environ.get("KMGRAM_LIB") or os.path.join(os.path.dirname(_HERE), "libkmgram.so")

(KMG_OK, KMG_EINVAL, KMG_EUNSUPPORTED, KMG_EHIP, KMG_ENOMEM, KMG_ERCCL, KMG_ENODEV,
 KMG_ESINGULAR, KMG_EINTERNAL) = range(9)
KMG_SPECTRUM, KMG_MISMATCH, KMG_WD, KMG_WDS, KMG_SUBSTRING, KMG_LOCALALIGN, KMG_GAPPY = range(1, 8)
KMG_I32, KMG_F32, KMG_F64 = 1, 2, 3
KMG_LA_REFERENCE, KMG_LA_INTENDED = 0, 1
KMG_MODE_REFERENCE, KMG_MODE_INTENDED = 0, 1  # GP semantics (include/kmgram.h)
KMG_MODE_SS_B = 2  # SS: B_k of the recursion instead of K_k (include/kmgram.h)
KMG_MAX_COEF = 64

DTYPES = {KMG_I32: np.int32, KMG_F32: np.float32, KMG_F64: np.float64}

# every entry point declared in include/kmgram.h (checked by tests/test_abi.py)
EXPORTS = (
    "kmg_version", "kmg_last_error", "kmg_device_count", "kmg_create", "kmg_destroy",
    "kmg_gram", "kmg_gram_device", "kmg_normalize", "kmg_center", "kmg_dmalloc", "kmg_dfree",
    "kmg_h2d", "kmg_d2h", "kmg_memset", "kmg_synchronize", "kmg_stream", "kmg_set_timing",
    "kmg_timing_reset", "kmg_stage_ms", "kmg_stage_stats", "kmg_comm_unique_id", "kmg_comm_init", "kmg_allgather_rows",
    "kmg_comm_destroy", "kmg_combine", "kmg_combine_device", "kmg_nlck_grad",
    "kmg_nlck_grad_device", "kmg_alignf", "kmg_alignf_device", "kmg_krr_solve",
    "kmg_krr_solve_device", "kmg_klr_fit", "kmg_klr_fit_device", "kmg_svm_fit",
    "kmg_svm_fit_device", "kmg_rows_padded", "kmg_gram_blocks", "kmg_reload_tuning",
    "kmg_gram_to_host", "kmg_gram_blocks_wire", "kmg_last_plan", "kmg_features",
    "kmg_last_factorisation", "kmg_features_sym", "kmg_gram_device_cols",
)
KMG_FEATURES_BCAST = 1
KMG_FACTOR_CHOLESKY, KMG_FACTOR_LU_ASYMMETRIC, KMG_FACTOR_LU_INDEFINITE = 1, 2, 3


class KmgParams(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32), ("k", ctypes.c_int32), ("m", ctypes.c_int32),
        ("d", ctypes.c_int32), ("S", ctypes.c_int32), ("g", ctypes.c_int32),
        ("window", ctypes.c_int32), ("normalize", ctypes.c_int32), ("smith", ctypes.c_int32),
        ("la_mode", ctypes.c_int32), ("span", ctypes.c_int32), ("reserved", ctypes.c_int32 * 5),
        ("lambda_", ctypes.c_double), ("lambda2", ctypes.c_double),
        ("la_e", ctypes.c_double), ("la_d", ctypes.c_double), ("la_beta", ctypes.c_double),
        ("coef_a", ctypes.c_double * KMG_MAX_COEF), ("coef_b", ctypes.c_double * KMG_MAX_COEF),
        ("diag_value", ctypes.c_double),
    ]


class KmgError(RuntimeError):
    """A libkmgram call returned a non-zero status."""

    def __init__(self, status, msg):
        super().__init__(f"libkmgram error {status}: {msg}")
        self.status = status


class KmgUnsupported(KmgError):
    pass


_lib = None
_lock = threading.Lock()


def load():
    """Load libkmgram.so (raises if it has not been built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libkmgram.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        lib = ctypes.CDLL(LIB_PATH)
        P, I32, I64, SZ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
        D = ctypes.c_double
        sig = {
            "kmg_version": ([], ctypes.c_int),
            "kmg_last_error": ([], ctypes.c_char_p),
            "kmg_device_count": ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
            "kmg_create": ([ctypes.POINTER(P), ctypes.c_int], ctypes.c_int),
            "kmg_destroy": ([P], ctypes.c_int),
            "kmg_gram": ([P, ctypes.POINTER(KmgParams), P, P, I64, I64, I32, P, I64], ctypes.c_int),
            "kmg_gram_device": ([P, ctypes.POINTER(KmgParams), P, P, I64, I64, I64, I64, I32, P,
                                 I64], ctypes.c_int),
            "kmg_gram_device_cols": ([P, ctypes.POINTER(KmgParams), P, P, I64, I64, I64, I64, I32,
                                      P, I64], ctypes.c_int),
            "kmg_features": ([P, ctypes.POINTER(KmgParams), P, P, I64, I64, P, I64, P, I64],
                             ctypes.c_int),
            "kmg_features_sym": ([P, ctypes.POINTER(KmgParams), P, P, I64, I64, P, I64, I32, P,
                                  I64], ctypes.c_int),
            "kmg_normalize": ([P, P, I64, I64, ctypes.POINTER(I32)], ctypes.c_int),
            "kmg_center": ([P, P, I64, P, I64, I64], ctypes.c_int),
            "kmg_dmalloc": ([P, ctypes.POINTER(P), SZ], ctypes.c_int),
            "kmg_dfree": ([P, P], ctypes.c_int),
            "kmg_h2d": ([P, P, P, SZ], ctypes.c_int),
            "kmg_d2h": ([P, P, P, SZ], ctypes.c_int),
            "kmg_memset": ([P, P, ctypes.c_int, SZ], ctypes.c_int),
            "kmg_synchronize": ([P], ctypes.c_int),
            "kmg_stream": ([P, ctypes.POINTER(P)], ctypes.c_int),
            "kmg_set_timing": ([P, I32], ctypes.c_int),
            "kmg_timing_reset": ([P], ctypes.c_int),
            "kmg_stage_ms": ([P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
            "kmg_last_plan": ([P, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
            "kmg_last_factorisation": ([P, ctypes.POINTER(ctypes.c_int32)], ctypes.c_int),
            "kmg_stage_stats": ([P, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(I32)], ctypes.c_int),
            "kmg_comm_unique_id": ([P], ctypes.c_int),
            "kmg_comm_init": ([P, P, I32, I32], ctypes.c_int),
            "kmg_allgather_rows": ([P, P, I64, I64, I32, P], ctypes.c_int),
            "kmg_comm_destroy": ([P], ctypes.c_int),
            "kmg_rows_padded": ([I64, I32, I64], I64),
            "kmg_gram_blocks": ([P, ctypes.POINTER(KmgParams), P, P, I64, I64, I32, P, I64, I32,
                                 I32, I64, I32], ctypes.c_int),
            "kmg_reload_tuning": ([P], ctypes.c_int),
            "kmg_gram_blocks_wire": ([P], ctypes.c_int),
            "kmg_gram_to_host": ([P, ctypes.POINTER(KmgParams), P, P, I64, I64, I32, I64, P,
                                  I64], ctypes.c_int),
            "kmg_combine": ([P, P, I32, P, I32, I64, I64, P, I64], ctypes.c_int),
            "kmg_combine_device": ([P, P, I32, P, I32, I64, I64, P, I64], ctypes.c_int),
            "kmg_nlck_grad": ([P, P, I32, P, I32, P, I64, I64, P], ctypes.c_int),
            "kmg_nlck_grad_device": ([P, P, I32, P, I32, P, I64, I64, P], ctypes.c_int),
            "kmg_alignf": ([P, P, I32, P, I64, I64, P, P], ctypes.c_int),
            "kmg_alignf_device": ([P, P, I32, P, I64, I64, P], ctypes.c_int),
            "kmg_krr_solve": ([P, P, I64, I64, P, D, P], ctypes.c_int),
            "kmg_krr_solve_device": ([P, P, I64, I64, P, D, P], ctypes.c_int),
            "kmg_klr_fit": ([P, P, I64, I64, P, D, D, I32, P, ctypes.POINTER(I32)],
                            ctypes.c_int),
            "kmg_klr_fit_device": ([P, P, I64, I64, P, D, D, I32, P, ctypes.POINTER(I32)],
                                   ctypes.c_int),
            "kmg_svm_fit": ([P, P, I64, I64, P, D, D, I32, P, ctypes.POINTER(I32),
                             ctypes.POINTER(D)], ctypes.c_int),
            "kmg_svm_fit_device": ([P, P, I64, I64, P, D, D, I32, P, ctypes.POINTER(I32),
                                    ctypes.POINTER(D)], ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = res
        _lib = lib
        return lib


def check(status):
    if status != KMG_OK:
        msg = load().kmg_last_error().decode(errors="replace")
        if status == KMG_EUNSUPPORTED:
            raise KmgUnsupported(status, msg)
        if status == KMG_ESINGULAR:
            raise np.linalg.LinAlgError(msg)
        raise KmgError(status, msg)


def device_count():
    n = ctypes.c_int(0)
    check(load().kmg_device_count(ctypes.byref(n)))
    return n.value


def ptr(a):
    """Raw pointer of a numpy array (None for empty)."""
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Context:
    """One libkmgram context (one HIP device, one stream, a device workspace)."""

    def __init__(self, device=0):
        self.lib = load()
        self._h = ctypes.c_void_p()
        check(self.lib.kmg_create(ctypes.byref(self._h), int(device)))
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            self.lib.kmg_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- compute
    def gram(self, params, codes, lens, out_dtype=KMG_F64, out=None):
        n, ldc = codes.shape
        if out is None:
            out = np.empty((n, n), dtype=DTYPES[out_dtype])
        assert out.flags.c_contiguous and out.shape == (n, n)
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        check(self.lib.kmg_gram(self._h, ctypes.byref(params), ptr(codes), ptr(lens), n, ldc,
                                out_dtype, ptr(out), n))
        return out

    def features(self, params, codes, lens, cols):
        """float64 [n, len(cols)] feature rows (kmg_features): column j scores the k-mer code
        cols[j] (0xFFFFFFFF: a beta no window can equal)."""
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        cols = np.ascontiguousarray(cols, dtype=np.uint32)
        n, ldc = codes.shape
        out = np.empty((n, len(cols)), dtype=np.float64)
        check(self.lib.kmg_features(self._h, ctypes.byref(params), ptr(codes), ptr(lens), n, ldc,
                                    ptr(cols), len(cols), ptr(out), len(cols)))
        return out

    def features_sym(self, params, codes, lens, cols, flags=0):
        """float64 [n, len(cols)] feature rows over symbol columns (kmg_features_sym): cols is
        uint8 [ncols, 16], column j the k symbol codes cols[j, :k] in the rows' code space."""
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        lens = np.ascontiguousarray(lens, dtype=np.int32)
        cols = np.ascontiguousarray(cols, dtype=np.uint8).reshape(-1, 16)
        n, ldc = codes.shape
        out = np.empty((n, len(cols)), dtype=np.float64)
        check(self.lib.kmg_features_sym(self._h, ctypes.byref(params), ptr(codes), ptr(lens), n,
                                        ldc, ptr(cols), len(cols), int(flags), ptr(out), len(cols)))
        return out

    def gram_device(self, params, d_codes, d_lens, n, ldc, row0, row1, out_dtype, d_out, ld):
        check(self.lib.kmg_gram_device(self._h, ctypes.byref(params), d_codes, d_lens, n, ldc,
                                       row0, row1, out_dtype, d_out, ld))

    def gram_device_cols(self, params, d_codes, d_lens, n, ldc, col0, col1, out_dtype, d_out, ld):
        """Column block K[:, col0:col1] (every row) at d_out, row stride ld (kmg_gram_device_cols)."""
        check(self.lib.kmg_gram_device_cols(self._h, ctypes.byref(params), d_codes, d_lens, n, ldc,
                                            col0, col1, out_dtype, d_out, ld))

    def gram_blocks(self, params, d_codes, d_lens, n, ldc, out_dtype, d_out, ld, nranks, rank,
                    block, gather):
        """Block-cyclic rows of this rank.  gather: False / 0 this rank's blocks only; True / 1
        full rows all-gathered in place over RCCL per round; 2 upper-triangle round slabs
        all-gathered + local mirror; 3 the upper-triangle layout with every rank's blocks
        computed locally (one-GPU rehearsal, no RCCL); 4 this rank's blocks packed (row
        t * block + y of d_out = K row t * nranks * block + rank * block + y); 5 column blocks:
        this rank's K[:, rank * block : (rank + 1) * block] (lists over its own sequences),
        transposed into those rows of d_out, all-gathered in place over RCCL (one round:
        nranks * block >= n rows); 6 the same with every rank's block on this GPU (no RCCL)."""
        g = int(gather) if not isinstance(gather, bool) else (1 if gather else 0)
        check(self.lib.kmg_gram_blocks(self._h, ctypes.byref(params), d_codes, d_lens, n, ldc,
                                       out_dtype, d_out, ld, int(nranks), int(rank), int(block),
                                       g))

    def gram_to_host(self, params, d_codes, d_lens, n, ldc, out_dtype, slab_rows, out):
        """K of all n rows into the host array ``out`` (n x n, C-contiguous rows; a numpy
        memmap works), built in device slabs of ``slab_rows`` rows with one index build and
        each slab's copy overlapping the next slab's Gram.  Synchronous."""
        if out.shape[0] < n or out.shape[1] < n or out.dtype != np.dtype(DTYPES[out_dtype]):
            raise ValueError("gram_to_host: output shape / dtype")
        if out.strides[1] != out.itemsize:
            raise ValueError("gram_to_host: output rows must be contiguous")
        check(self.lib.kmg_gram_to_host(self._h, ctypes.byref(params), d_codes, d_lens, n, ldc,
                                        out_dtype, int(slab_rows), out.ctypes.data,
                                        out.strides[0] // out.itemsize))

    def blocks_wire(self):
        """Bytes per element of the last gram_blocks call's all-gathered slabs."""
        return int(self.lib.kmg_gram_blocks_wire(self._h))

    def reload_tuning(self):
        """Re-read the KMG_* environment knobs (read once at context creation)."""
        check(self.lib.kmg_reload_tuning(self._h))

    def normalize(self, K):
        skipped = ctypes.c_int32(0)
        check(self.lib.kmg_normalize(self._h, ptr(K), K.shape[0], K.strides[0] // 8,
                                     ctypes.byref(skipped)))
        return bool(skipped.value)

    def center(self, K):
        n = K.shape[0]
        out = np.empty((n, n), dtype=np.float64)
        check(self.lib.kmg_center(self._h, ptr(K), K.strides[0] // 8, ptr(out), n, n))
        return out

    # ---------------------------------------------------------------- combination consumers
    @staticmethod
    def _mats(kernels):
        mats = [np.ascontiguousarray(K, dtype=np.float64) for K in kernels]
        n = mats[0].shape[0]
        for K in mats:
            if K.shape != (n, n):
                raise ValueError("every kernel must be a square matrix of the same size")
        arr = (ctypes.c_void_p * len(mats))(*[K.ctypes.data for K in mats])
        return mats, arr, n

    def combine(self, kernels, u, degree, out=None):
        """(sum_m u[m] K_m) ** degree on the device (kmg_combine)."""
        mats, arr, n = self._mats(kernels)
        u = np.ascontiguousarray(u, dtype=np.float64)
        if out is None:
            out = np.empty((n, n), dtype=np.float64)
        check(self.lib.kmg_combine(self._h, arr, len(mats), ptr(u), int(degree), n, n, ptr(out), n))
        return out

    def nlck_grad(self, kernels, u, degree, alpha):
        mats, arr, n = self._mats(kernels)
        u = np.ascontiguousarray(u, dtype=np.float64)
        alpha = np.ascontiguousarray(alpha, dtype=np.float64)
        grad = np.empty(len(mats), dtype=np.float64)
        check(self.lib.kmg_nlck_grad(self._h, arr, len(mats), ptr(u), int(degree), ptr(alpha), n,
                                     n, ptr(grad)))
        return grad

    def alignf(self, kernels, y):
        mats, arr, n = self._mats(kernels)
        y = np.ascontiguousarray(y, dtype=np.float64)
        p = len(mats)
        a = np.empty(p, dtype=np.float64)
        M = np.empty((p, p), dtype=np.float64)
        check(self.lib.kmg_alignf(self._h, arr, p, ptr(y), n, n, ptr(a), ptr(M)))
        return a, M

    # ---------------------------------------------------------------- dense learners
    @staticmethod
    def _system(K, y):
        K = np.asarray(K, dtype=np.float64)
        if K.ndim != 2 or K.shape[0] != K.shape[1]:
            raise ValueError("K must be a square matrix")
        if K.strides[1] != 8 or K.strides[0] % 8:
            K = np.ascontiguousarray(K)
        y = np.ascontiguousarray(y, dtype=np.float64).reshape(-1)
        if y.shape[0] != K.shape[0]:
            raise ValueError(f"y has {y.shape[0]} entries for a {K.shape[0]} x {K.shape[0]} K")
        return K, y

    def krr_solve(self, K, y, lbda):
        """alpha = inv(K + lbda * n * I) . y (KRR.py:33), factorised on the device."""
        K, y = self._system(K, y)
        n = K.shape[0]
        alpha = np.empty(n, dtype=np.float64)
        check(self.lib.kmg_krr_solve(self._h, ptr(K), K.strides[0] // 8, n, ptr(y), float(lbda),
                                     ptr(alpha)))
        return alpha

    def klr_fit(self, K, y, lbda, tol, maxiter):
        """IRLS of KLR.fit (KLR.py:57-75); returns (alpha, iterations)."""
        K, y = self._system(K, y)
        n = K.shape[0]
        alpha = np.empty(n, dtype=np.float64)
        it = ctypes.c_int32(0)
        check(self.lib.kmg_klr_fit(self._h, ptr(K), K.strides[0] // 8, n, ptr(y), float(lbda),
                                   float(tol), int(maxiter), ptr(alpha), ctypes.byref(it)))
        return alpha, it.value

    def svm_fit(self, K, y, C, tol=1e-10, maxiter=100):
        """C_SVM.fit's QP (SVM.py:78-89) on the device; returns (alpha, steps, objective)."""
        K, y = self._system(K, y)
        n = K.shape[0]
        alpha = np.empty(n, dtype=np.float64)
        it, obj = ctypes.c_int32(0), ctypes.c_double(0.0)
        check(self.lib.kmg_svm_fit(self._h, ptr(K), K.strides[0] // 8, n, ptr(y), float(C),
                                   float(tol), int(maxiter), ptr(alpha), ctypes.byref(it),
                                   ctypes.byref(obj)))
        return alpha, it.value, obj.value

    # ---------------------------------------------------------------- device memory
    def dmalloc(self, nbytes):
        p = ctypes.c_void_p()
        check(self.lib.kmg_dmalloc(self._h, ctypes.byref(p), int(nbytes)))
        return p

    def dfree(self, p):
        check(self.lib.kmg_dfree(self._h, p))

    def h2d(self, dst, arr):
        arr = np.ascontiguousarray(arr)
        check(self.lib.kmg_h2d(self._h, dst, ptr(arr), arr.nbytes))

    def d2h(self, arr, src):
        check(self.lib.kmg_d2h(self._h, ptr(arr), src, arr.nbytes))
        return arr

    def memset(self, dst, value, nbytes):
        check(self.lib.kmg_memset(self._h, dst, int(value), int(nbytes)))

    def synchronize(self):
        check(self.lib.kmg_synchronize(self._h))

    def set_timing(self, on=True):
        """on: True / 1 every stage, 2 the Gram / gather / memset stages only, False off."""
        check(self.lib.kmg_set_timing(self._h, 2 if on == 2 else (1 if on else 0)))

    def timing_reset(self):
        check(self.lib.kmg_timing_reset(self._h))

    def stage_stats(self, stage):
        """(total_ms, count) of a stage over every timed call since timing_reset()."""
        t, n = ctypes.c_double(0.0), ctypes.c_int32(0)
        check(self.lib.kmg_stage_stats(self._h, stage.encode(), ctypes.byref(t), ctypes.byref(n)))
        return t.value, n.value

    def stream_handle(self):
        s = ctypes.c_void_p()
        check(self.lib.kmg_stream(self._h, ctypes.byref(s)))
        return s.value

    def last_plan(self):
        """How the last spectrum / mismatch call was built (include/kmgram.h kmg_last_plan)."""
        v = (ctypes.c_int32 * 6)()
        check(self.lib.kmg_last_plan(self._h, v))
        # (5, "pair_lines": round 3's pair-lines table, removed in round 5)
        names = ("dense", "hamming", "posting", "slots", "pairs", "pair_lines", "neighbourhood",
                 "generic")
        return {"formulation": names[v[0]] if 0 <= v[0] < len(names) else None,
                "chunk": v[1], "nchunks": v[2], "triangle": bool(v[3]), "threads": v[4],
                "packed": bool(v[5])}

    def last_factorisation(self):
        """The last KRR / KLR solve's factorisation: "cholesky", "lu_asymmetric",
        "lu_indefinite" or None (include/kmgram.h kmg_last_factorisation)."""
        v = ctypes.c_int32(0)
        check(self.lib.kmg_last_factorisation(self._h, ctypes.byref(v)))
        return {1: "cholesky", 2: "lu_asymmetric", 3: "lu_indefinite"}.get(v.value)

    def stage_ms(self, stage):
        v = ctypes.c_double(0.0)
        check(self.lib.kmg_stage_ms(self._h, stage.encode(), ctypes.byref(v)))
        return v.value

    # ---------------------------------------------------------------- RCCL
    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * 128)()
        check(load().kmg_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid, nranks, rank):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        check(self.lib.kmg_comm_init(self._h, buf, int(nranks), int(rank)))

    def allgather_rows(self, d_K, n, ld, dtype, splits):
        sp = np.ascontiguousarray(np.asarray(splits, dtype=np.int64))
        check(self.lib.kmg_allgather_rows(self._h, d_K, n, ld, dtype, ptr(sp)))

    def comm_destroy(self):
        check(self.lib.kmg_comm_destroy(self._h))
