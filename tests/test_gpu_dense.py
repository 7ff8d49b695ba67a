"""GPU parity of the dense count-vector formulation (kmg_dense.hip: int8 F, K = F F^T on
the int8 matrix cores) against the C oracle, for spectrum and mismatch at every small k
and m, at tile-edge sizes, on row slabs, and against the posting-list path.  Integer
results are exact (tolerance 0); the float64 normalised mismatch is bit-exact."""
import ctypes

import numpy as np
import pytest

import cref
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[0, 1], ids=["wg8", "half"])
def dense(tune, request):
    """The dense path, with each tile on one 8-wave workgroup or split over two 4-wave ones
    (KMG_DENSE_HALF; auto: half when the feature width is <= 1024)."""
    tune(KMG_ALGO=1, KMG_DENSE_HALF=request.param)


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 6, 7, 8])
def test_dense_spectrum_k(ctx, dense, k):
    codes, lens = E.synthetic(333, 101, seed=100 + k)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=k), codes, lens, L.KMG_I32)
    assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, k))


@pytest.mark.parametrize("n", [1, 2, 127, 128, 129, 255, 257, 640])
def test_dense_tile_edges(ctx, dense, n):
    codes, lens = E.synthetic(n, 101, seed=7 * n)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=5), codes, lens, L.KMG_I32)
    assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, 5))
    Km = ctx.gram(P.make(L.KMG_MISMATCH, k=5, m=1, window=101, normalize=1), codes, lens,
                  L.KMG_F64)
    assert np.array_equal(Km, cref.mismatch_rows(codes, lens, 5, 1))


def test_dense_spectrum_ragged_and_non_acgt(ctx, dense):
    """Per-sequence window count len-k+1, windows holding a non-ACGT symbol dropped
    (kernels.py:21-24), lengths 0..126+k (<= 127 windows)."""
    rng = np.random.default_rng(41)
    for k in (3, 7):
        seqs = ["".join(rng.choice(list("ACGTN"), p=[.24, .24, .24, .24, .04],
                                   size=rng.integers(0, 127 + k))) for _ in range(500)]
        codes, lens = E.encode(seqs)
        K = ctx.gram(P.make(L.KMG_SPECTRUM, k=k), codes, lens, L.KMG_I32)
        assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, k)), k


def test_dense_spectrum_max_counts(ctx, dense):
    """127 windows of poly-A: the int8 feature ceiling, K = 127^2."""
    codes, lens = E.synthetic(40, 130, seed=4)
    codes[3] = 0
    codes[7] = 0
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=4), codes, lens, L.KMG_I32)
    assert K[3, 3] == 127 * 127 and K[3, 7] == 127 * 127
    assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, 4))


def test_dense_refuses_over_127_windows(ctx, dense):
    codes, lens = E.synthetic(8, 140, seed=4)
    with pytest.raises(L.KmgUnsupported):
        ctx.gram(P.make(L.KMG_SPECTRUM, k=4), codes, lens, L.KMG_I32)


@pytest.mark.parametrize("k,m", [(1, 1), (2, 1), (3, 1), (4, 1), (5, 1), (6, 1), (7, 1), (8, 1),
                                 (4, 0), (5, 2), (6, 2), (4, 3), (3, 3), (2, 5), (6, 3)])
def test_dense_mismatch(ctx, dense, k, m):
    codes, lens = E.synthetic(260, 101, seed=10 * k + m)
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=0), codes, lens,
                   L.KMG_I32)
    assert np.array_equal(raw.astype(np.int64), cref.mismatch_raw(codes, lens, k, m))
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=1), codes, lens,
                 L.KMG_F64)
    assert np.array_equal(K, cref.mismatch_rows(codes, lens, k, m))
    K32 = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=1), codes, lens,
                   L.KMG_F32)
    assert np.array_equal(K32, K.astype(np.float32))


def test_dense_mismatch_repeats(ctx, dense):
    """Homopolymer / dinucleotide rows: the largest neighbour counts (93 per column)."""
    codes, lens = E.synthetic(50, 101, seed=12)
    codes[3] = 0
    codes[4] = np.tile([0, 1], 51)[:101]
    codes[5] = 3
    for k in (5, 6):
        raw = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0), codes, lens,
                       L.KMG_I32)
        assert np.array_equal(raw.astype(np.int64), cref.mismatch_raw(codes, lens, k, 1)), k


def test_dense_equals_index_path(ctx, tune):
    """The two formulations of the same Gram agree bit for bit."""
    codes, lens = E.synthetic(700, 101, seed=77)
    out = {}
    for algo in ("1", "2"):
        tune(KMG_ALGO=algo)
        out[algo] = (ctx.gram(P.make(L.KMG_SPECTRUM, k=6), codes, lens, L.KMG_I32),
                     ctx.gram(P.make(L.KMG_MISMATCH, k=7, m=1, window=101, normalize=1), codes,
                              lens, L.KMG_F64))
    assert np.array_equal(out["1"][0], out["2"][0])
    assert np.array_equal(out["1"][1], out["2"][1])


def test_dense_row_slabs(ctx, dense):
    """kmg_gram_device on row slabs with unaligned boundaries == full matrix."""
    codes, lens = E.synthetic(900, 101, seed=21)
    n, ldc = codes.shape
    cases = ((P.make(L.KMG_SPECTRUM, k=6), L.KMG_I32),
             (P.make(L.KMG_MISMATCH, k=5, m=1, window=101, normalize=1), L.KMG_F64))
    d_codes = ctx.dmalloc(codes.nbytes)
    d_lens = ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    try:
        for params, dt in cases:
            ref = ctx.gram(params, codes, lens, dt)
            esz = np.dtype(L.DTYPES[dt]).itemsize
            out = np.zeros((n, n), dtype=L.DTYPES[dt])
            d_out = ctx.dmalloc(n * n * esz)
            splits = [0, 1, 129, 300, 301, 899, 900]
            for a, b in zip(splits[:-1], splits[1:]):
                ctx.gram_device(params, d_codes, d_lens, n, ldc, a, b, dt,
                                ctypes.c_void_p(d_out.value + a * n * esz), n)
            ctx.synchronize()
            ctx.d2h(out, d_out)
            ctx.dfree(d_out)
            assert np.array_equal(out, ref)
    finally:
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)


def test_auto_picks_dense_for_run_py_kernels(ctx, tune):
    """run.py's SP_k4/5 and MM_k4..6_m1 at the production shape (N=9000 train+val+test,
    utils.py:149-153) go through the dense path; checked on oracle rows."""
    tune(KMG_ALGO=None)
    codes, lens = E.synthetic(9000, 101, seed=9000)
    ctx.set_timing(True)
    try:
        for params, dt, ref in (
                (P.make(L.KMG_SPECTRUM, k=5), L.KMG_I32,
                 lambda r: cref.spectrum(codes, lens, 5, rows=(r, r + 1))[0]),
                (P.make(L.KMG_MISMATCH, k=5, m=1, window=101, normalize=1), L.KMG_F64,
                 lambda r: cref.mismatch_rows(codes, lens, 5, 1, rows=(r, r + 1))[0])):
            K = ctx.gram(params, codes, lens, dt)
            assert ctx.stage_ms("features") >= 0.0  # the dense feature stage ran
            for r in (0, 4500, 8999):
                assert np.array_equal(K[r].astype(ref(r).dtype), ref(r)), r
            assert np.array_equal(K, K.T)
    finally:
        ctx.set_timing(False)


@pytest.mark.parametrize("k", [4, 6, 8])
def test_fp32_gemm_spectrum(ctx, tune, k):
    """KMG_ALGO=3: BASELINE configs[3]'s literal "count-vector fp32 GEMM" (rocblas_sgemm on
    the widened count rows) gives the exact integer K (every partial sum < 2^24)."""
    tune(KMG_ALGO=3)
    codes, lens = E.synthetic(300, 101, seed=500 + k)
    codes[7] = codes[3]  # a duplicate row: the largest off-diagonal counts
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=k), codes, lens, L.KMG_I32)
    assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, k))
    Kd = ctx.gram(P.make(L.KMG_SPECTRUM, k=k), codes, lens, L.KMG_F64)
    assert np.array_equal(Kd, K.astype(np.float64))


def test_fp32_gemm_mismatch_normalised(ctx, tune):
    tune(KMG_ALGO=3)
    codes, lens = E.synthetic(200, 101, seed=505)
    Kn = ctx.gram(P.make(L.KMG_MISMATCH, k=5, m=1, window=101, normalize=1), codes, lens, L.KMG_F64)
    assert np.array_equal(Kn, cref.mismatch_rows(codes, lens, 5, 1))
