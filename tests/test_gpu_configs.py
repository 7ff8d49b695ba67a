"""GPU parity at the BASELINE config sizes that do not fit an oracle run: configs[3]
(spectrum k=8, N=100000, full K on one GPU) and configs[4] (mismatch (9,1), N=200000, the
row slabs of two of its eight ranks).  Every Gram entry is checked in aggregate through
exact integer row sums (tests/invariants.py), plus oracle rows at slab edges, exact
diagonals and symmetric blocks.  Reference: kernels.py:28-47 (spectrum) and 196-217
(mismatch), normalize_K 398-415."""
import ctypes

import numpy as np
import pytest

import cref
import invariants as I
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P

pytestmark = pytest.mark.gpu


def _spectrum_diag(codes, k):
    """K_ii = sum_u phi_i(u)^2 for every row (unique (row, k-mer) pairs, counts squared)."""
    km = I.kmers(codes, k)
    n = km.shape[0]
    keyed = km + (np.arange(n, dtype=np.int64)[:, None] << (2 * k))
    u, cnt = np.unique(keyed.ravel(), return_counts=True)
    return np.bincount(u >> (2 * k), weights=cnt.astype(np.float64) ** 2, minlength=n).astype(np.int64)


def _fetch_rows(ctx, d_base, r0, r1, n, dtype, out=None):
    esz = np.dtype(dtype).itemsize
    if out is None:
        out = np.empty((r1 - r0, n), dtype=dtype)
    ctx.d2h(out, ctypes.c_void_p(d_base.value + r0 * n * esz))
    return out


def test_config4_spectrum_k8_n100000(ctx):
    """BASELINE configs[3]: the full 100000 x 100000 int32 K (40 GB) in one device build;
    every row's sum and diagonal exact, oracle rows at slab edges, symmetric blocks."""
    n, k, slab = 100000, 8, 5000
    codes, lens = E.synthetic(n, 101, seed=4)
    sums = I.spectrum_row_sums(codes, k)
    diag = _spectrum_diag(codes, k)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_K = ctx.dmalloc(n * n * 4)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(P.make(L.KMG_SPECTRUM, k=k), d_codes, d_lens, n, codes.shape[1], 0, n,
                        L.KMG_I32, d_K, n)
        ctx.synchronize()
        buf = np.empty((slab, n), dtype=np.int32)
        for a in range(0, n, slab):
            blk = _fetch_rows(ctx, d_K, a, a + slab, n, np.int32, buf)
            assert np.array_equal(blk.sum(axis=1, dtype=np.int64), sums[a:a + slab]), a
            assert np.array_equal(blk[np.arange(slab), a + np.arange(slab)].astype(np.int64),
                                  diag[a:a + slab]), a
        for r in (0, slab - 1, slab, 54321, n - 1):
            row = _fetch_rows(ctx, d_K, r, r + 1, n, np.int32)[0]
            assert np.array_equal(row.astype(np.int64), cref.spectrum(codes, lens, k, rows=(r, r + 1))[0]), r
        for a, b in ((0, 97000), (31000, 64000), (99744, 512)):
            A = _fetch_rows(ctx, d_K, a, a + 256, n, np.int32)
            B = _fetch_rows(ctx, d_K, b, b + 256, n, np.int32)
            assert np.array_equal(A[:, b:b + 256], B[:, a:a + 256].T), (a, b)
    finally:
        for p in (d_K, d_codes, d_lens):
            ctx.dfree(p)


@pytest.mark.parametrize("form", ["0", "1"])
@pytest.mark.parametrize("r0", [0, 100000])
def test_config5_mismatch_k9_n200000_rank_slab(ctx, tune, r0, form):
    """BASELINE configs[4] per-GPU share: rows [r0, r0 + 25000) of the N=200000 mismatch
    (9,1) Gram (ranks 0 and 4 of 8).  Raw int32 counts: every row sum exact (<Phi_i, C>),
    oracle rows at the slab edges, a symmetric block inside the slab; then the normalised
    float64 rows at the slab edges bit-exact against the oracle."""
    tune(KMG_MM_FORM=form)
    n, k, rows, piece = 200000, 9, 25000, 2500
    codes, lens = E.synthetic(n, 101, seed=5)
    sums = I.mismatch1_row_sums(codes, k, rows=(r0, r0 + rows))
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_K = ctx.dmalloc(rows * n * 4)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0), d_codes,
                        d_lens, n, codes.shape[1], r0, r0 + rows, L.KMG_I32, d_K, n)
        ctx.synchronize()
        buf = np.empty((piece, n), dtype=np.int32)
        for a in range(0, rows, piece):
            blk = _fetch_rows(ctx, d_K, a, a + piece, n, np.int32, buf)
            assert np.array_equal(blk.sum(axis=1, dtype=np.int64), sums[a:a + piece]), r0 + a
        for r in (r0, r0 + rows - 1):
            row = _fetch_rows(ctx, d_K, r - r0, r - r0 + 1, n, np.int32)[0]
            ref = cref.mismatch_raw(codes, lens, k, 1, rows=(r, r + 1))[0]
            assert np.array_equal(row.astype(np.int64), ref), r
        A = _fetch_rows(ctx, d_K, 1000, 1256, n, np.int32)
        B = _fetch_rows(ctx, d_K, 20000, 20256, n, np.int32)
        assert np.array_equal(A[:, r0 + 20000:r0 + 20256], B[:, r0 + 1000:r0 + 1256].T)
        # normalised float64 rows (the config's output) at both slab edges
        d_F = ctx.dmalloc(4 * n * 8)
        try:
            for a in (r0, r0 + rows - 4):
                ctx.gram_device(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=1),
                                d_codes, d_lens, n, codes.shape[1], a, a + 4, L.KMG_F64, d_F, n)
                got = _fetch_rows(ctx, d_F, 0, 4, n, np.float64)
                assert np.array_equal(got, cref.mismatch_rows(codes, lens, k, 1, rows=(a, a + 4))), a
        finally:
            ctx.dfree(d_F)
    finally:
        for p in (d_K, d_codes, d_lens):
            ctx.dfree(p)


def _row_sums_parallel(blk, pool):
    """int64 row sums of an int32 block, split over a thread pool (numpy releases the GIL)."""
    parts = np.array_split(np.arange(blk.shape[0]), 8)
    return np.concatenate(list(pool.map(lambda r: blk[r].sum(axis=1, dtype=np.int64), parts)))


@pytest.mark.parametrize("form", ["0", "1"])
def test_config5_mismatch_k9_n200000_full_one_gpu(ctx, tune, form):
    """BASELINE configs[4] on ONE GPU, the G=1 point of its strong-scaling line: the full
    200000 x 200000 raw int32 K (160 GB) in one kmg_gram_device call -- the upper block
    triangle of column chunks plus the in-place mirror (mirror_chunks_kernel, 64-bit
    offsets past 2^32 entries).  Every row sum exact, the exact diagonal, oracle rows on both
    sides of every chunk edge, symmetric 256 x 256 blocks straddling chunk edges, and the
    plan the library reports (kernels.py:211-215: K[j, i] = K[i, j])."""
    from concurrent.futures import ThreadPoolExecutor
    tune(KMG_MM_FORM=form)
    n, k, piece = 200000, 9, 2000
    codes, lens = E.synthetic(n, 101, seed=5)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_K = ctx.dmalloc(n * n * 4)
    pool = ThreadPoolExecutor(8)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0), d_codes,
                        d_lens, n, codes.shape[1], 0, n, L.KMG_I32, d_K, n)
        ctx.synchronize()
        plan = ctx.last_plan()
        assert plan["formulation"] in ("slots", "neighbourhood") and plan["triangle"], plan
        assert plan["nchunks"] >= 2 and plan["chunk"] * plan["nchunks"] >= n, plan
        ch = plan["chunk"]
        edges = [c * ch for c in range(1, plan["nchunks"]) if c * ch < n]
        sums = I.mismatch1_row_sums(codes, k)
        diag = cref.mismatch_diag(codes, lens, k, 1)
        buf = np.empty((piece, n), dtype=np.int32)
        for a in range(0, n, piece):
            blk = _fetch_rows(ctx, d_K, a, a + piece, n, np.int32, buf)
            assert np.array_equal(_row_sums_parallel(blk, pool), sums[a:a + piece]), a
            assert np.array_equal(blk[np.arange(piece), a + np.arange(piece)].astype(np.int64),
                                  diag[a:a + piece]), a
        # oracle rows on both sides of every chunk edge (and the first / last row)
        pairs = [(e - 1, e + 1) for e in edges] + [(0, 1), (n - 1, n)]
        refs = list(pool.map(lambda ab: cref.mismatch_raw(codes, lens, k, 1, rows=ab), pairs))
        for (a, b), ref in zip(pairs, refs):
            got = _fetch_rows(ctx, d_K, a, b, n, np.int32)
            assert np.array_equal(got.astype(np.int64), ref), (a, b)
        # symmetric blocks straddling chunk edges (mirrored entries against computed ones)
        for e0, e1 in zip(edges, edges[1:] + [edges[0]]):
            a, b = e0 - 128, e1 - 128
            A = _fetch_rows(ctx, d_K, a, a + 256, n, np.int32)
            B = _fetch_rows(ctx, d_K, b, b + 256, n, np.int32)
            assert np.array_equal(A[:, b:b + 256], B[:, a:a + 256].T), (a, b)
    finally:
        pool.shutdown()
        for p in (d_K, d_codes, d_lens):
            ctx.dfree(p)


def test_mismatch_k9_n20000_row_sums(ctx):
    """BASELINE configs[2] at full size: the raw (9,1) Gram of all 20000 rows, every row
    sum exact, symmetric, exact self-kernels from the oracle's diagonal."""
    n, k = 20000, 9
    codes, lens = E.synthetic(n, 101, seed=3)
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0), codes, lens,
                   L.KMG_I32)
    assert np.array_equal(raw.sum(axis=1, dtype=np.int64), I.mismatch1_row_sums(codes, k))
    assert np.array_equal(raw, raw.T)
    assert np.array_equal(np.diag(raw).astype(np.int64), cref.mismatch_diag(codes, lens, k, 1))
