"""GPU parity of kmg_gram_device_cols: column blocks K[:, col0:col1] of the mismatch (k, 1)
Gram (kernels.py:196-217) with the neighbourhood lists built over the block's sequences.
Checked bit-exact against the oracle (raw and normalised), and against the row slab of
the same sequences transposed (K is symmetric) at N=20000."""
import ctypes

import numpy as np
import pytest

import cref
import invariants as I
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P

pytestmark = pytest.mark.gpu


def _col_block(ctx, params, codes, lens, col0, col1, dt):
    n = codes.shape[0]
    w = col1 - col0
    npdt = L.DTYPES[dt]
    wa = max(1, w)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(n * wa * np.dtype(npdt).itemsize)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device_cols(params, d_codes, d_lens, n, codes.shape[1], col0, col1, dt, d_out, w)
        ctx.synchronize()
        out = np.empty((n, w), dtype=npdt)
        ctx.d2h(out, d_out)
        return out
    finally:
        for p in (d_out, d_codes, d_lens):
            ctx.dfree(p)


@pytest.mark.parametrize("k", [8, 9, 10])
@pytest.mark.parametrize("fill", ["0", "1", "4"])
@pytest.mark.parametrize("threads", ["0", "1024"])
def test_column_blocks_vs_oracle(ctx, tune, k, fill, threads):
    """Blocks at the start, inside, at the end and of one column; 30 poly-A rows make lists
    past the fills' LDS buffers (lane-per-run fallbacks).  Gram workgroups of 512 threads
    (the column blocks' default) and of 1024."""
    codes, lens = E.synthetic(700, 101, seed=200 + k)
    codes[:30] = 0
    tune(KMG_NB_FILL=fill, KMG_NB_THREADS=None if threads == "0" else threads)
    raw_p = P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0)
    if fill == "1" and k == 10:  # segment 2 too sparse to pack: the forced sorted fill refuses
        with pytest.raises(L.KmgUnsupported, match="sorted fill"):
            _col_block(ctx, raw_p, codes, lens, 0, 700, L.KMG_I32)
        return
    ref = cref.mismatch_raw(codes, lens, k, 1)
    for col0, col1 in ((0, 700), (0, 123), (250, 611), (699, 700)):
        K = _col_block(ctx, raw_p, codes, lens, col0, col1, L.KMG_I32)
        assert ctx.last_plan()["formulation"] == "neighbourhood"
        assert ctx.last_plan()["threads"] == (512 if threads == "0" else 1024)
        assert np.array_equal(K.astype(np.int64), ref[:, col0:col1]), (col0, col1)
    Kn = _col_block(ctx, P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=1), codes, lens,
                    250, 611, L.KMG_F64)
    refn = cref.mismatch_rows(codes, lens, k, 1)
    assert np.array_equal(Kn, refn[:, 250:611])


def test_column_block_is_row_slab_transposed_n20000(ctx):
    """N=20000, columns [5000, 12000): the block equals rows [5000, 12000) of the row-slab
    path transposed, bit for bit (float64 normalised); oracle rows at both block edges."""
    n, c0, c1 = 20000, 5000, 12000
    codes, lens = E.synthetic(n, 101, seed=3)
    params = P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1)
    Kc = _col_block(ctx, params, codes, lens, c0, c1, L.KMG_F64)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_K = ctx.dmalloc((c1 - c0) * n * 8)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(params, d_codes, d_lens, n, codes.shape[1], c0, c1, L.KMG_F64, d_K, n)
        ctx.synchronize()
        Kr = np.empty((c1 - c0, n), dtype=np.float64)
        ctx.d2h(Kr, d_K)
    finally:
        for p in (d_K, d_codes, d_lens):
            ctx.dfree(p)
    assert np.array_equal(Kc, Kr.T)
    for r in (c0, c1 - 1):
        assert np.array_equal(Kr[r - c0], cref.mismatch_rows(codes, lens, 9, 1, rows=(r, r + 1))[0])


def test_column_block_argument_checks(ctx):
    codes, lens = E.synthetic(64, 101, seed=5)
    with pytest.raises(L.KmgUnsupported):  # k > 16: the generic per-pair kernels
        _col_block(ctx, P.make(L.KMG_SPECTRUM, k=20), codes, lens, 0, 32, L.KMG_I32)
    with pytest.raises(L.KmgUnsupported):  # whole-row kernels (a block's ld cannot hold a row)
        _col_block(ctx, P.make(L.KMG_WD, d=5), codes, lens, 0, 32, L.KMG_F64)
    with pytest.raises(L.KmgUnsupported):
        _col_block(ctx, P.make(L.KMG_MISMATCH, k=20, m=1, window=101), codes, lens, 0, 32, L.KMG_I32)
    with pytest.raises(L.KmgUnsupported):
        _col_block(ctx, P.make(L.KMG_MISMATCH, k=9, m=2, window=101), codes, lens, 0, 32, L.KMG_I32)
    with pytest.raises(L.KmgError):
        _col_block(ctx, P.make(L.KMG_MISMATCH, k=9, m=1, window=101), codes, lens, 40, 30, L.KMG_I32)


def _row_sums_parallel(blk, pool):
    parts = np.array_split(np.arange(blk.shape[0]), 8)
    return np.concatenate(list(pool.map(lambda r: blk[r].sum(axis=1, dtype=np.int64), parts)))


@pytest.mark.parametrize("c0", [0, 100000])
def test_config5_column_block_n200000_full(ctx, c0):
    """The block bench.py times for config 5's G=8 share (BENCH `configs.config5_*colblock*`):
    N=200000, columns [c0, c0 + 25000), raw int32, the packed two-chunk plan asserted.  Every
    row's sum over the block's columns exact (invariants.mismatch1_row_sums with the block's
    column histogram), oracle rows on both sides of the block's chunk edge and at its ends,
    and the block's own square part symmetric across the chunk edge (kernels.py:196-217)."""
    from concurrent.futures import ThreadPoolExecutor
    n, k, w, piece = 200000, 9, 25000, 8000
    c1 = c0 + w
    codes, lens = E.synthetic(n, 101, seed=5)
    params = P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(n * w * 4)
    pool = ThreadPoolExecutor(8)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device_cols(params, d_codes, d_lens, n, codes.shape[1], c0, c1, L.KMG_I32, d_out, w)
        ctx.synchronize()
        plan = ctx.last_plan()
        assert plan["formulation"] == "neighbourhood" and plan["packed"], plan
        assert plan["nchunks"] == 2 and not plan["triangle"] and plan["threads"] == 512, plan
        ch = plan["chunk"]
        sums = I.mismatch1_row_sums(codes, k, cols=(c0, c1))
        buf = np.empty((piece, w), dtype=np.int32)
        for a in range(0, n, piece):
            ctx.d2h(buf, ctypes.c_void_p(d_out.value + a * w * 4))
            assert np.array_equal(_row_sums_parallel(buf, pool), sums[a:a + piece]), a
        rows = sorted({0, n - 1, max(0, c0 - 1), c0, c0 + ch - 1, c0 + ch, c1 - 1, min(n - 1, c1)})
        refs = list(pool.map(lambda r: cref.mismatch_raw(codes, lens, k, 1, rows=(r, r + 1))[0], rows))
        row = np.empty(w, dtype=np.int32)
        for r, ref in zip(rows, refs):
            ctx.d2h(row, ctypes.c_void_p(d_out.value + r * w * 4))
            assert np.array_equal(row.astype(np.int64), ref[c0:c1]), r
        # K[c0 + a, c0 + b] for a 256-square straddling the chunk edge: symmetric
        e = ch - 128
        sq = np.empty((256, w), dtype=np.int32)
        ctx.d2h(sq, ctypes.c_void_p(d_out.value + (c0 + e) * w * 4))
        S = sq[:, e:e + 256]
        assert np.array_equal(S, S.T)
    finally:
        pool.shutdown()
        for p in (d_out, d_codes, d_lens):
            ctx.dfree(p)


def test_column_block_packed_float64_n20000(ctx, tune):
    """The packed lists (KMG_NB_FILL=1) on a float64 normalised column block at N=20000:
    the raw int32 block, every row sum exact over the block's columns, then the normalised
    block entry for entry = raw / (sqrt(K_ii) * sqrt(K_jj)) with the diagonal 1.0 --
    normalize_K's expression (kernels.py:408-414) -- from the oracle's diagonal."""
    n, k, c0, c1 = 20000, 9, 6000, 13500
    w = c1 - c0
    tune(KMG_NB_FILL="1")
    codes, lens = E.synthetic(n, 101, seed=3)
    raw = _col_block(ctx, P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0), codes, lens,
                     c0, c1, L.KMG_I32)
    assert ctx.last_plan()["packed"]
    assert np.array_equal(raw.sum(axis=1, dtype=np.int64), I.mismatch1_row_sums(codes, k, cols=(c0, c1)))
    Kn = _col_block(ctx, P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=1), codes, lens,
                    c0, c1, L.KMG_F64)
    assert ctx.last_plan()["packed"]
    d = np.sqrt(cref.mismatch_diag(codes, lens, k, 1).astype(np.float64))
    ref = raw.astype(np.float64) / (d[:, None] * d[None, c0:c1])
    ref[np.arange(c0, c1), np.arange(w)] = 1.0
    assert np.array_equal(Kn, ref)


# (KMG_SP_CB_CHUNK, KMG_SP_ROWS): blocks as one chunk (the default) or as 64-column chunks,
# one / two / four rows a workgroup (0: by chunk width)
SP_CB_TUNES = [("32768", "0"), ("64", "0"), ("64", "1"), ("32768", "2"), ("64", "4")]


@pytest.mark.parametrize("k", [6, 8, 12])
@pytest.mark.parametrize("cb_chunk,rows", SP_CB_TUNES)
def test_spectrum_column_blocks_vs_full(ctx, tune, k, cb_chunk, rows):
    """Spectrum column blocks (get_spectrum_K, kernels.py:28-47): the posting index over the
    block's sequences only, every row; int32 raw and float64 normalised blocks equal the
    columns of the single-call K bit for bit (ragged rows: lengths 60..101), whether a block
    is one column chunk or several and whatever the rows a workgroup (odd row counts leave
    a workgroup one row short)."""
    codes, lens = E.synthetic(901, 101, seed=300 + k)
    lens[::7] = 60 + (np.arange(len(lens[::7])) % 41)
    full = ctx.gram(P.make(L.KMG_SPECTRUM, k=k), codes, lens, L.KMG_I32)
    fulln = ctx.gram(P.make(L.KMG_SPECTRUM, k=k, normalize=1), codes, lens, L.KMG_F64)
    # (a block wider than KMG_SP_CB_CHUNK is chunked by KMG_SP_CHUNK)
    tune(KMG_SP_CB_CHUNK=cb_chunk, KMG_SP_CHUNK="64" if cb_chunk == "64" else "24576",
         KMG_SP_ROWS=rows)
    for col0, col1 in ((0, 901), (0, 113), (400, 777), (900, 901)):
        K = _col_block(ctx, P.make(L.KMG_SPECTRUM, k=k), codes, lens, col0, col1, L.KMG_I32)
        plan = ctx.last_plan()
        assert plan["formulation"] == "posting"
        if cb_chunk == "64" and col1 - col0 > 64:
            assert plan["nchunks"] > 1
        else:
            assert plan["nchunks"] == 1
        assert np.array_equal(K, full[:, col0:col1]), (col0, col1)
        Kn = _col_block(ctx, P.make(L.KMG_SPECTRUM, k=k, normalize=1), codes, lens, col0, col1,
                        L.KMG_F64)
        assert np.array_equal(Kn, fulln[:, col0:col1]), (col0, col1)


def test_spectrum_column_block_n100000(ctx):
    """The G = 8 share of the headline (BASELINE configs[3]) as a column block: K[:, 37500:
    50000] of all 100000 rows, every row sum exact over the block's columns (sum_u phi_i(u)
    T_block(u)) and oracle rows."""
    n, k, c0, c1 = 100000, 8, 37500, 50000
    codes, lens = E.synthetic(n, 101, seed=4)
    K = _col_block(ctx, P.make(L.KMG_SPECTRUM, k=k), codes, lens, c0, c1, L.KMG_I32)
    km = I.kmers(codes, k)
    T = np.bincount(km[c0:c1].ravel(), minlength=4 ** k)
    assert np.array_equal(K.sum(axis=1, dtype=np.int64), T[km].sum(axis=1))
    for r in (0, c0, c1 - 1, n - 1):
        assert np.array_equal(K[r].astype(np.int64), cref.spectrum(codes, lens, k, rows=(r, r + 1))[0, c0:c1]), r
