"""Ingest / cache formats (kmgram/store.py): the ``Id,seq`` CSV reader
(reference utils.py:20-45 reads the same files with pandas) and the slab-streamed ``.npy``
K cache that replaces the ``training_data_<method>.pkl`` pickle (utils.py:139-155) at
large N.  CPU tests cover parsing and the method grammar; the GPU tests check that the
streamed file equals the in-memory Gram bit for bit."""
import numpy as np
import pytest

from kmgram import _lib as L
from kmgram import encode as E
from kmgram import store


def _write_csv(path, ids, seqs):
    with open(path, "w") as f:
        f.write("Id,seq\n")
        for i, s in zip(ids, seqs):
            f.write(f"{i},{s}\n")


def test_read_csv_codes_matches_encode(tmp_path):
    codes, lens = E.synthetic(50, 101, seed=4)
    seqs = E.decode(codes, lens)
    seqs[3] = seqs[3][:60]  # ragged
    ids = np.arange(1000, 1050)
    p = tmp_path / "Xtr9.csv"
    _write_csv(p, ids, seqs)
    rid, rc, rl = store.read_csv_codes(p)
    ec, el = E.encode(seqs)
    assert np.array_equal(rid, ids)
    assert np.array_equal(rc, ec) and np.array_equal(rl, el)


def test_read_csv_codes_columns_and_errors(tmp_path):
    p = tmp_path / "x.csv"
    p.write_text("seq,Id\nACGT,7\nTTTT,8\n\n")
    rid, rc, rl = store.read_csv_codes(p)
    assert list(rid) == [7, 8] and list(rl) == [4, 4] and list(rc[1, :4]) == [3, 3, 3, 3]
    p.write_text("Id,sequence\n1,ACGT\n")
    with pytest.raises(ValueError):
        store.read_csv_codes(p)
    p.write_text("Id,seq\n1,AC,GT\n")
    with pytest.raises(ValueError):
        store.read_csv_codes(p)


def test_method_params_grammar():
    p, mm = store.method_params("SP_k8")
    assert (p.kind, p.k, mm) == (L.KMG_SPECTRUM, 8, False)
    p, mm = store.method_params("MM_k9_m1")
    assert (p.kind, p.k, p.m, p.window, p.normalize, mm) == (L.KMG_MISMATCH, 9, 1, 101, 1, True)
    with pytest.raises(NotImplementedError):
        store.method_params("WD_d5")


@pytest.mark.gpu
@pytest.mark.parametrize("method,dt,slab", [("SP_k8", L.KMG_I32, 37), ("SP_k6", L.KMG_F64, 300),
                                            ("MM_k9_m1", L.KMG_F64, 41), ("MM_k5_m1", L.KMG_F64, 64)])
def test_gram_to_npy_equals_gram(ctx, tmp_path, method, dt, slab):
    codes, lens = E.synthetic(300, 101, seed=21)
    path = tmp_path / f"K_{method}.npy"
    K = store.gram_to_npy(path, codes, lens, method, out_dtype=dt, slab_rows=slab, ctx=ctx)
    params, _ = store.method_params(method)
    ref = ctx.gram(params, codes, lens, dt)
    assert K.dtype == ref.dtype and not K.flags.writeable
    assert np.array_equal(np.asarray(K), ref)
    assert np.array_equal(np.asarray(store.load_gram(path)), ref)


@pytest.mark.gpu
def test_gram_to_npy_mismatch_validation(ctx, tmp_path):
    codes, lens = E.synthetic(20, 101, seed=2)
    codes[3, 7] = 9
    with pytest.raises(ValueError):
        store.gram_to_npy(tmp_path / "a.npy", codes, lens, "MM_k9_m1", ctx=ctx)


@pytest.mark.gpu
def test_gram_to_host_strided_output(ctx):
    """kmg_gram_to_host into a host array whose rows are longer than n (ld_host > n): the
    n x n block equals the one-call Gram, the columns past n stay untouched."""
    from kmgram import params as P
    codes, lens = E.synthetic(230, 101, seed=23)
    n, ldc = codes.shape
    params = P.make(L.KMG_SPECTRUM, k=8)
    ref = ctx.gram(params, codes, lens, L.KMG_I32)
    buf = np.full((n, n + 5), -7, dtype=np.int32)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_to_host(params, d_codes, d_lens, n, ldc, L.KMG_I32, 50, buf[:, :n])
    finally:
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    assert np.array_equal(buf[:, :n], ref)
    assert np.all(buf[:, n:] == -7)
