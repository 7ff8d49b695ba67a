"""Ingest and cache formats around the Gram.

Reference data flow (afiliot/Kernel-Methods-For-Genomics):
  * ``utils.get_train`` / ``get_test`` read ``Data/Xtr<k>.csv`` / ``Xte<k>.csv`` (columns
    ``Id,seq``) with pandas (utils.py:20-45);
  * ``utils.get_training_datas`` computes ``K = km.select_method(X, method)`` on the
    concatenated sequences and caches ``[X_train, y_train, X_val, y_val, X_test, K, ID]``
    in the pickle ``training_data_<method>.pkl`` (utils.py:139-155).

At N >= 100k a float64 K is 80+ GB, so a pickle (one in-memory blob) no longer works.
Here:
  * ``read_csv_codes`` parses an ``Id,seq`` CSV straight into the symbol codes the C ABI
    takes (no DataFrame, no per-row Python strings kept);
  * ``gram_to_npy`` builds K on the device in row slabs (``kmg_gram_to_host``: posting
    index and diagonal built once, each slab's copy overlapping the next slab's Gram) and
    streams them into a ``.npy`` file opened with ``numpy.lib.format.open_memmap``, so
    host memory never holds K;
  * ``load_gram`` maps such a file read-only (``np.load(..., mmap_mode='r')``).
The ``.npy`` file holds exactly the array ``select_method`` would return for SP / MM
(float64, or int32 raw spectrum counts on request).
"""
import numpy as np

from . import _lib as L
from . import encode as E
from . import params as P


def read_csv_codes(path):
    """``Id,seq`` CSV -> (ids int64[n], codes uint8[n, ldc], lens int32[n]).

    Same column contract as the reference's ``pd.read_csv`` use (utils.py:28,41): a
    header line naming ``Id`` and ``seq``, one record per line, no quoting.
    """
    with open(path, "rb") as f:
        data = f.read()
    lines = data.splitlines()
    if not lines:
        raise ValueError(f"{path}: empty file")
    header = [h.strip() for h in lines[0].decode("ascii").split(",")]
    try:
        ci, cs = header.index("Id"), header.index("seq")
    except ValueError:
        raise ValueError(f"{path}: header must name 'Id' and 'seq', got {header}") from None
    ids, seqs = [], []
    for ln in lines[1:]:
        if not ln.strip():
            continue
        fields = ln.split(b",")
        if len(fields) != len(header):
            raise ValueError(f"{path}: malformed record {ln[:60]!r}")
        ids.append(int(fields[ci]))
        seqs.append(fields[cs].strip().decode("ascii"))
    codes, lens = E.encode(seqs)
    return np.asarray(ids, dtype=np.int64), codes, lens


def method_params(method):
    """Device parameters of the SP / MM method strings (grammar of kernels.py:479-489:
    ``SP_k<k>``, ``MM_k<k>_m<m>``; integer fields parsed as ``int(tok[1:])``)."""
    tok = method.split("_")
    if method.startswith("SP"):
        return P.make(L.KMG_SPECTRUM, k=int(tok[1][1:])), False
    if method.startswith("MM"):
        return P.make(L.KMG_MISMATCH, k=int(tok[1][1:]), m=int(tok[2][1:]), window=101,
                      normalize=1), True
    raise NotImplementedError(f"gram_to_npy: method {method!r} (SP / MM only)")


def gram_to_npy(path, codes, lens, method, out_dtype=L.KMG_F64, slab_rows=None, ctx=None):
    """Build the full K of ``method`` over (codes, lens) into the ``.npy`` file ``path``.

    K is computed on the device one row slab at a time and copied into the memory-mapped
    file, so host memory holds one slab.  Returns the read-only memmap of the result.
    """
    params, is_mm = method_params(method)
    if is_mm and not E.is_acgt_only(codes, lens):
        raise ValueError("mismatch kernel: non-ACGT symbols (reference format() raises)")
    if is_mm and (lens < 101).any():
        raise ValueError("mismatch kernel: sequences shorter than the fixed 101 window")
    if out_dtype == L.KMG_I32 and is_mm:
        raise ValueError("normalised mismatch K is float64")
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    lens = np.ascontiguousarray(lens, dtype=np.int32)
    n, ldc = codes.shape
    dt = np.dtype(L.DTYPES[out_dtype])
    if slab_rows is None:  # ~2 GB slabs
        slab_rows = max(1, min(n, (2 << 30) // max(1, n * dt.itemsize)))
    out = np.lib.format.open_memmap(path, mode="w+", dtype=dt, shape=(n, n))
    own = ctx is None
    ctx = ctx or L.Context(0)
    d_codes = d_lens = None
    try:
        d_codes, d_lens = ctx.dmalloc(max(1, codes.nbytes)), ctx.dmalloc(max(1, lens.nbytes))
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        if n:
            # one index / diagonal build for all slabs; slab t's copy into the memmap
            # overlaps slab t+1's Gram (kmg_gram_to_host)
            ctx.gram_to_host(params, d_codes, d_lens, n, ldc, out_dtype, slab_rows, out)
        out.flush()
    finally:
        for p in (d_codes, d_lens):
            if p is not None:
                ctx.dfree(p)
        if own:
            ctx.close()
    del out
    return load_gram(path)


def load_gram(path):
    """Read-only memory map of a K written by ``gram_to_npy`` (no pickle, nothing executed)."""
    return np.load(path, mmap_mode="r", allow_pickle=False)
