"""Time kmg_gram_blocks assemblies on one GPU (device-resident, stage timing off):
world=1 direct rows vs the upper-triangle slab path (gather 2: slabs + copy + mirror, no
RCCL on one rank), and gather 3 (every rank's slabs of a G-rank layout computed locally).
Usage: python3 tools/time_blocks.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kernel-methods-for-genomics_amd")]
import numpy as np  # noqa: E402
from kmgram import _lib as L, encode as E, params as P  # noqa: E402
from kmgram.shard import default_block, rows_padded  # noqa: E402


def main():
    ctx = L.Context(0)
    cases = (("sp", 20000, L.KMG_I32), ("mm", 20000, L.KMG_F64))
    if len(sys.argv) > 1:  # e.g. '[["sp", 100000, 1]]' (dtype codes of kmgram._lib)
        cases = [tuple(c) for c in json.loads(sys.argv[1])]
    check = os.environ.get("KMG_BLOCKS_CHECK") == "1"
    for kind, n, dt in cases:
        prm = (P.make(L.KMG_SPECTRUM, k=8) if kind == "sp" else
               P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1))
        codes, lens = E.synthetic(n, 101, seed=5)
        dc, dl = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
        ctx.h2d(dc, codes)
        ctx.h2d(dl, lens)
        esz = np.dtype(L.DTYPES[dt]).itemsize
        for world, gather in ((1, 0), (1, 2), (8, 3), (8, 0)):
            block = n if (world == 1 and gather == 0) else default_block(n, world, n * esz)
            npad = rows_padded(n, world, block)
            do = ctx.dmalloc(npad * n * esz)
            steps = 10 if kind == "sp" else 3
            ctx.gram_blocks(prm, dc, dl, n, codes.shape[1], dt, do, n, world, 0, block, gather)
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                ctx.gram_blocks(prm, dc, dl, n, codes.shape[1], dt, do, n, world, 0, block, gather)
            ctx.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            rec = {"kind": kind, "n": n, "world": world, "gather": gather, "block": block, "ms": ms}
            if check and kind == "sp":  # oracle rows at the ends and the middle
                import ctypes
                sys.path.insert(0, os.path.join(ROOT, "oracle"))
                import cref
                ok = True
                for r in (0, n // 2 + 3, n - 1):
                    row = np.empty(n, dtype=L.DTYPES[dt])
                    ctx.d2h(row, ctypes.c_void_p(do.value + r * n * esz))
                    ok &= bool(np.array_equal(row.astype(np.int64),
                                              cref.spectrum(codes, lens, 8, rows=(r, r + 1))[0]))
                rec["oracle_rows_ok"] = ok
            print(json.dumps(rec), flush=True)
            ctx.dfree(do)
        ctx.dfree(dc)
        ctx.dfree(dl)
    ctx.close()


if __name__ == "__main__":
    main()
