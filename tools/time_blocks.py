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
    for kind, n, dt in (("sp", 20000, L.KMG_I32), ("mm", 20000, L.KMG_F64)):
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
            print(json.dumps({"kind": kind, "n": n, "world": world, "gather": gather,
                              "block": block, "ms": ms}), flush=True)
            ctx.dfree(do)
        ctx.dfree(dc)
        ctx.dfree(dl)
    ctx.close()


if __name__ == "__main__":
    main()
