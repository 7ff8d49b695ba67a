"""Spectrum k=8 N=20000 device build: wall per build with stage timing on vs off (the
launch gaps the stage events add).  Usage: python3 tools/time_gap.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kernel-methods-for-genomics_amd")]
from kmgram import _lib as L, encode as E, params as P  # noqa: E402


def main():
    n, steps = 20000, 50
    ctx = L.Context(0)
    codes, lens = E.synthetic(n, 101, seed=3)
    dc, dl = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(dc, codes)
    ctx.h2d(dl, lens)
    do = ctx.dmalloc(n * n * 4)
    prm = P.make(L.KMG_SPECTRUM, k=8)
    for rep in range(3):
        for timing in (False, True):
            ctx.set_timing(timing)
            for _ in range(3):
                ctx.gram_device(prm, dc, dl, n, codes.shape[1], 0, n, L.KMG_I32, do, n)
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                ctx.gram_device(prm, dc, dl, n, codes.shape[1], 0, n, L.KMG_I32, do, n)
            ctx.synchronize()
            ms = (time.perf_counter() - t0) / steps * 1e3
            print(json.dumps({"timing": timing, "rep": rep, "ms": ms}), flush=True)
    ctx.set_timing(False)
    ctx.close()


if __name__ == "__main__":
    main()
