"""Does the 40 GB K buffer's allocation decide the 'slow box' mode?  One process: a
hipMalloc buffer and a hipExtMallocWithFlags(hipDeviceMallocContiguous) buffer (order
given by argv[1]), each timed with hipMemsetAsync (the fill ceiling) and the N=100000
spectrum Gram.  Run in several processes."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kernel-methods-for-genomics_amd")]
from kmgram import _lib as L, encode as E, params as P  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def alloc(nbytes, contiguous):
    p = ctypes.c_void_p()
    if contiguous:
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(0x4))
    else:
        rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes))
    if rc != 0:
        raise RuntimeError(f"alloc rc {rc}")
    return p


def main():
    order = [bool(int(c)) for c in sys.argv[1]] if len(sys.argv) > 1 else [False, True]
    n = 100000
    ctx = L.Context(0)
    codes, lens = E.synthetic(n, 101, seed=4)
    p8 = P.make(L.KMG_SPECTRUM, k=8)
    dc, dl = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(dc, codes)
    ctx.h2d(dl, lens)
    nb = n * n * 4
    bufs = [(contig, alloc(nb, contig)) for contig in order]
    for rep in range(2):
        for contig, b in bufs:
            ctx.memset(b, 0, nb)
            ctx.synchronize()
            t = time.perf_counter()
            for _ in range(5):
                ctx.memset(b, 0, nb)
            ctx.synchronize()
            fill = nb / ((time.perf_counter() - t) / 5) / 1e9
            ctx.gram_device(p8, dc, dl, n, 101, 0, n, L.KMG_I32, b, n)
            ctx.synchronize()
            ctx.set_timing(2)
            ctx.timing_reset()
            for _ in range(5):
                ctx.gram_device(p8, dc, dl, n, 101, 0, n, L.KMG_I32, b, n)
            ctx.synchronize()
            tot, cnt = ctx.stage_stats("gram")
            ctx.set_timing(0)
            print(json.dumps({"pid": os.getpid(), "rep": rep, "contiguous": contig,
                              "fill_GBps": round(fill, 1), "gram_ms": round(tot / cnt, 3)}), flush=True)
    for _, b in bufs:
        hip.hipFree(b)


if __name__ == "__main__":
    main()
