"""A/B of the spectrum grid order (KMG_SP_ORDER 0 / 1) in ONE process on ONE output
buffer, alternating, so placement / clock drift cannot masquerade as a difference."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kernel-methods-for-genomics_amd")]
from kmgram import _lib as L, encode as E, params as P  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    ctx = L.Context(0)
    codes, lens = E.synthetic(n, 101, seed=4)
    p = P.make(L.KMG_SPECTRUM, k=8)
    dc, dl = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(dc, codes)
    ctx.h2d(dl, lens)
    do = ctx.dmalloc(n * n * 4)
    for rep in range(reps):
        for order in (0, 1):
            os.environ["KMG_SP_ORDER"] = str(order)
            ctx.reload_tuning()
            ctx.gram_device(p, dc, dl, n, 101, 0, n, L.KMG_I32, do, n)
            ctx.synchronize()
            ctx.set_timing(2)
            ctx.timing_reset()
            t = time.perf_counter()
            for _ in range(5):
                ctx.gram_device(p, dc, dl, n, 101, 0, n, L.KMG_I32, do, n)
            ctx.synchronize()
            wall = (time.perf_counter() - t) / 5 * 1e3
            tot, cnt = ctx.stage_stats("gram")
            ctx.set_timing(0)
            print(json.dumps({"n": n, "rep": rep, "order": order, "ms": wall, "gram_ms": tot / cnt}),
                  flush=True)


if __name__ == "__main__":
    main()
