"""Time device-resident Gram builds under KMG_* settings (one JSON line per setting).
Usage: python3 tools/time_mm.py '<json list of {env..., "kind":..}>'"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kernel-methods-for-genomics_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
from kmgram import _lib as L, encode as E, params as P  # noqa: E402

STAGES = ("count", "place", "fine", "pack", "lists", "slots", "nbfill", "diag", "gram", "mirror")


def main():
    cases = json.loads(sys.argv[1])
    ctx = L.Context(0)
    for case in cases:
        env = {k: str(v) for k, v in case.items() if k.startswith("KMG_")}
        for k in [k for k in os.environ if k.startswith("KMG_")]:
            del os.environ[k]
        os.environ.update(env)
        ctx.reload_tuning()
        n = case.get("n", 20000)
        rows = case.get("rows", n)
        kind = case.get("kind", "mm")
        codes, lens = E.synthetic(n, 101, seed=case.get("seed", 3))
        if kind == "mm":
            params = P.make(L.KMG_MISMATCH, k=case.get("k", 9), m=1, window=101,
                            normalize=case.get("norm", 1))
            dt = L.KMG_F64 if case.get("norm", 1) else L.KMG_I32
        elif kind == "sp":
            params, dt = P.make(L.KMG_SPECTRUM, k=case.get("k", 8)), L.KMG_I32
        elif kind == "wd":
            params, dt = P.make(L.KMG_WD, d=case.get("d", 5)), L.KMG_F64
        else:
            raise ValueError(kind)
        if case.get("f64"):
            dt = L.KMG_F64
        esz = np.dtype(L.DTYPES[dt]).itemsize
        dc, dl = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
        ctx.h2d(dc, codes)
        ctx.h2d(dl, lens)
        steps = case.get("steps", 5)
        # pre_mb: device memory held while the output is allocated (shifts where it lands)
        pre = ctx.dmalloc(case["pre_mb"] << 20) if case.get("pre_mb") else None
        cols = case.get("cols")  # [c0, c1]: the column block K[:, c0:c1] (kmg_gram_device_cols)
        if cols:
            c0, c1 = cols
            rows, width = n, c1 - c0
            do = ctx.dmalloc(n * width * esz)

            def run():
                ctx.gram_device_cols(params, dc, dl, n, codes.shape[1], c0, c1, dt, do, width)
        else:
            width = n
            do = ctx.dmalloc(rows * n * esz)

            def run():
                ctx.gram_device(params, dc, dl, n, codes.shape[1], 0, rows, dt, do, n)
        run()
        ctx.synchronize()
        ctx.set_timing(True)
        ctx.timing_reset()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        ctx.synchronize()
        wall = (time.perf_counter() - t0) / steps
        st = {}
        for s in STAGES:
            tot, cnt = ctx.stage_stats(s)
            if cnt:
                st[s] = round(tot / cnt, 4)
        ctx.set_timing(False)
        ok = None
        if case.get("check", True) and kind == "wd":
            import cref
            import ctypes
            ok = True
            for r in (0, rows // 2, rows - 1):
                row = np.empty(n, dtype=np.float64)
                ctx.d2h(row, ctypes.c_void_p(do.value + r * n * esz))
                ok &= bool(np.array_equal(row, cref.wd(codes, lens, case.get("d", 5), rows=(r, r + 1))[0]))
        if case.get("check", True) and kind == "mm":
            import cref
            r = rows - 1
            row = np.empty(width, dtype=L.DTYPES[dt])
            import ctypes
            ctx.d2h(row, ctypes.c_void_p(do.value + r * width * esz))
            ref = (cref.mismatch_rows(codes, lens, case.get("k", 9), 1, rows=(r, r + 1))[0]
                   if case.get("norm", 1) else
                   cref.mismatch_raw(codes, lens, case.get("k", 9), 1, rows=(r, r + 1))[0])
            if cols:
                ref = ref[cols[0]:cols[1]]
            ok = bool(np.array_equal(row.astype(ref.dtype), ref))
        addr = do.value
        for p in (do, dc, dl) + ((pre,) if pre else ()):
            ctx.dfree(p)
        print(json.dumps({"case": case, "ms": wall * 1e3, "stages": st, "check": ok,
                          "out_addr": hex(addr)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
