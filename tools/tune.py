#!/usr/bin/env python3
"""Parameter sweep for the device Gram path (GPU box): runs one workload under several
environment settings in ONE process and prints per-stage device times (HIP events).

usage: python tools/tune.py <sp|mm> [--n N] [--reps R] [--sets JSON]
  --sets: JSON list of {ENV: value} dicts (default: a built-in sweep per workload)
Every setting's output rows are compared with the first setting's (must be identical).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kernel-methods-for-genomics_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

from kmgram import _lib as L  # noqa: E402
from kmgram import encode as E  # noqa: E402
from kmgram import params as P  # noqa: E402

DEFAULT = {
    "sp": [{}, {"KMG_SP_NT": "1"}, {"KMG_SP_CHUNK": "10000"}, {"KMG_IDX_SEQS": "32"},
           {"KMG_IDX_SEQS": "128"}, {"KMG_IDX_THREADS": "256"}, {"KMG_IDX_THREADS": "1024"},
           {"KMG_IDX_BUCKETS": "128"}, {"KMG_IDX_BUCKETS": "1024"}],
    "mm": [{}, {"KMG_MM_G": "2"}, {"KMG_MM_G": "8"}, {"KMG_MM_CHUNK": "16384"},
           {"KMG_MM_CHUNK": "5120"}, {"KMG_MM_CHUNK": "16384", "KMG_MM_G": "8"}],
}
KNOBS = ("KMG_ALGO", "KMG_MM_SLOTV", "KMG_SP_PERSIST", "KMG_MM_TRI", "KMG_MM_PORDER", "KMG_SP_NT", "KMG_SP_CHUNK", "KMG_MM_G", "KMG_MM_U", "KMG_MM_V", "KMG_MM_D", "KMG_MM_THREADS",
         "KMG_MM_CHUNK", "KMG_IDX_SEQS", "KMG_IDX_THREADS", "KMG_IDX_BUCKETS", "KMG_MM_VARIANT",
         "KMG_SP_G", "KMG_DIAG_SMALL")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload", choices=["sp", "mm"])
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sets", type=str, default=None)
    ap.add_argument("--k", type=int, default=None, help="k-mer length (default 8 sp / 9 mm)")
    ap.add_argument("--m", type=int, default=1)
    args = ap.parse_args()
    sets = json.loads(args.sets) if args.sets else DEFAULT[args.workload]
    n = args.n
    codes, lens = E.synthetic(n, 101, seed=2 if args.workload == "sp" else 3)
    ctx = L.Context(0)
    k = args.k or (8 if args.workload == "sp" else 9)
    if args.workload == "sp":
        params, dt = P.make(L.KMG_SPECTRUM, k=k), L.KMG_I32
    else:
        params, dt = P.make(L.KMG_MISMATCH, k=k, m=args.m, window=101, normalize=1), L.KMG_F64
    esz = np.dtype(L.DTYPES[dt]).itemsize
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    d_out = ctx.dmalloc(n * n * esz)
    probe_rows = [0, n // 3, n - 1]
    import cref
    if args.workload == "sp":
        oracle = {r: cref.spectrum(codes, lens, k, rows=(r, r + 1))[0] for r in probe_rows}
    else:
        oracle = {r: cref.mismatch_rows(codes, lens, k, args.m, rows=(r, r + 1))[0]
                  for r in probe_rows}
    ref = None
    for st in sets:
        for kn in KNOBS:
            os.environ.pop(kn, None)
        os.environ.update({k: str(v) for k, v in st.items()})
        for _ in range(2):
            ctx.gram_device(params, d_codes, d_lens, n, 101, 0, n, dt, d_out, n)
        ctx.synchronize()
        ctx.set_timing(True)
        ctx.timing_reset()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ctx.gram_device(params, d_codes, d_lens, n, 101, 0, n, dt, d_out, n)
        ctx.synchronize()
        wall = (time.perf_counter() - t0) / args.reps * 1e3
        ctx.set_timing(False)
        stages = {}
        for s in ("count", "scan", "place", "fine", "pack", "extract", "features", "diag", "gram", "mirror"):
            tot, cnt = ctx.stage_stats(s)
            if cnt:
                stages[s] = round(tot / cnt * 1e3, 1)
        ctx.memset(d_out, 0xA5, n * n * esz)  # poison, then one checked run
        ctx.gram_device(params, d_codes, d_lens, n, 101, 0, n, dt, d_out, n)
        ctx.synchronize()
        rows, ok = [], True
        for r in probe_rows:
            row = np.empty(n, dtype=L.DTYPES[dt])
            ctx.d2h(row, ctypes.c_void_p(d_out.value + r * n * esz))
            rows.append(row)
            ok &= bool(np.array_equal(row.astype(oracle[r].dtype), oracle[r]))
        same = None
        if ref is None:
            ref = rows
        else:
            same = all(np.array_equal(a, b) for a, b in zip(rows, ref))
        print(json.dumps({"k": k, "set": st, "wall_ms": round(wall, 4), "stages_us": stages,
                          "same_as_first": same, "oracle_ok": ok}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
