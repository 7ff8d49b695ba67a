#!/usr/bin/env python3
"""KRR solve (rocSOLVER dpotrf + dpotrs) at n=9000: lower vs upper triangle variant, device
time from the context's "solve" stage.  GPU box only."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kernel-methods-for-genomics_amd"))
import numpy as np  # noqa: E402
from kmgram import _lib as L  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 9000
rng = np.random.default_rng(0)
A = rng.standard_normal((n, 64))
K = A @ A.T / 64.0
y = rng.choice([-1.0, 1.0], size=n)
ctx = L.Context(0)
ref = None
for upper in ("0", "1", "0", "1"):
    os.environ["KMG_POTRF_UPPER"] = upper
    ctx.krr_solve(K, y, 1e-3)  # warm
    ctx.set_timing(True)
    ctx.timing_reset()
    t0 = time.perf_counter()
    for _ in range(3):
        a = ctx.krr_solve(K, y, 1e-3)
    wall = (time.perf_counter() - t0) / 3
    tot, cnt = ctx.stage_stats("solve")
    ctx.set_timing(False)
    if ref is None:
        ref = a
    print({"upper": upper, "solve_ms": tot / max(cnt, 1), "wall_ms_incl_h2d": wall * 1e3,
           "max_rel_diff_vs_first": float(np.max(np.abs(a - ref)) / np.max(np.abs(ref)))}, flush=True)
ctx.close()
