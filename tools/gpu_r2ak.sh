#!/bin/bash
# LA intended kernel tests + timing.
set -u
TAG=${1:-r2ak}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_la_intended.py tests/test_gpu_parity.py -k "la or LA or golden" -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 200 python3 -u - > "$OUT/la_time.json" 2>&1 <<'PY' || { echo "timing failed"; cat "$OUT/la_time.json"; exit 1; }
import json, sys, time
sys.path[:0] = ["kernel-methods-for-genomics_amd", "oracle"]
import numpy as np
from kmgram import _lib as L, encode as E, params as P
ctx = L.Context(0)
for n in (2000, 4000):
    codes, lens = E.synthetic(n, 101, seed=4)
    for smith in (0, 1):
        p = P.make(L.KMG_LOCALALIGN, smith=smith, la_mode=L.KMG_LA_INTENDED, la_e=11, la_d=1, la_beta=0.5)
        dc, dl = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
        ctx.h2d(dc, codes); ctx.h2d(dl, lens)
        do = ctx.dmalloc(n * n * 8)
        ctx.gram_device(p, dc, dl, n, 101, 0, n, L.KMG_F64, do, n); ctx.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            ctx.gram_device(p, dc, dl, n, 101, 0, n, L.KMG_F64, do, n)
        ctx.synchronize()
        ms = (time.perf_counter() - t) / 3 * 1e3
        cells = n * (n + 1) / 2 * 101 * 101
        print(json.dumps({"n": n, "smith": smith, "ms": ms, "Gcells_per_s": cells / ms / 1e6}))
        for x in (dc, dl, do): ctx.dfree(x)
PY
cat "$OUT/la_time.json"
