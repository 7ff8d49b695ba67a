#!/bin/bash
# dense MFMA path: parity (both tile shapes), timings
set -u
TAG=${1:-r2w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for W in 2 4; do
KMG_DENSE_SYM=0 KMG_DENSE_WN=$W timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dense.py tests/test_gappy_intended.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest$W.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest$W.txt"; exit 1; }
tail -1 "$OUT/pytest$W.txt"
done
C='[{"kind": "sp", "k": 5, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 4, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 5, "f64": 1, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 1}, {"kind": "mm", "k": 6, "norm": 0, "steps": 10, "check": false, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 5, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 1}, {"kind": "mm", "k": 6, "n": 9000, "steps": 10, "check": false, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 5, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 4, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 5, "f64": 1, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 1}, {"kind": "mm", "k": 6, "norm": 0, "steps": 10, "check": false, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 5, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 1}, {"kind": "mm", "k": 6, "n": 9000, "steps": 10, "check": false, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 1}, {"kind": "sp", "k": 5, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 0}, {"kind": "sp", "k": 4, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 0}, {"kind": "sp", "k": 5, "f64": 1, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 0}, {"kind": "mm", "k": 6, "norm": 0, "steps": 10, "check": false, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 0}, {"kind": "sp", "k": 5, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 0}, {"kind": "mm", "k": 6, "n": 9000, "steps": 10, "check": false, "KMG_DENSE_WN": 2, "KMG_DENSE_SYM": 0}, {"kind": "sp", "k": 5, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 0}, {"kind": "sp", "k": 4, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 0}, {"kind": "sp", "k": 5, "f64": 1, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 0}, {"kind": "mm", "k": 6, "norm": 0, "steps": 10, "check": false, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 0}, {"kind": "sp", "k": 5, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 0}, {"kind": "mm", "k": 6, "n": 9000, "steps": 10, "check": false, "KMG_DENSE_WN": 4, "KMG_DENSE_SYM": 0}]'
timeout -k 10 300 python3 -u tools/time_mm.py "$C" > "$OUT/time.jsonl" 2>&1 || { echo "time failed"; tail "$OUT/time.jsonl"; exit 1; }
cat "$OUT/time.jsonl"
timeout -k 10 120 python3 -u tools/time_gap.py > "$OUT/gap.jsonl" 2>&1 || { echo gap failed; tail "$OUT/gap.jsonl"; exit 1; }
cat "$OUT/gap.jsonl"
