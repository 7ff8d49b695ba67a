#!/bin/bash
set -u
OUT=gpurun_out/${1:-r2z}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/time_mm.py '[{"kind": "sp", "k": 5, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 5}, {"kind": "sp", "k": 4, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 5}, {"kind": "sp", "k": 5, "steps": 10, "KMG_DENSE_KMAX_SP": 5}, {"kind": "sp", "k": 6, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 5}, {"kind": "sp", "k": 5, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 4}, {"kind": "sp", "k": 4, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 4}, {"kind": "sp", "k": 5, "steps": 10, "KMG_DENSE_KMAX_SP": 4}, {"kind": "sp", "k": 6, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 4}, {"kind": "sp", "k": 5, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 3}, {"kind": "sp", "k": 4, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 3}, {"kind": "sp", "k": 5, "steps": 10, "KMG_DENSE_KMAX_SP": 3}, {"kind": "sp", "k": 6, "n": 9000, "f64": 1, "steps": 10, "KMG_DENSE_KMAX_SP": 3}]' > "$OUT/time.jsonl" 2>&1 || { echo "time failed"; tail "$OUT/time.jsonl"; exit 1; }
cat "$OUT/time.jsonl"
