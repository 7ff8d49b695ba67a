#!/bin/bash
set -u
TAG=${1:-r2ar}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/ab_env.py '{"kind": "sp", "n": 20000, "reps": 4, "steps": 20}' '[{}, {"KMG_SP_STORE": 1}, {"KMG_SP_CHUNK": 10000}, {"KMG_SP_CHUNK": 10000, "KMG_SP_STORE": 2}]' > "$OUT/ab.jsonl" 2>&1 || { echo "ab failed"; tail $OUT/ab.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/ab_env.py '{"kind": "sp", "n": 20000, "reps": 3, "steps": 10, "f64": 1}' '[{}, {"KMG_SP_ORDER": 0}, {"KMG_SP_CHUNK": 10000}]' >> "$OUT/ab.jsonl" 2>&1 || { echo "ab2 failed"; tail $OUT/ab.jsonl; exit 1; }
cut -c1-200 $OUT/ab.jsonl
