#!/bin/bash
set -u
TAG=${1:-r2aw}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/ab_env.py '{"kind": "sp", "n": 100000, "reps": 3, "steps": 5, "seed": 4}' '[{}, {"KMG_SP_ORDER": 7919}, {"KMG_SP_ORDER": 257}, {"KMG_SP_ORDER": 50021}]' > "$OUT/ab.jsonl" 2>&1 || { echo "ab failed"; tail $OUT/ab.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/ab_env.py '{"kind": "sp", "n": 20000, "reps": 3, "steps": 20}' '[{}, {"KMG_SP_ORDER": 7919}, {"KMG_SP_ORDER": 257}]' >> "$OUT/ab.jsonl" 2>&1 || { echo "ab2 failed"; tail $OUT/ab.jsonl; exit 1; }
cut -c1-200 $OUT/ab.jsonl
