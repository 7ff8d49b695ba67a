#!/bin/bash
set -u
TAG=${1:-r2ax}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u tools/ab_env.py '{"kind": "sp", "n": 100000, "reps": 3, "steps": 5, "seed": 4}' '[{}, {"KMG_SP_CHUNK": 25000}, {"KMG_SP_CHUNK": 33336}, {"KMG_SP_CHUNK": 16672}, {"KMG_SP_CHUNK": 12504}]' > "$OUT/ab.jsonl" 2>&1 || { echo "ab failed"; tail $OUT/ab.jsonl; exit 1; }
cut -c1-200 $OUT/ab.jsonl
