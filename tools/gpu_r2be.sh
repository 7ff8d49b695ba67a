#!/bin/bash
set -u
TAG=${1:-r2be}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u tools/time_mm.py '[
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "check": false},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "check": false, "KMG_IDX_SEQS": 800},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "check": false, "KMG_IDX_SEQS": 400},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "check": false, "KMG_IDX_SEQS": 800, "KMG_IDX_BUCKETS": 2048}
]' > "$OUT/idx.jsonl" 2>&1 || { echo "time failed"; tail $OUT/idx.jsonl; exit 1; }
cut -c1-250 $OUT/idx.jsonl
