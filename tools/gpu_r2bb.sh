#!/bin/bash
set -u
TAG=${1:-r2bb}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/time_mm.py '[
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false, "KMG_IDX_SEQS": 400},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false, "KMG_IDX_SEQS": 200},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false, "KMG_IDX_SEQS": 400, "KMG_IDX_BUCKETS": 1024},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false, "KMG_IDX_BUCKETS": 1024},
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false},
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false, "KMG_IDX_SEQS": 40},
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false, "KMG_IDX_SEQS": 160}
]' > "$OUT/idx.jsonl" 2>&1 || { echo "time failed"; tail $OUT/idx.jsonl; exit 1; }
cut -c1-230 $OUT/idx.jsonl
