#!/bin/bash
# Spectrum grid order (row- vs chunk-major) x chunking, N=20000 and N=100000.
set -u
TAG=${1:-r2ao}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u tools/time_mm.py '[
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false},
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false, "KMG_SP_CHUNK": 10000},
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false, "KMG_SP_CHUNK": 10000, "KMG_SP_ORDER": 1},
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false, "KMG_SP_CHUNK": 10000, "KMG_SP_ORDER": 1, "KMG_SP_STORE": 2},
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false, "KMG_SP_CHUNK": 6672, "KMG_SP_ORDER": 1, "KMG_SP_STORE": 2},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false, "KMG_SP_ORDER": 1},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false, "KMG_SP_ORDER": 1, "KMG_SP_STORE": 2},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false, "KMG_SP_ORDER": 1, "KMG_SP_CHUNK": 12504}
]' > "$OUT/order.jsonl" 2>&1 || { echo "time failed"; tail $OUT/order.jsonl; exit 1; }
cut -c1-220 $OUT/order.jsonl
