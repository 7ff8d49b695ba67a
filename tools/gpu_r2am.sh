#!/bin/bash
# Slot kernel: 16-bit accumulator / workgroup size experiment (k = 9).
set -u
TAG=${1:-r2am}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python3 -u tools/time_mm.py '[
 {"kind": "mm", "n": 20000, "norm": 1, "steps": 5},
 {"kind": "mm", "n": 20000, "norm": 1, "steps": 5, "KMG_MM_ACC16": 1, "KMG_MM_THREADS": 512},
 {"kind": "mm", "n": 20000, "norm": 1, "steps": 5, "KMG_MM_ACC16": 1, "KMG_MM_THREADS": 256},
 {"kind": "mm", "n": 20000, "norm": 1, "steps": 5, "KMG_MM_ACC16": 1, "KMG_MM_THREADS": 1024},
 {"kind": "mm", "n": 20000, "norm": 1, "steps": 5, "KMG_MM_THREADS": 512},
 {"kind": "mm", "n": 20000, "norm": 0, "steps": 5},
 {"kind": "mm", "n": 20000, "norm": 0, "steps": 5, "KMG_MM_ACC16": 1, "KMG_MM_THREADS": 512},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_MM_ACC16": 1, "KMG_MM_THREADS": 512}
]' > "$OUT/acc16.jsonl" 2>&1 || { echo "time failed"; tail $OUT/acc16.jsonl; exit 1; }
cut -c1-260 $OUT/acc16.jsonl
