#!/bin/bash
# Index-build geometry at N=200000 (config 5 slab): coarse buckets / sequences per block.
set -u
TAG=${1:-r2ad}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u tools/time_mm.py '[
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_IDX_BUCKETS": 4096},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_IDX_BUCKETS": 8192},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_IDX_BUCKETS": 4096, "KMG_IDX_SEQS": 200},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_IDX_SEQS": 200},
 {"kind": "mm", "n": 20000, "norm": 0, "steps": 5, "KMG_IDX_BUCKETS": 2048},
 {"kind": "mm", "n": 20000, "norm": 0, "steps": 5}
]' > "$OUT/idx.jsonl" 2>&1 || { echo "time failed"; tail $OUT/idx.jsonl; exit 1; }
cat $OUT/idx.jsonl
