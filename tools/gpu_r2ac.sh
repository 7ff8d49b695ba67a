#!/bin/bash
# Slot-table chunk model at N=200000 (config 5 slab) + config-5 GPU tests.
set -u
TAG=${1:-r2ac}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u tools/time_mm.py '[
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_MM_CHUNK": 28576},
 {"kind": "mm", "n": 20000, "norm": 1, "steps": 5}
]' > "$OUT/c5.jsonl" 2>&1 || { echo "time failed"; tail $OUT/c5.jsonl; exit 1; }
cat $OUT/c5.jsonl
bash tools/gpu_tests.sh "$TAG" -k "config or mismatch" > /dev/null || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
