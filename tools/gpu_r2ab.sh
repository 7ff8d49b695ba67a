#!/bin/bash
# GPU suite on the restored tree + config-5 (N=200000 MM(9,1) raw slab) formulation /
# chunk experiments.  Usage: tools/gpu_r2ab.sh <tag>
set -u
TAG=${1:-r2ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/gpu_tests.sh "$TAG" > /dev/null || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 400 python3 -u tools/time_mm.py '[
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_MM_FORM": 2},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_MM_CHUNK": 28576},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2, "KMG_MM_CHUNK": 14288}
]' > "$OUT/c5.jsonl" 2>&1 || { echo "time failed"; tail $OUT/c5.jsonl; exit 1; }
cat $OUT/c5.jsonl
