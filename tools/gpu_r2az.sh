#!/bin/bash
# WD on bit planes: parity + timings (N=9000 run.py sizes, N=20000).
set -u
TAG=${1:-r2az}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread -k "wd or WD or golden or blocks or triangle" > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.txt"; exit 1; }
tail -n 1 "$OUT/pytest.txt"
timeout -k 10 300 python3 -u tools/time_mm.py '[
 {"kind": "wd", "d": 4, "n": 9000, "steps": 10},
 {"kind": "wd", "d": 5, "n": 9000, "steps": 10},
 {"kind": "wd", "d": 10, "n": 9000, "steps": 10},
 {"kind": "wd", "d": 5, "n": 20000, "steps": 5}
]' > "$OUT/wd.jsonl" 2>&1 || { echo "time failed"; tail $OUT/wd.jsonl; exit 1; }
cut -c1-200 $OUT/wd.jsonl
