#!/bin/bash
# Index gather pass with register-cached items: parity tests + stage timings.
set -u
TAG=${1:-r2al}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 300 python3 -u tools/time_mm.py '[
 {"kind": "sp", "k": 8, "n": 20000, "steps": 20, "check": false},
 {"kind": "sp", "k": 8, "n": 100000, "steps": 5, "check": false},
 {"kind": "mm", "n": 20000, "norm": 1, "steps": 5},
 {"kind": "mm", "n": 200000, "rows": 25000, "norm": 0, "steps": 2}
]' > "$OUT/idx.jsonl" 2>&1 || { echo "time failed"; tail $OUT/idx.jsonl; exit 1; }
cat $OUT/idx.jsonl
