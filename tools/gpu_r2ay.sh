#!/bin/bash
# Dense int8 Gram: k-stage of 64 vs 128 bytes (parity with both, interleaved A/B timings).
set -u
TAG=${1:-r2ay}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dense.py tests/test_gappy_intended.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest64.txt" 2>&1 || { echo "pytest64 failed"; tail -30 "$OUT/pytest64.txt"; exit 1; }
KMG_DENSE_BK=128 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dense.py tests/test_gappy_intended.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest128.txt" 2>&1 || { echo "pytest128 failed"; tail -30 "$OUT/pytest128.txt"; exit 1; }
tail -1 "$OUT/pytest64.txt" "$OUT/pytest128.txt"
timeout -k 10 300 python3 -u tools/ab_env.py '{"kind": "mm", "k": 6, "n": 20000, "norm": 0, "reps": 3, "steps": 10, "seed": 3}' '[{}, {"KMG_DENSE_BK": 128}]' > "$OUT/ab.jsonl" 2>&1 || { echo "ab failed"; tail $OUT/ab.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/ab_env.py '{"kind": "sp", "k": 5, "n": 20000, "reps": 3, "steps": 10}' '[{}, {"KMG_DENSE_BK": 128}]' >> "$OUT/ab.jsonl" 2>&1 || { echo "ab2 failed"; tail $OUT/ab.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/ab_env.py '{"kind": "mm", "k": 7, "n": 20000, "norm": 0, "reps": 2, "steps": 3, "seed": 3}' '[{}, {"KMG_DENSE_BK": 128}]' >> "$OUT/ab.jsonl" 2>&1 || { echo "ab3 failed"; tail $OUT/ab.jsonl; exit 1; }
cut -c1-220 $OUT/ab.jsonl
