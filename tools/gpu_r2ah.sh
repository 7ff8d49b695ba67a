#!/bin/bash
set -u
OUT=gpurun_out/${1:-r2ah}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 300 python3 -u tools/time_blocks.py > "$OUT/blocks.jsonl" 2>&1 || { echo "blocks failed"; tail "$OUT/blocks.jsonl"; exit 1; }
cat "$OUT/blocks.jsonl"
