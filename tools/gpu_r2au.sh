#!/bin/bash
# 8-bit round slabs: multi-GPU assembly tests + one-GPU rehearsal timings.
set -u
TAG=${1:-r2au}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_multi.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
KMG_BLOCKS_CHECK=1 timeout -k 10 400 python3 -u tools/time_blocks.py '[["sp", 100000, 1], ["sp", 20000, 1], ["mm", 20000, 3]]' > "$OUT/blocks.jsonl" 2>&1 || { echo "blocks failed"; tail $OUT/blocks.jsonl; exit 1; }
cat $OUT/blocks.jsonl
