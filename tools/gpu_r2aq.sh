#!/bin/bash
set -u
TAG=${1:-r2aq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/ab_sp_order.py 100000 4 > "$OUT/ab.jsonl" 2>&1 || { echo "ab failed"; tail $OUT/ab.jsonl; exit 1; }
timeout -k 10 300 python3 -u tools/ab_sp_order.py 60000 3 >> "$OUT/ab.jsonl" 2>&1 || { echo "ab60 failed"; tail $OUT/ab.jsonl; exit 1; }
cat $OUT/ab.jsonl
