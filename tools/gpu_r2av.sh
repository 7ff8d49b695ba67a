#!/bin/bash
set -u
TAG=${1:-r2av}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/alloc.jsonl"
for ord in 01 10 01 10; do
  timeout -k 10 120 python3 -u tools/alloc_modes.py $ord >> "$OUT/alloc.jsonl" 2>&1 || { echo "alloc failed"; tail $OUT/alloc.jsonl; exit 1; }
done
cat $OUT/alloc.jsonl
