#!/bin/bash
set -u
OUT=gpurun_out/${1:-r2x}
mkdir -p "$OUT"
timeout -k 10 120 ./tools/store_patterns 20000 > "$OUT/store.jsonl" 2>&1 || { echo failed; cat "$OUT/store.jsonl"; exit 1; }
cat "$OUT/store.jsonl"
