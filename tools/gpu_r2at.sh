#!/bin/bash
# Upper-triangle assembly at the new headline N=100000 (one-GPU rehearsal of G=8) with oracle rows.
set -u
TAG=${1:-r2at}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KMG_BLOCKS_CHECK=1 timeout -k 10 400 python3 -u tools/time_blocks.py '[["sp", 100000, 1]]' > "$OUT/blocks.jsonl" 2>&1 || { echo "blocks failed"; tail $OUT/blocks.jsonl; exit 1; }
cat $OUT/blocks.jsonl
