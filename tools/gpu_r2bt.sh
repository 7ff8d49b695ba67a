#!/bin/bash
# Substring (k=5, k=12) and LA (sum / max form) Gram timing at N=1000, one process.
set -u
OUT=gpurun_out/r2bt
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/timing.jsonl"
for cfg in '{"kind": "ss", "k": 5, "n": 1000, "reps": 2, "steps": 3}' \
           '{"kind": "ss", "k": 12, "n": 1000, "reps": 2, "steps": 3}' \
           '{"kind": "la", "smith": 0, "n": 1000, "reps": 2, "steps": 3}' \
           '{"kind": "la", "smith": 1, "n": 1000, "reps": 2, "steps": 3}'; do
  timeout -k 10 200 python3 -u tools/ab_env.py "$cfg" '[{}]' >> "$OUT/timing.jsonl" 2>> "$OUT/timing.err" || { echo "timing failed"; tail -20 $OUT/timing.err; exit 1; }
done
cat "$OUT/timing.jsonl"
