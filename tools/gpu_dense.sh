#!/bin/bash
# GPU session: dense-path parity, then timing of dense vs posting formulations.
set -u
TAG=${1:-d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -m pytest tests/test_gpu_dense.py -x -q > "$OUT/pytest_dense.log" 2>&1 || { echo "dense tests failed $?"; tail -40 "$OUT/pytest_dense.log"; exit 1; }
tail -2 "$OUT/pytest_dense.log"
for k in 4 5 6 7 8; do
  timeout -k 10 200 python3 tools/tune.py sp --k $k --reps 5 --sets '[{"KMG_ALGO":"1"},{"KMG_ALGO":"2"}]' >> "$OUT/tune.jsonl" 2>> "$OUT/tune.err" || { echo "tune sp $k failed"; tail -20 "$OUT/tune.err"; exit 1; }
done
for k in 4 5 6; do
  timeout -k 10 200 python3 tools/tune.py mm --k $k --reps 5 --sets '[{"KMG_ALGO":"1"}]' >> "$OUT/tune.jsonl" 2>> "$OUT/tune.err" || { echo "tune mm $k failed"; tail -20 "$OUT/tune.err"; exit 1; }
done
for k in 7 8 9; do
  timeout -k 10 200 python3 tools/tune.py mm --k $k --reps 3 --sets '[{"KMG_ALGO":"1"},{"KMG_ALGO":"2"}]' >> "$OUT/tune.jsonl" 2>> "$OUT/tune.err" || { echo "tune mm $k failed"; tail -20 "$OUT/tune.err"; exit 1; }
done
cat "$OUT/tune.jsonl"
