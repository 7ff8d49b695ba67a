#!/bin/bash
# r01 session 3: parity suite, default bench, mismatch v7 vs v6 sweep, index knobs.
set -u
OUT=gpurun_out/r01s3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed $?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -u tools/tune.py mm --reps 5 --sets '[{}, {"KMG_MM_G":"8","KMG_MM_D":"2"}, {"KMG_MM_G":"2","KMG_MM_D":"2"}, {"KMG_MM_G":"4","KMG_MM_D":"3"}, {"KMG_MM_G":"8","KMG_MM_D":"3"}, {"KMG_MM_G":"4","KMG_MM_D":"4"}, {"KMG_MM_VARIANT":"6"}]' > "$OUT/tune_mm.jsonl" 2> "$OUT/tune_mm.err" || { echo "tune mm failed $?"; tail -20 "$OUT/tune_mm.err"; exit 1; }
cat "$OUT/tune_mm.jsonl"
timeout -k 10 300 python3 -u tools/tune.py sp --reps 10 --sets '[{}, {"KMG_IDX_SEQS":"40"}, {"KMG_IDX_SEQS":"80"}, {"KMG_IDX_SEQS":"128"}, {"KMG_IDX_SEQS":"32"}, {"KMG_IDX_THREADS":"512"}, {"KMG_IDX_SEQS":"160"}]' > "$OUT/tune_sp.jsonl" 2> "$OUT/tune_sp.err" || { echo "tune sp failed $?"; tail -20 "$OUT/tune_sp.err"; exit 1; }
cat "$OUT/tune_sp.jsonl"
timeout -k 10 300 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
