#!/bin/bash
# r01 session 3: parity suite, default bench, mismatch / index sweeps.
set -u
OUT=gpurun_out/r01s3d
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed $?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -u tools/tune.py sp --reps 10 --sets '[{}, {"KMG_SP_G":"2"}, {"KMG_IDX_V2":"0"}, {"KMG_IDX_SEQS":"40"}, {"KMG_IDX_SEQS":"160"}]' > "$OUT/tune_sp.jsonl" 2> "$OUT/tune_sp.err" || { echo "tune sp failed $?"; tail -20 "$OUT/tune_sp.err"; exit 1; }
cat "$OUT/tune_sp.jsonl"
timeout -k 10 300 python3 -u tools/tune.py mm --reps 5 --sets '[{}, {"KMG_IDX_V2":"0"}, {"KMG_IDX_BUCKETS":"2048"}, {"KMG_IDX_BUCKETS":"4096"}, {"KMG_IDX_BUCKETS":"384"}]' > "$OUT/tune_mm.jsonl" 2> "$OUT/tune_mm.err" || { echo "tune mm failed $?"; tail -20 "$OUT/tune_mm.err"; exit 1; }
cat "$OUT/tune_mm.jsonl"
timeout -k 10 300 python3 -u tools/tune.py mm --k 8 --reps 5 --sets '[{}, {"KMG_MM_VARIANT":"6"}]' > "$OUT/tune_mm8.jsonl" 2> "$OUT/tune_mm8.err" || { echo "tune mm8 failed $?"; tail -20 "$OUT/tune_mm8.err"; exit 1; }
cat "$OUT/tune_mm8.jsonl"
timeout -k 10 300 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
