#!/bin/bash
# One GPU-box session: parity tests, default bench, mismatch variant sweep.
# usage: bash tools/gpu_session.sh <tag>
set -u
TAG=${1:-s}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed $?"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ "${SWEEP:-0}" = "1" ]; then
  timeout -k 10 400 python3 tools/tune.py mm --reps 5 --sets '[{}, {"KMG_MM_VARIANT":"6","KMG_MM_G":"2","KMG_MM_V":"8","KMG_MM_U":"2"}, {"KMG_MM_VARIANT":"6","KMG_MM_G":"1","KMG_MM_V":"8","KMG_MM_U":"4"}, {"KMG_MM_VARIANT":"6","KMG_MM_G":"8","KMG_MM_V":"4","KMG_MM_U":"1"}, {"KMG_MM_VARIANT":"6","KMG_MM_G":"4","KMG_MM_V":"8","KMG_MM_U":"1"}, {"KMG_MM_VARIANT":"5"}, {"KMG_MM_VARIANT":"5","KMG_MM_G":"2","KMG_MM_U":"12"}, {"KMG_MM_VARIANT":"4"}, {"KMG_MM_VARIANT":"3"}, {"KMG_MM_VARIANT":"2"}, {"KMG_MM_VARIANT":"6","KMG_MM_THREADS":"512"}, {"KMG_MM_VARIANT":"6","KMG_MM_CHUNK":"10240"}]' > "$OUT/tune_mm.jsonl" 2> "$OUT/tune_mm.err" || { echo "tune failed $?"; tail -20 "$OUT/tune_mm.err"; exit 1; }
  cat "$OUT/tune_mm.jsonl"
fi
