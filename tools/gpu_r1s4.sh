#!/bin/bash
# r01 session 4: dense learners (KRR/KLR) parity, full GPU parity suite, default bench
# (with the downstream consumer measurements).
set -u
OUT=gpurun_out/r01s4${1:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_learners.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_learners.log" 2>&1 || { echo "learner tests failed $?"; tail -60 "$OUT/pytest_learners.log"; exit 1; }
tail -3 "$OUT/pytest_learners.log"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed $?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
