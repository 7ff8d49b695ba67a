#!/bin/bash
# Default bench.py on the box (+ optional rocprofv3 passes).  Usage: tools/gpu_bench.sh <tag> [prof]
set -u
TAG=${1:-bench}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ "${2:-}" = "prof" ]; then
  bash profiles/run_profiles.sh "$TAG" || { echo "profiles failed $?"; exit 1; }
fi
echo all done
