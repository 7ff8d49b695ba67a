#!/bin/bash
# Collect the rocprofv3 evidence for bench.py on the GPU box (run from the repo root):
#   1. kernel trace + stats of the default bench command
#   2. separate PMC passes (FETCH_SIZE, then WRITE_SIZE) on the spectrum workload
# Usage: bash profiles/run_profiles.sh <tag>   (outputs under gpurun_out/prof_<tag>/)
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 10 --no-cpu --no-extra > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-mismatch --no-extra > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err" || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-mismatch --no-extra > "$OUT/bench_write.json" 2> "$OUT/write.err" || exit $?
echo done
