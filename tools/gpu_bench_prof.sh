#!/bin/bash
# Default bench (with the config-4/5 lines) + rocprofv3 evidence for the bench's kernels.
set -u
OUT=gpurun_out/r01s3e
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
bash profiles/run_profiles.sh r01s3 || { echo "profiles failed $?"; exit 1; }
echo all done
