#!/bin/bash
# r01 session 5d: default bench + rocprofv3 evidence on the final tree of the session.
set -u
TAG=${1:-r01s5d}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
bash profiles/run_profiles.sh "$TAG" || { echo "profiles failed $?"; exit 1; }
echo all done
