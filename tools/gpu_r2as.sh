#!/bin/bash
# Bench with the config-4 headline + its rocprof evidence (trace + FETCH/WRITE passes).
set -u
TAG=${1:-r2as}
bash tools/gpu_bench.sh "$TAG" > /dev/null || { echo bench failed; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cut -c1-1500 gpurun_out/$TAG/bench.json
bash profiles/run_profiles.sh "$TAG" || { echo prof failed; exit 1; }
