#!/bin/bash
# Run the GPU test suite on the box: one pytest process, per-test time limit, log under
# gpurun_out/<tag>/.  Usage: tools/gpu_tests.sh <tag> [pytest args...]
set -u
TAG=${1:-gpu}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  -p no:cacheprovider "$@" > "$OUT/pytest.txt" 2>&1
rc=$?
tail -40 "$OUT/pytest.txt"
exit $rc
