#!/bin/bash
# Round-2 re-entry check: full GPU suite then default bench.  Usage: tools/gpu_r2s.sh <tag>
set -u
TAG=${1:-r2s}
bash tools/gpu_tests.sh "$TAG" || exit 1
bash tools/gpu_bench.sh "$TAG" || exit 1
