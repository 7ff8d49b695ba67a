#!/bin/bash
# Final round-2 check: full GPU suite, smoke(), default bench (driver form).
set -u
TAG=${1:-r2bg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$TAG" > /dev/null || { tail -30 $OUT/pytest.txt; exit 1; }
tail -n 1 $OUT/pytest.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.txt; exit 1; }
tail -n 1 $OUT/smoke.txt
start=$(date +%s)
timeout -k 10 500 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
cut -c1-600 $OUT/bench.json
