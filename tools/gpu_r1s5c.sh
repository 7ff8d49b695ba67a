#!/bin/bash
# r01 session 5c: PMC passes of the v8 mismatch kernel, full GPU suite, smoke, bench, rocprofv3 evidence.
set -u
TAG=${1:-r01s5c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/pmc_pass.sh ${TAG}_mm mm '[{}]' || { echo "pmc failed"; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "gpu tests failed $?"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed $?"; tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed $?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
bash profiles/run_profiles.sh "$TAG" || { echo "profiles failed $?"; exit 1; }
echo all done
