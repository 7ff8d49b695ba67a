#!/bin/bash
# full GPU suite, then spectrum / mismatch timings
set -u
TAG=${1:-r2v}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_tests.sh "$TAG" > /dev/null || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
timeout -k 10 300 python3 -u tools/time_mm.py '[{"kind":"sp","steps":20},{"kind":"sp","steps":20},{"kind":"mm","steps":5},{"kind":"mm","steps":5,"norm":0},{"kind":"mm","steps":5,"k":10},{"kind":"mm","steps":5,"KMG_MM_FORM":2}]' > "$OUT/time.jsonl" 2>&1 || { echo "time failed"; tail "$OUT/time.jsonl"; exit 1; }
cat "$OUT/time.jsonl"
