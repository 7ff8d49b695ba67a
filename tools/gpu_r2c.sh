#!/bin/bash
# pair-table mismatch: parity tests, then timing of both formulations
set -u
OUT=gpurun_out/r02c
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -rf \
  --timeout 300 --timeout-method thread -p no:cacheprovider -k "mismatch" > "$OUT/pytest.txt" 2>&1
rc=$?
tail -15 "$OUT/pytest.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/time_mm.py '[{"KMG_MM_FORM":1},{"KMG_MM_FORM":2},{"KMG_MM_FORM":2,"norm":0},{"KMG_MM_FORM":1,"norm":0},{"KMG_MM_FORM":2,"n":200000,"rows":25000,"steps":2},{"KMG_MM_FORM":1,"n":200000,"rows":25000,"steps":2},{"KMG_MM_FORM":2,"k":10},{"KMG_MM_FORM":1,"k":10},{"KMG_MM_FORM":2,"k":8},{"KMG_MM_FORM":1,"k":8}]' > "$OUT/time.jsonl" 2>&1
rc=$?
cat "$OUT/time.jsonl"
exit $rc
