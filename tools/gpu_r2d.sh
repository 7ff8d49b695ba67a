#!/bin/bash
# dense GEMM + pair-table mismatch: parity tests, then timings
set -u
OUT=gpurun_out/r02d
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dense.py tests/test_gpu_multi.py -m gpu -x -q -rf \
  --timeout 300 --timeout-method thread -p no:cacheprovider -k "mismatch or dense or blocks" > "$OUT/pytest.txt" 2>&1
rc=$?
tail -15 "$OUT/pytest.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/time_mm.py '[{"KMG_MM_FORM":1},{"KMG_MM_FORM":2},{"KMG_MM_FORM":2,"norm":0},{"KMG_MM_FORM":2,"n":200000,"rows":25000,"steps":2},{"KMG_MM_FORM":2,"k":10},{"kind":"sp","k":5,"KMG_ALGO":1,"check":false},{"kind":"sp","k":5,"KMG_ALGO":1,"n":9000,"f64":1},{"kind":"sp","k":4,"KMG_ALGO":1,"n":9000,"f64":1},{"kind":"mm","k":6,"KMG_ALGO":1,"n":9000},{"kind":"mm","k":5,"KMG_ALGO":1,"n":9000}]' > "$OUT/time.jsonl" 2>&1
rc=$?
cat "$OUT/time.jsonl"
exit $rc
