#!/bin/bash
# Dense int8 MFMA Gram: super-block tile order (KMG_DENSE_SB) sweep + dense GPU tests.
set -u
TAG=${1:-r2ae}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_dense.py tests/test_gappy_intended.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 $OUT/pytest.txt
C='['
for SB in 1 2 4 8; do
  C="$C{\"kind\": \"sp\", \"k\": 5, \"steps\": 10, \"KMG_DENSE_SB\": $SB},"
  C="$C{\"kind\": \"sp\", \"k\": 4, \"steps\": 10, \"KMG_DENSE_SB\": $SB},"
  C="$C{\"kind\": \"sp\", \"k\": 5, \"n\": 9000, \"f64\": 1, \"steps\": 10, \"KMG_DENSE_SB\": $SB},"
  C="$C{\"kind\": \"mm\", \"k\": 6, \"norm\": 0, \"steps\": 10, \"check\": false, \"KMG_DENSE_SB\": $SB},"
done
C="$C{\"kind\": \"sp\", \"k\": 5, \"steps\": 10}]"
timeout -k 10 300 python3 -u tools/time_mm.py "$C" > "$OUT/sb.jsonl" 2>&1 || { echo "time failed"; tail $OUT/sb.jsonl; exit 1; }
cut -c1-200 $OUT/sb.jsonl
