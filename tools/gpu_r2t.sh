#!/bin/bash
# Spectrum kernel A/B: parity of variant 1, then timing sweep.  Usage: tools/gpu_r2t.sh <tag>
set -u
TAG=${1:-r2t}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
KMG_SP_VARIANT=21 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "spectrum or golden or config1 or index or slabs" > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.txt"; exit 1; }
KMG_SP_VARIANT=5 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "spectrum or golden or config1 or index or slabs" > "$OUT/pytest5.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest5.txt"; exit 1; }
timeout -k 10 300 python3 -u tools/time_mm.py '[{"kind": "sp", "steps": 20, "KMG_SP_VARIANT": 0}, {"kind": "sp", "steps": 20, "KMG_SP_VARIANT": 5}, {"kind": "sp", "steps": 20, "KMG_SP_VARIANT": 21}, {"kind": "sp", "steps": 20, "KMG_SP_VARIANT": 37}, {"kind": "sp", "steps": 10, "f64": 1, "KMG_SP_VARIANT": 0}, {"kind": "sp", "steps": 10, "f64": 1, "KMG_SP_VARIANT": 5}, {"kind": "sp", "steps": 10, "f64": 1, "KMG_SP_VARIANT": 21}, {"kind": "sp", "n": 100000, "steps": 4, "KMG_SP_VARIANT": 0}, {"kind": "sp", "n": 100000, "steps": 4, "KMG_SP_VARIANT": 1}, {"kind": "sp", "n": 100000, "steps": 4, "KMG_SP_VARIANT": 5}, {"kind": "sp", "n": 100000, "steps": 4, "KMG_SP_VARIANT": 21}, {"kind": "sp", "n": 100000, "steps": 4, "KMG_SP_VARIANT": 33}, {"kind": "sp", "n": 9000, "k": 6, "f64": 1, "steps": 20, "KMG_SP_VARIANT": 0}, {"kind": "sp", "n": 9000, "k": 6, "f64": 1, "steps": 20, "KMG_SP_VARIANT": 5}]' > "$OUT/time.jsonl" 2>&1 || { echo "time failed"; tail "$OUT/time.jsonl"; exit 1; }
cat "$OUT/time.jsonl"
