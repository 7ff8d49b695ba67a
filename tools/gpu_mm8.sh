#!/bin/bash
# mismatch slot kernels v7 vs v8: parity of the slot tests, then timings at N=20000 / 200000-slab.
set -u
OUT=gpurun_out/mm8${1:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_store.py -k "slots or mismatch_k9" -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "tests failed $?"; tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python3 -u tools/tune.py mm --reps 10 --sets '[{}, {"KMG_MM_SLOTV": "4"}, {"KMG_MM_SLOTV": "4", "KMG_MM_D": "3"}, {}, {"KMG_MM_SLOTV": "4"}]' > "$OUT/tune20k.jsonl" 2> "$OUT/tune20k.err" || { echo "tune failed $?"; tail -20 "$OUT/tune20k.err"; exit 1; }
cat "$OUT/tune20k.jsonl"
