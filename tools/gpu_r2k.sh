#!/bin/bash
set -u
mkdir -p gpurun_out/r2k
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "mismatch" > gpurun_out/r2k/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r2k/pytest.txt; exit 1; }
tail -2 gpurun_out/r2k/pytest.txt
timeout -k 10 300 python3 -u tools/time_mm.py '[{"KMG_MM_FORM":1,"norm":0,"steps":5},{"KMG_MM_FORM":2,"norm":0,"steps":5},{"KMG_MM_FORM":1,"k":10,"norm":0,"steps":5},{"KMG_MM_FORM":2,"k":10,"norm":0,"steps":5},{"KMG_MM_FORM":1,"k":11,"norm":0,"steps":3},{"KMG_MM_FORM":2,"k":11,"norm":0,"steps":3}]' > gpurun_out/r2k/time.jsonl 2>&1 || { echo "time failed"; tail gpurun_out/r2k/time.jsonl; exit 1; }
cat gpurun_out/r2k/time.jsonl
