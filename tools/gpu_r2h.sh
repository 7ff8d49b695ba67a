#!/bin/bash
set -u
mkdir -p gpurun_out/r2h
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "wd or goldens or pair or slabs" > gpurun_out/r2h/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r2h/pytest.txt; exit 1; }
tail -2 gpurun_out/r2h/pytest.txt
timeout -k 10 300 python3 -u tools/time_mm.py '[{"kind":"wd","n":9000,"d":4,"steps":10},{"kind":"wd","n":9000,"d":10,"steps":10},{"kind":"wd","n":9000,"d":4,"steps":10,"KMG_WD_FORM":1},{"kind":"wd","n":9000,"d":10,"steps":10,"KMG_WD_FORM":1},{"kind":"wd","n":9000,"d":5,"steps":10,"rows":4500}]' > gpurun_out/r2h/time.jsonl 2>&1 || { echo "time failed"; tail gpurun_out/r2h/time.jsonl; exit 1; }
cat gpurun_out/r2h/time.jsonl
