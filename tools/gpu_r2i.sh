#!/bin/bash
set -u
mkdir -p gpurun_out/r2i
timeout -k 10 300 python3 -u tools/time_mm.py '[{"kind":"sp","k":8,"n":20000,"steps":20},{"kind":"sp","k":8,"n":20000,"steps":20},{"kind":"sp","k":8,"n":100000,"steps":5}]' > gpurun_out/r2i/time.jsonl 2>&1 || { echo "time failed"; tail gpurun_out/r2i/time.jsonl; exit 1; }
cat gpurun_out/r2i/time.jsonl
