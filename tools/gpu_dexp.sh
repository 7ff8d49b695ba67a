#!/bin/bash
set -u
mkdir -p gpurun_out/dexp
C='[{"kind":"sp","k":5,"n":20000,"steps":10,"check":false},{"kind":"sp","k":4,"n":20000,"steps":10,"check":false},{"kind":"mm","k":6,"n":20000,"steps":10,"check":false,"norm":0}]'
timeout -k 10 120 python3 tools/time_mm.py "$C" > gpurun_out/dexp/sk7.jsonl 2>&1 || exit 1
for e in 0 4 12; do
cp tools/exp/libkmgram_sk$e.so kernel-methods-for-genomics_amd/libkmgram.so
timeout -k 10 120 python3 tools/time_mm.py "$C" > gpurun_out/dexp/sk$e.jsonl 2>&1 || exit 1
done
for f in sk0 sk4 sk7 sk12; do echo $f; cat gpurun_out/dexp/$f.jsonl | cut -c1-60,120-200; done
