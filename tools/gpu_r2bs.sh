#!/bin/bash
# Final check of the tree: full GPU suite, smoke(), default bench (driver form).
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r2bs > /dev/null || { tail -30 gpurun_out/r2bs/pytest.txt; exit 1; }
tail -n 1 gpurun_out/r2bs/pytest.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2bs/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r2bs/smoke.txt; exit 1; }
tail -n 1 gpurun_out/r2bs/smoke.txt
start=$(date +%s)
timeout -k 10 500 python3 -u bench.py > gpurun_out/r2bs/bench.json 2> gpurun_out/r2bs/bench.err || { echo "bench failed"; tail -30 gpurun_out/r2bs/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - start )) s"
cut -c1-300 gpurun_out/r2bs/bench.json
