#!/bin/bash
# Dense Gram, LDS-DMA staging + swizzled epilogue tile: full GPU suite, smoke, rocprofv3
# kernel stats + PMC of the dense SP k=5 workload and the WD n=9000 workload (run.py's).
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r2bn > /dev/null || { tail -30 gpurun_out/r2bn/pytest.txt; exit 1; }
tail -n 1 gpurun_out/r2bn/pytest.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2bn/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r2bn/smoke.txt; exit 1; }
tail -n 1 gpurun_out/r2bn/smoke.txt
bash profiles/run_profiles_r02.sh r02bn dense_sp5 > gpurun_out/r2bn/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r2bn/prof.log; exit 1; }
tail -30 gpurun_out/r2bn/prof.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/r2bn/bench.json 2> gpurun_out/r2bn/bench.err || { echo "bench failed"; tail -30 gpurun_out/r2bn/bench.err; exit 1; }
cut -c1-300 gpurun_out/r2bn/bench.json
