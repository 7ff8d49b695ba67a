#!/bin/bash
# Dense Gram with LDS-DMA staging as the only path: full GPU suite, smoke, then rocprofv3
# kernel stats + PMC of the dense SP k=5 workload and the WD n=9000 workload (run.py's).
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r2bl > /dev/null || { tail -30 gpurun_out/r2bl/pytest.txt; exit 1; }
tail -n 1 gpurun_out/r2bl/pytest.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2bl/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r2bl/smoke.txt; exit 1; }
tail -n 1 gpurun_out/r2bl/smoke.txt
bash profiles/run_profiles_r02.sh r02bl dense_sp5 > gpurun_out/r2bl/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r2bl/prof.log; exit 1; }
tail -30 gpurun_out/r2bl/prof.log
