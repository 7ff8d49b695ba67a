#!/bin/bash
# WD four rows a pass, LA shuffles by DPP: full GPU suite, smoke, rocprofv3
# kernel stats + PMC of the WD n=9000 workload (run.py's), default bench.
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r2bq > /dev/null || { tail -30 gpurun_out/r2bq/pytest.txt; exit 1; }
tail -n 1 gpurun_out/r2bq/pytest.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2bq/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r2bq/smoke.txt; exit 1; }
tail -n 1 gpurun_out/r2bq/smoke.txt
bash profiles/run_profiles_r02.sh r02bq wd_n9000 > gpurun_out/r2bq/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r2bq/prof.log; exit 1; }
tail -30 gpurun_out/r2bq/prof.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/r2bq/bench.json 2> gpurun_out/r2bq/bench.err || { echo "bench failed"; tail -30 gpurun_out/r2bq/bench.err; exit 1; }
cut -c1-300 gpurun_out/r2bq/bench.json
bash tools/gpu_r2ak.sh r2bq_la || { echo "la failed"; exit 1; }
cat gpurun_out/r2bq_la/la_time.json
