#!/bin/bash
# Full GPU suite, default bench, bench rocprof (trace + PMC) and config-4 / SP N=20000
# profiles.  Usage: tools/gpu_r2ba.sh <tag>
set -u
TAG=${1:-r2ba}
bash tools/gpu_tests.sh "$TAG" > /dev/null || { tail -30 gpurun_out/$TAG/pytest.txt; exit 1; }
tail -2 gpurun_out/$TAG/pytest.txt
bash tools/gpu_bench.sh "$TAG" > /dev/null || { echo bench failed; exit 1; }
cut -c1-900 gpurun_out/$TAG/bench.json
bash profiles/run_profiles.sh "$TAG" || { echo prof failed; exit 1; }
bash profiles/run_profiles_r02.sh "$TAG" sp_n20000 config4 dense_sp5 mm_n20000 wd_n9000 || { echo prof2 failed; exit 1; }
