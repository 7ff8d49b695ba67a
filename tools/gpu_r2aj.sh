#!/bin/bash
# Store / multi / configs GPU tests after kmg_gram_to_host.
set -u
TAG=${1:-r2aj}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_store.py tests/test_gpu_multi.py tests/test_abi_host.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
