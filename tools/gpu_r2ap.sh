#!/bin/bash
# Chunk-major spectrum default: parity/config tests + config-4 profile with PMC.
set -u
TAG=${1:-r2ap}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_store.py -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
bash profiles/run_profiles_r02.sh "$TAG" config4 || { echo prof failed; exit 1; }
