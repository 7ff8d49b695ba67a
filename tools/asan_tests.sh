#!/bin/bash
# Run tests against the host-AddressSanitizer build of libkmgram (make -C
# kernel-methods-for-genomics_amd/csrc asan): every host path of the C ABI instrumented,
# device code unchanged.  CPU here: the ABI host tests; on the GPU box pass a pytest -k
# expression to run GPU tests through the same library.
# usage: bash tools/asan_tests.sh [tag] [pytest -k expression (GPU box)]
set -u
TAG=${1:-asan}
EXPR=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n 1)
export KMGRAM_LIB=$PWD/kernel-methods-for-genomics_amd/libkmgram_asan.so
# leaks: the HIP runtime's own allocations at exit are not ours; device memory is not seen
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0
if [ -z "$EXPR" ]; then
  LD_PRELOAD=$RT timeout -k 10 600 python3 -m pytest tests/test_abi_host.py -q -p no:cacheprovider \
    > "$OUT/asan_host.txt" 2>&1
else
  LD_PRELOAD=$RT timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -k "$EXPR" -p no:cacheprovider \
    --timeout 300 --timeout-method thread > "$OUT/asan_gpu.txt" 2>&1
fi
rc=$?
tail -5 "$OUT"/asan_*.txt
grep -l "AddressSanitizer" "$OUT"/asan_*.txt && rc=1
exit $rc
