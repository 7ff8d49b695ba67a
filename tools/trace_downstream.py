"""bench.py's downstream legs (NLCK combine, KRR / KLR / SVM solves on a symmetric K) without
the labelled asymmetric-K LU line, for a rocprofv3 kernel trace: every factorisation there
must be Cholesky (no rocSOLVER getf2 / getrf launches).
usage: rocprofv3 --kernel-trace --stats -d <dir> -o run -- python3 tools/trace_downstream.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kernel-methods-for-genomics_amd")]
import bench  # noqa: E402
from kmgram import _lib as L  # noqa: E402


def main():
    ctx = L.Context(0)
    try:
        out = bench.downstream(ctx, asym=False)
    finally:
        ctx.close()
    print(json.dumps({k: {kk: v[kk] for kk in ("ms", "factorisation") if kk in v}
                      for k, v in out.items()}))


if __name__ == "__main__":
    main()
