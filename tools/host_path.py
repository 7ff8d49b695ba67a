"""Time bench.host_path_config4 alone (GPU box): python3 tools/host_path.py [n] [slab_rows] [f64]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
slab = int(sys.argv[2]) if len(sys.argv) > 2 else 2500
f64 = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
ctx = bench.L.Context(0)
print(json.dumps(bench.host_path_config4(ctx, n, slab, f64)), flush=True)
ctx.close()
