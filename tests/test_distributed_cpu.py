"""World-size-2 gloo tests of the multi-rank host logic on CPU (no GPU):
row sharding covers every row exactly once, the weak-scaled N keeps per-rank work
constant, and the bench's barrier / max-over-ranks protocol works."""
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT
from kmgram.shard import even_splits, rank_rows, weak_scaled_n


@pytest.mark.parametrize("n,parts", [(0, 1), (7, 2), (20000, 8), (56568, 8), (5, 8)])
def test_even_splits_cover(n, parts):
    s = even_splits(n, parts)
    assert s[0] == 0 and s[-1] == n and all(a <= b for a, b in zip(s, s[1:]))
    sizes = [b - a for a, b in zip(s, s[1:])]
    assert max(sizes) - min(sizes) <= 1


def test_weak_scaling_pairs_per_rank():
    for world in (1, 2, 4, 8):
        n = weak_scaled_n(20000, world)
        per_rank = n * n / world
        assert abs(per_rank / 20000 ** 2 - 1) < 1e-3
        assert n % 8 == 0


WORKER = r"""
import os, sys, json
sys.path.insert(0, os.path.join(os.environ["ROOT"], "kernel-methods-for-genomics_amd"))
import torch, torch.distributed as dist
from kmgram.shard import rank_rows, weak_scaled_n
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
n = weak_scaled_n(20000, w)
a, b = rank_rows(n, w, r)
t = torch.tensor([float(b - a)], dtype=torch.float64)
dist.all_reduce(t, op=dist.ReduceOp.SUM)
mx = torch.tensor([float(r + 1)], dtype=torch.float64)
dist.all_reduce(mx, op=dist.ReduceOp.MAX)
dist.barrier()
obj = [b"uid-bytes" if r == 0 else None]
dist.broadcast_object_list(obj, src=0)
if r == 0:
    print(json.dumps({"rows": t.item(), "n": n, "max": mx.item(), "obj": obj[0].decode()}))
dist.destroy_process_group()
"""


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_protocol(tmp_path):
    pytest.importorskip("torch")
    script = tmp_path / "w.py"
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), str(script)]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    import json
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["rows"] == d["n"] == weak_scaled_n(20000, 2)
    assert d["max"] == 2.0 and d["obj"] == "uid-bytes"
