#!/usr/bin/env python3
"""bench.py — Gram pairs/s of the MI355X string-kernel Gram engine.

Workload (BASELINE.json configs[3], the north_star's target: "≥100× the reference CPU Gram
build at N=100k, L=101, spectrum k=8 on one MI355X"): spectrum k=8 Gram of N=100000
synthetic DNA sequences of length L=101, int32 exact counts (40 GB), device-resident (input
codes already in HBM when the timed region starts); posting-list formulation (DESIGN.md §4
on the configs[3] "count-vector GEMM" wording).  A "step" is one full-K build (SURVEY §8d t_build):
2-bit packing + posting-index build + Gram kernel (G > 1: this GPU's rows of it).

Multi-GPU: one process per GPU.  `python bench.py --gpus G` starts the G rank processes
itself (launch_ranks: rank r on device r, rendezvous on 127.0.0.1, rank 0's JSON line
relayed, non-zero exit if any rank fails); under `python -m torch.distributed.run
--nproc-per-node G bench.py --gpus G` the launcher's environment is used as is, and a
WORLD_SIZE different from --gpus is an error.  The rows of K are independent and K is
symmetric, so the headline shards K with no data-path collective and scales
STRONGLY at the north-star's named N = 100000: every GPU computes its 1/G share -- at
G = 2 its rows x all N columns (the replicated index), at G >= 4 all N rows x its columns
as one column chunk (the index over its own sequences; share_mode: the faster shape
there, the other one reported as `other_share`) -- in its own buffer; `value` = N^2 /
max-over-ranks step time.  At G = 1 the G = 2 / 4 / 8 shares are also timed on the one GPU
(`shares_measured`: a collective-free rank's time is the job's).  The
north-star's final RCCL all-gather is measured beside it at the same N (`assembled`:
upper-triangle uint8 round slabs all-gathered in place over RCCL/xGMI on a second stream
while the next round is computed, every GPU unpacking / mirroring them into the whole K),
and the weak-scaled build (N = 100000 sqrt(G), every GPU 1e10 pairs) as `weak_scaled`.

Also reported: the mismatch (k=9, m=1) Gram at N=20000 (BASELINE configs[2], float64
normalised), per-stage device times from HIP events, the HBM roofline of the dominant
kernel, the oracle timed on the host cores (cpu_baseline), and (N=1) BASELINE configs[1]
(N=20000 spectrum) and [4], the drop-in host path, run.py's nine kernels at N=9000 and the downstream
consumers.  At G > 1 the config[4] strong-scaling line (N=200000, raw int32 K gathered)
is added.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kernel-methods-for-genomics_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

from kmgram import _lib as L  # noqa: E402
from kmgram import encode as E  # noqa: E402
from kmgram import params as P  # noqa: E402
from kmgram.shard import (block_cyclic_ranges, default_block, rank_rows,  # noqa: E402
                          rows_padded, scaling_projection, triangle_rounds, weak_scaled_n)

HBM_PEAK = 8.0e12  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
GATHER_MODE = 2  # G > 1: upper-triangle round slabs + local mirror (--gather-mode 1: full rows)
XGMI_IN_PEAK = 7 * 76.5e9  # per-GPU ingress: 7 xGMI links x ~76.5 GB/s per direction
GATHER_CEILING = 56.38e9  # random 128-B lines/s from a 78.6 MB table (profiles/r02_mall_gather.jsonl)
INT8_PEAK = 5.0e15  # dense int8 MFMA (2x the ~2.5 PF dense bf16, MI355X_MICROARCH.md)
METRIC = ("Gram pairs/sec (N×N) + full-K build time, spectrum k=8 and mismatch "
          "(k=9,m=1), 1/2/4/8 GPUs")
STAGES = ("count", "scan", "place", "fine", "pack", "lists", "nbfill", "slots", "extract", "features", "diag",
          "gram", "mirror", "gather")


def rank_env(base, world, rank, port, addr="127.0.0.1"):
    """The environment of rank `rank` of a `world`-rank job started by launch_ranks: the
    variables torch.distributed.run sets (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
    MASTER_ADDR / MASTER_PORT; one node, so the local rank is the rank and picks the GPU),
    plus KMG_BENCH_LAUNCHED so a child never launches again."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", MASTER_ADDR=addr,
               MASTER_PORT=str(port), KMG_BENCH_LAUNCHED="1")
    return env


def free_port(addr="127.0.0.1"):
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def launch_ranks(world, argv, poll_s=0.5):
    """`bench.py --gpus G` started without a launcher (WORLD_SIZE unset): start G rank
    processes of this script (one per GPU, rank r on device r) and relay rank 0's JSON line.
    Runs before this process loads libkmgram or makes any HIP call; the children are
    started as new processes (never an exec of this one).  If a rank fails, the others are
    terminated (their own PIDs) and the exit status is non-zero.  Returns the exit status."""
    import subprocess
    port = int(os.environ.get("MASTER_PORT") or free_port())
    addr = os.environ.get("MASTER_ADDR") or "127.0.0.1"
    cmd = [sys.executable, os.path.abspath(__file__)] + list(argv)
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen(cmd, env=rank_env(os.environ, world, r, port, addr),
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
    status = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"launch_ranks: rank {r} exited with status {c}; stopping the others",
                      file=sys.stderr)
                status = c if c > 0 else 128 - c
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out = procs[0].stdout.read().decode(errors="replace")
    procs[0].stdout.close()
    lines = [ln for ln in out.splitlines() if ln.strip()]
    if status == 0:
        if not lines:
            print("launch_ranks: rank 0 printed no JSON line", file=sys.stderr)
            return 1
        rec = json.loads(lines[-1])
        if rec.get("n_gpus") != world:
            print(f"launch_ranks: rank 0 reports n_gpus={rec.get('n_gpus')}, not {world}",
                  file=sys.stderr)
            return 1
        print(lines[-1], flush=True)
    return status


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")  # host barrier / max / uid broadcast only
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v):
        if self.world == 1:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def all_true(self, v):
        return self.max(0.0 if v else 1.0) == 0.0

    def gather(self, v):
        """[v of rank 0, v of rank 1, ...] on every rank."""
        if self.world == 1:
            return [v]
        out = [None] * self.world
        self.dist.all_gather_object(out, v)
        return out

    def bcast_bytes(self, b):
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def stage_means(ctx):
    out = {}
    for st in STAGES:
        tot, cnt = ctx.stage_stats(st)
        if cnt:
            out[st] = round(tot / cnt, 5)
            if st in ("gram", "gather", "mirror"):
                out[st + "_launches"] = cnt
                out[st + "_total"] = round(tot, 5)
    return out


def run_build(ctx, dist, name, params, out_dtype, n, seed, steps, warmup, check_row,
              gather=None):
    """Timed full-K builds of one workload: kmg_gram_blocks over this rank's block-cyclic
    rows; gather (default: GATHER_MODE when G > 1) all-gathers them in place over RCCL,
    0 keeps every rank to its own rows (no data-path collective).  Returns timings, stages
    and a spot check."""
    codes, lens = E.synthetic(n, 101, seed=seed)
    ldc = codes.shape[1]
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    world, rank = dist.world, dist.rank
    if gather is None:
        gather = GATHER_MODE if world > 1 else 0
    # collective-free: one block a rank (one Gram launch per step); assembled: rounds of
    # ~256 MB, so each round's all-gather overlaps the next round's Gram
    block = (n if world == 1 else
             default_block(n, world, n * esz) if gather else (-(-n // world) + 7) // 8 * 8)
    npad = rows_padded(n, world, block)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    # collective-free at G > 1: this rank's blocks packed in its own buffer (gather 4; a rank
    # share of the weak-scaled K, which no one GPU could hold); else the whole padded K
    mine = block_cyclic_ranges(n, world, rank, block)
    packed = gather == 0 and world > 1
    d_out = ctx.dmalloc((len(mine) * block if packed else npad) * n * esz)
    res = {"name": name, "N": n, "block_rows": block, "rounds": npad // (world * block),
           "gather_mode": gather,
           "rows_this_rank": sum(b - a for a, b in block_cyclic_ranges(n, world, rank, block))}
    try:
        def step(g):
            ctx.gram_blocks(params, d_codes, d_lens, n, ldc, out_dtype, d_out, n, world, rank,
                            block, 4 if (g == 0 and world > 1) else g)

        def timed(g, k):
            for _ in range(warmup):
                step(g)
            ctx.synchronize()
            # timed region: HIP events around the Gram launches (and gathers) only, two per
            # launch; events around every index stage add ~20 us of bubbles per build
            ctx.set_timing(2)
            ctx.timing_reset()
            dist.barrier()
            ctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                step(g)
            ctx.synchronize()
            dist.barrier()
            wall = dist.max(time.perf_counter() - t0)
            kern = stage_means(ctx)
            # per-stage breakdown (index build etc.) from a separate, untimed pass
            ctx.set_timing(True)
            ctx.timing_reset()
            for _ in range(min(k, 5)):
                step(g)
            ctx.synchronize()
            stages = stage_means(ctx)
            ctx.set_timing(False)
            stages.update(kern)
            return wall / k, stages

        t, stages = timed(gather, steps)
        res.update({"ms_per_step": t * 1e3, "pairs_per_s": n * n / t, "stages_ms": stages,
                    "wire_bytes": ctx.blocks_wire(), "plan": ctx.last_plan()})
        if gather:
            tcf, scf = timed(0, steps)
            res["collective_free"] = {"ms_per_step": tcf * 1e3, "pairs_per_s": n * n / tcf,
                                      "stages_ms": scf}
            alt = 1 if gather == 2 else 2  # the other assembly, for comparison
            ta, sa = timed(alt, steps)
            res["other_gather_mode"] = {"gather_mode": alt, "ms_per_step": ta * 1e3,
                                        "pairs_per_s": n * n / ta, "stages_ms": sa}
            step(gather)  # leave the gathered K for the spot check
            ctx.synchronize()
        # spot check: the first row of this rank's first block, plus (G > 1) a row computed
        # by the next rank and received through the all-gather
        rows = [mine[0][0], mine[0][1] - 1]
        ch = (res.get("plan") or {}).get("chunk") or 0
        if world == 1 and 0 < ch < n:  # a row at a column-chunk edge (its diagonal entry
            rows += [ch - 1, ch]          # on either side of the edge)
        if gather:
            rows.append(block_cyclic_ranges(n, world, (rank + 1) % world, block)[0][0])
        rows = sorted(set(rows))
        ok = True
        for r in rows:
            row = np.empty(n, dtype=L.DTYPES[out_dtype])
            orow = r - mine[0][0] if packed else r  # (packed: the rank's first block at row 0)
            ctx.d2h(row, ctypes.c_void_p(d_out.value + orow * n * esz))
            ok &= check_row(codes, lens, r, row)
        res["spot_check_rows"] = rows
        res["spot_check"] = dist.all_true(ok)
        if name == "spectrum_k8" and world == 1:
            res["write_ceiling_GBps"] = write_ceiling(ctx, d_out, n * n * esz)
    finally:
        ctx.dfree(d_out)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    return res


def check_spectrum(codes, lens, r, row):
    import cref
    return bool(np.array_equal(row.astype(np.int64), cref.spectrum(codes, lens, 8, rows=(r, r + 1))[0]))


def check_mismatch(codes, lens, r, row):
    import cref
    return bool(np.array_equal(row, cref.mismatch_rows(codes, lens, 9, 1, rows=(r, r + 1))[0]))


def check_mismatch_raw(codes, lens, r, row):
    import cref
    return bool(np.array_equal(row.astype(np.int64),
                               cref.mismatch_raw(codes, lens, 9, 1, rows=(r, r + 1))[0]))


def write_ceiling(ctx, d_out, nbytes, reps=10):
    """hipMemsetAsync over the same K buffer (context stream, HIP events) -> GB/s: the
    runtime fill's rate on this box, reported as `memset_GBps` beside the 8 TB/s spec peak
    (not a ceiling: the spectrum Gram kernel's 16-byte row stores run above it)."""
    ctx.memset(d_out, 0, nbytes)
    ctx.synchronize()
    ctx.set_timing(True)
    ctx.timing_reset()
    for _ in range(reps):
        ctx.memset(d_out, 0, nbytes)
    ctx.synchronize()
    tot, cnt = ctx.stage_stats("memset")
    ctx.set_timing(False)
    return nbytes / (tot / cnt / 1e3) / 1e9 if cnt else None


# ----------------------------------------------------------------------- CPU baseline
_F = _FT = None


def _rows_product(ab):
    """Rows [a, b) of Phi Phi^T as dense float64 rows (what the reference materialises), in
    sub-blocks of 256 rows so a worker holds at most 256 x N doubles (0.2 GB at N=100000)."""
    a, b = ab
    t0 = time.perf_counter()
    for s in range(a, b, 256):
        (_F[s:min(b, s + 256)] @ _FT).toarray()
    return time.perf_counter() - t0


def host_cpus():
    """The host cores this process may use: os.cpu_count() (the whole machine), the
    scheduler affinity mask and the cgroup CPU quota (cgroup v2 cpu.max or v1
    cfs_quota_us / cfs_period_us), plus the CPU model.  workers = the smallest of them (a
    GPU box's CPU share is a cgroup quota below the machine's core count: more processes
    than the quota only time-slice); KMG_BENCH_CPU_WORKERS overrides."""
    info = {"host_cores": os.cpu_count()}
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            q = float(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = float(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    info["cgroup_cpu_quota"] = quota
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    info["cpu_model"] = model
    w = info["affinity_cpus"] or 1
    if quota:
        w = min(w, max(1, int(quota)))
    env = os.environ.get("KMG_BENCH_CPU_WORKERS")
    info["workers"] = int(env) if env else w
    info["workers_rule"] = ("KMG_BENCH_CPU_WORKERS" if env else
                            "min(affinity CPUs, cgroup CPU quota)" if quota else "affinity CPUs")
    return info


def cpu_baseline(name, n, budget_s, seed, workers=None):
    """The strongest CPU restatement of the reference we have, on this box's host cores:
    scipy-sparse Phi Phi^T (oracle/cpu_ref.py spectrum_phi / mismatch_phi = the reference's
    own feature maps get_phi_u / get_phi_km, kernels.py:12-25, 161-175, and its np.dot pair
    loop, kernels.py:41-45, 211-215, as one sparse product).  Phi is built once for all N
    (timed); the product runs over a bounded row sample split across `workers` forked
    processes (one row block each, Phi shared copy-on-write), and the whole job is
    extrapolated as t_phi + (N / rows) * t_rows.  Also returns the 1-process figure."""
    import multiprocessing as mp
    import cpu_ref
    global _F, _FT
    hw = host_cpus()
    workers = workers or hw["workers"]
    codes, lens = E.synthetic(n, 101, seed=seed)  # the timed workload's own input
    t0 = time.perf_counter()
    _F = (cpu_ref.spectrum_phi(codes, lens, 8) if name == "spectrum_k8"
          else cpu_ref.mismatch_phi(codes, lens, 9, 1))
    _FT = _F.T.tocsr()
    t_phi = time.perf_counter() - t0
    # 1 process: size the sample to ~budget/4
    r = 16
    while True:
        t = _rows_product((0, r))
        if t >= budget_s / 8 or r >= n:
            break
        r = min(n, max(r * 2, int(r * (budget_s / 8) / max(t, 1e-3))))
    rate1 = r / t  # rows per second, one process
    # all workers: each takes a block sized for ~budget/2 of wall time
    per = max(1, min(n // workers, int(rate1 * budget_s / 2)))
    blocks = [(w * per, (w + 1) * per) for w in range(workers) if (w + 1) * per <= n]
    # forked before this process makes any HIP call (main() runs the CPU baseline first),
    # and ended by close() + join(): the workers exit on their own, nobody is SIGTERMed
    ctx_mp = mp.get_context("fork")
    t0 = time.perf_counter()
    pool = ctx_mp.Pool(len(blocks))
    try:
        pool.map(_rows_product, blocks)
    finally:
        pool.close()
        pool.join()
    t_rows = time.perf_counter() - t0
    rows = per * len(blocks)
    t_job = t_phi + (n / rows) * t_rows
    t_job1 = t_phi + n / rate1
    _F = _FT = None
    label = "spectrum_phi" if name == "spectrum_k8" else "mismatch_phi"
    return {"value": n * n / t_job, "unit": "Gram pairs/s", "cores": len(blocks), "kind": "port",
            "host_cores": hw["host_cores"], "cpu_model": hw["cpu_model"],
            "affinity_cpus": hw["affinity_cpus"], "cgroup_cpu_quota": hw["cgroup_cpu_quota"],
            "workers": len(blocks), "workers_rule": hw["workers_rule"],
            "sample": f"scipy-sparse Phi Phi^T (oracle/cpu_ref.py {label}): Phi of all {n} "
                      f"sequences {t_phi:.2f} s (1 process) + rows 0..{rows} x {n} over "
                      f"{len(blocks)} forked processes in {t_rows:.2f} s wall, whole job "
                      + (f"{t_job:.1f} s (every row computed)" if rows >= n else
                         f"extrapolated to {t_job:.1f} s"),
            "one_process": {"value": n * n / t_job1, "cores": 1,
                            "sample": f"{r} rows in {t:.2f} s, whole job {t_job1:.1f} s"}}


# reference kernels.py cost model (measured in the survey container: 8-core
# Xeon, numpy/OpenBLAS; not this box): seconds for the whole Gram build
def reference_model_s(kind, n):
    if kind == "spectrum_k8":
        return 1.10 * n + 10.0e-6 * n * (n + 1) / 2
    return 78.0 * n + 35e-6 * n * (n + 1) / 2 + 0.46e-6 * n * n / 2


# ----------------------------------------------------------------------- N = 1 extras
def run_slab(ctx, params, out_dtype, n, seed, r0, r1, steps, warmup, spot_rows, oracle_row,
             cols=None, timing=True):
    """One workload on rows [r0, r1) x all n columns, device-resident, one launch set;
    cols = (c0, c1): instead the column block K[:, c0:c1] of every row (kmg_gram_device_cols;
    the same pairs as rows [c0, c1) x all n, K being symmetric), spot rows checked on it."""
    codes, lens = E.synthetic(n, 101, seed=seed)
    ldc = codes.shape[1]
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    width = n if cols is None else cols[1] - cols[0]
    nrows = (r1 - r0) if cols is None else n
    d_out = ctx.dmalloc(nrows * width * esz)
    try:
        def step():
            if cols is None:
                ctx.gram_device(params, d_codes, d_lens, n, ldc, r0, r1, out_dtype, d_out, n)
            else:
                ctx.gram_device_cols(params, d_codes, d_lens, n, ldc, cols[0], cols[1], out_dtype,
                                     d_out, width)

        for _ in range(warmup):
            step()
        ctx.synchronize()
        ctx.set_timing(timing)  # (2: events around the Gram launches only)
        ctx.timing_reset()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ctx.synchronize()
        wall = time.perf_counter() - t0
        ctx.set_timing(False)
        stages = stage_means(ctx)
        if "mirror_total" in stages:  # (the mirror runs as one launch per row chunk)
            stages["mirror_per_build"] = round(stages["mirror_total"] / steps, 5)
        plan = ctx.last_plan()
        ok = True
        for r in spot_rows:
            row = np.empty(width, dtype=L.DTYPES[out_dtype])
            ctx.d2h(row, ctypes.c_void_p(d_out.value + (r - (r0 if cols is None else 0)) * width * esz))
            ref = oracle_row(codes, lens, r)
            if cols is not None:
                ref = ref[cols[0]:cols[1]]
            ok &= bool(np.array_equal(row.astype(ref.dtype), ref))
    finally:
        ctx.dfree(d_out)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    ms = wall / steps * 1e3
    out = {"N": n, "rows": nrows, "steps": steps, "ms_per_step": ms,
           "pairs_per_s": nrows * width / (ms / 1e3), "stages_ms": stages, "plan": plan,
           "spot_check_rows": list(spot_rows), "spot_check": ok}
    if cols is not None:
        out["cols"] = list(cols)
    return out


def run_colblock_dist(ctx, dist, params, out_dtype, n, seed, steps, warmup, oracle_row):
    """G > 1, collective-free: rank r computes the column block K[:, C_r] of all n rows,
    C_r = rank_rows(n, G, r) (kmg_gram_device_cols: the lists over the rank's own columns,
    packed).  Timed like run_build: barrier + synchronise on both sides, max over ranks."""
    codes, lens = E.synthetic(n, 101, seed=seed)
    ldc = codes.shape[1]
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    c0, c1 = rank_rows(n, dist.world, dist.rank)
    w = c1 - c0
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    d_out = ctx.dmalloc(n * w * esz)
    try:
        def step():
            ctx.gram_device_cols(params, d_codes, d_lens, n, ldc, c0, c1, out_dtype, d_out, w)

        for _ in range(warmup):
            step()
        ctx.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ctx.synchronize()
        dist.barrier()
        t = dist.max(time.perf_counter() - t0)
        plan = ctx.last_plan()
        ok = True
        for r in (0, n - 1):
            row = np.empty(w, dtype=L.DTYPES[out_dtype])
            ctx.d2h(row, ctypes.c_void_p(d_out.value + r * w * esz))
            ref = oracle_row(codes, lens, r)[c0:c1]
            ok &= bool(np.array_equal(row.astype(ref.dtype), ref))
        ok = dist.all_true(ok)
    finally:
        ctx.dfree(d_out)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    ms = t / steps * 1e3
    return {"N": n, "cols_this_rank": w, "steps": steps, "ms_per_step": ms,
            "pairs_per_s": n * n / (ms / 1e3), "plan": plan, "spot_check": ok}


# widest spectrum share taken as a column block: the library makes a block this wide or
# narrower one column chunk (kmg_api.cpp Tuning::sp_cb_chunk), the fastest share shape
# measured at G >= 4 (N=100000: G=4 1.73 vs 1.81-1.85 ms, G=8 0.95-0.97 vs 1.02-1.06 ms as
# row shares; at G=2 the 50000-row share is faster; profiles/r06k_*)
SP_COLSHARE_MAX = 32768


def share_mode(n, world):
    """The headline's per-rank share at G ranks: "cols" (K[:, C_r], one column chunk) when
    the rank's columns fit one chunk, else "rows" (K[R_r, :])."""
    return "cols" if world > 1 and -(-n // world) <= SP_COLSHARE_MAX else "rows"


def run_colshare(ctx, dist, name, params, out_dtype, n, seed, steps, warmup, oracle_row,
                 world=None, rank=None):
    """Timed column-block shares (kmg_gram_device_cols): rank r computes K[:, C_r] of all n
    rows, C_r = rank_rows(n, G, r) -- by symmetry the row share K[C_r, :], column-major.
    world / rank given: that rank's share of a G-rank job timed on this one GPU (the
    collective-free build has no exchange, so its per-rank time is the job's).  Timed like
    run_build: HIP events around the Gram launch, barrier + synchronise on both sides, the
    max over ranks; spot rows against the oracle (first, last, the block's own diagonal)."""
    codes, lens = E.synthetic(n, 101, seed=seed)
    ldc = codes.shape[1]
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    world = dist.world if world is None else world
    rank = dist.rank if rank is None else rank
    c0, c1 = rank_rows(n, world, rank)
    w = c1 - c0
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    d_out = ctx.dmalloc(max(1, n * w * esz))
    res = {"name": name, "N": n, "share": "cols", "world": world, "rank": rank,
           "cols_this_rank": w, "col_range": [c0, c1]}
    try:
        def step():
            ctx.gram_device_cols(params, d_codes, d_lens, n, ldc, c0, c1, out_dtype, d_out, w)

        for _ in range(warmup):
            step()
        ctx.synchronize()
        ctx.set_timing(2)
        ctx.timing_reset()
        dist.barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ctx.synchronize()
        dist.barrier()
        t = dist.max(time.perf_counter() - t0) / steps
        kern = stage_means(ctx)
        ctx.set_timing(True)
        ctx.timing_reset()
        for _ in range(min(steps, 5)):
            step()
        ctx.synchronize()
        stages = stage_means(ctx)
        ctx.set_timing(False)
        stages.update(kern)
        res.update({"ms_per_step": t * 1e3, "pairs_per_s": n * n / t, "stages_ms": stages,
                    "plan": ctx.last_plan()})
        rows = sorted({0, n - 1, c0, c1 - 1})
        ok = True
        for r in rows:
            row = np.empty(w, dtype=L.DTYPES[out_dtype])
            ctx.d2h(row, ctypes.c_void_p(d_out.value + r * w * esz))
            ref = oracle_row(codes, lens, r)[c0:c1]
            ok &= bool(np.array_equal(row.astype(ref.dtype), ref))
        res["spot_check_rows"] = rows
        res["spot_check"] = dist.all_true(ok)
    finally:
        ctx.dfree(d_out)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    return res


def measured_shares(ctx, dist, n, seed, steps, warmup, full_ms):
    """The headline's G = 2 / 4 / 8 per-rank shares timed on this one GPU (rank 0's, in the
    shape share_mode picks): the collective-free G-rank build exchanges nothing, so a rank's
    time is the job's, and full / share is its strong-scaling speedup -- measured, not
    modelled (each GPU of a node at its own clocks and HBM)."""
    out = {}
    params = P.make(L.KMG_SPECTRUM, k=8)
    for g in (2, 4, 8):
        mode = share_mode(n, g)
        if mode == "cols":
            r = run_colshare(ctx, dist, "spectrum_k8", params, L.KMG_I32, n, seed, steps, warmup,
                             spectrum_row, world=g, rank=0)
            width = r["cols_this_rank"]
        else:
            block = (-(-n // g) + 7) // 8 * 8
            r = run_slab(ctx, params, L.KMG_I32, n, seed, 0, block, steps, warmup, (0, block - 1),
                         spectrum_row, timing=2)
            width = block
        out[str(g)] = {"share": mode, "rows_or_cols": width, "ms": r["ms_per_step"],
                       "gram_ms": r["stages_ms"].get("gram"), "speedup": full_ms / r["ms_per_step"],
                       "spot_check": r["spot_check"]}
    return out


def sp_kernel_name(plan):
    """The gram_sp_kernel instance a spectrum build at this plan launches (int32 K, L=101:
    packed 16-bit accumulators; plain stores for one column chunk; two rows a workgroup at
    chunks <= 16384 columns, launch_gram_spectrum)."""
    ch, nch = plan.get("chunk") or 0, plan.get("nchunks") or 1
    return "kmg::gram_sp_kernel<true,1,%s,%d>" % ("false" if nch == 1 else "true",
                                                  2 if 0 < ch <= 16384 else 1)


def spectrum_row(codes, lens, r):
    import cref
    return cref.spectrum(codes, lens, 8, rows=(r, r + 1))[0].astype(np.int64)


def run_colblock_assembly(ctx, dist, params, out_dtype, n, seed, steps, warmup, oracle_row,
                          world=None):
    """Config 5 assembled from column blocks (kmg_gram_blocks gather 5): each rank
    its column block K[:, C_r] (lists over its own n/G sequences, packed), transposed into
    its row slab, then one in-place RCCL all-gather -- K on every GPU.  world (with
    dist.world == 1): the one-GPU rehearsal (gather 6) of a `world`-rank job, every rank's
    block computed here: its Gram / transpose stage times are what the projection uses.
    Timed like run_build: barrier + synchronise on both sides, max over ranks."""
    rehearsal = world is not None
    world = world if rehearsal else dist.world
    codes, lens = E.synthetic(n, 101, seed=seed)
    ldc = codes.shape[1]
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    block = -(-n // world)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    d_out = ctx.dmalloc(world * block * n * esz)
    gather = 6 if rehearsal else 5
    try:
        def step():
            ctx.gram_blocks(params, d_codes, d_lens, n, ldc, out_dtype, d_out, n, world,
                            0 if rehearsal else dist.rank, block, gather)

        for _ in range(warmup):
            step()
        ctx.synchronize()
        ctx.set_timing(2)
        ctx.timing_reset()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ctx.synchronize()
        dist.barrier()
        t = dist.max(time.perf_counter() - t0) / steps
        stages = stage_means(ctx)
        unpack_tot, unpack_cnt = ctx.stage_stats("unpack")
        ctx.set_timing(False)
        plan = ctx.last_plan()
        # spot rows: the first row of rank 0's and of the last rank's slab, and the last row
        # (each received through the all-gather on every other rank)
        rows = sorted({0, (world - 1) * block, n - 1})
        ok = True
        for r in rows:
            row = np.empty(n, dtype=L.DTYPES[out_dtype])
            ctx.d2h(row, ctypes.c_void_p(d_out.value + r * n * esz))
            ref = oracle_row(codes, lens, r)
            ok &= bool(np.array_equal(row.astype(ref.dtype), ref))
        ok = dist.all_true(ok)
    finally:
        ctx.dfree(d_out)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    out = {"N": n, "world": world, "block": block, "gather_mode": gather, "steps": steps,
           "ms_per_step": t * 1e3, "pairs_per_s": n * n / t, "stages_ms": stages,
           "transpose_ms_per_step": unpack_tot / steps, "transposes_per_step": unpack_cnt / steps,
           "plan": plan, "spot_check_rows": rows, "spot_check": ok}
    if rehearsal:
        out["per_rank_ms_model"] = t * 1e3 / world
    return out


def extras(ctx, cpu_rates, steps4):
    """BASELINE configs[3] and [4], the drop-in host path, run.py's kernels, downstream."""
    import cref
    out = {}
    sp = lambda c, l, r: cref.spectrum(c, l, 8, rows=(r, r + 1))[0]  # noqa: E731
    mmr = lambda c, l, r: cref.mismatch_raw(c, l, 9, 1, rows=(r, r + 1))[0]  # noqa: E731
    mm = lambda c, l, r: cref.mismatch_rows(c, l, 9, 1, rows=(r, r + 1))[0]  # noqa: E731
    n2 = 20000
    c2 = run_slab(ctx, P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32, n2, 2, 0, n2, steps4, 3,
                  (0, 12345, n2 - 1), sp)
    c2["workload"] = ("BASELINE configs[1]: spectrum k=8, N=20000 x L=101, full K on 1 GPU, "
                      "int32 (1.6 GB), bit-exact spot rows")
    c2["gram_hbm_frac"] = (4.0 * n2 * n2 + 52.0 * n2) / (c2["stages_ms"]["gram"] / 1e3) / HBM_PEAK
    c2["reference_model_s"] = reference_model_s("spectrum_k8", n2)
    c2["speedup_vs_reference_model"] = c2["reference_model_s"] / (c2["ms_per_step"] / 1e3)
    out["config2_spectrum_k8_n20000"] = c2
    n5 = 200000
    c5 = run_slab(ctx, P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), L.KMG_F64, n5,
                  5, 0, n5 // 8, 2, 1, (0, n5 // 8 - 1), mm)
    c5["workload"] = ("BASELINE configs[4] per-GPU share: mismatch (9,1), N=200000, rows "
                      "0..25000 (one of 8 ranks) x 200000 columns, float64 normalised (40 GB)")
    c5["reference_model_s"] = reference_model_s("mismatch_k9_m1", n5)
    out["config5_mismatch_k9_n200000_rank_slab"] = c5
    # the same share as a column block: K[:, 0:25000] of all 200000 rows (= rows 0..25000
    # transposed; the lists are built over the block's 25000 sequences only and each is read
    # by all 200000 rows, so they pack -- DESIGN §5)
    c5c = run_slab(ctx, P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), L.KMG_F64, n5,
                   5, 0, n5, 2, 1, (0, n5 - 1), mm, cols=(0, n5 // 8))
    c5c["workload"] = ("BASELINE configs[4] per-GPU share as a column block: K[:, 0:25000] x "
                       "all 200000 rows (= the rank slab transposed), float64 normalised (40 GB)")
    out["config5_mismatch_k9_n200000_rank_colblock"] = c5c
    c5cr = run_slab(ctx, P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), L.KMG_I32, n5,
                    5, 0, n5, 2, 1, (0, n5 - 1), mmr, cols=(0, n5 // 8))
    c5cr["workload"] = ("config-5 raw int32 K's 1/8 share as a column block (the G=8 share of the "
                        "config5 full_1gpu build, collective-free)")
    out["config5_mismatch_k9_n200000_colblock_raw_int32"] = c5cr
    # the G = 8 column-block assembly rehearsed on this GPU: all 8 ranks' blocks + transposes
    # into one 160 GB K (no RCCL); the all-gather is modelled in projection()
    c5ca = run_colblock_assembly(ctx, Dist(), P.make(L.KMG_MISMATCH, k=9, m=1, window=101,
                                                     normalize=0), L.KMG_I32, n5, 5, 1, 1, mmr,
                                 world=8)
    c5ca["workload"] = ("config-5 raw int32 K from 8 column blocks, each transposed into its row "
                        "slab (kmg_gram_blocks gather 6: the G=8 column-block assembly without "
                        "its all-gather, every rank on this GPU)")
    out["config5_mismatch_k9_n200000_colblock_assembly_rehearsal_g8"] = c5ca
    c5f = run_slab(ctx, P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), L.KMG_I32,
                   n5, 5, 0, n5, 1, 1, (0, n5 - 1), mmr)
    c5f["workload"] = ("BASELINE configs[4] on ONE GPU: the full 200000 x 200000 raw int32 K "
                       "(160 GB; the G=1 point of the config-5 strong-scaling line)")
    out["config5_mismatch_k9_n200000_full_1gpu"] = c5f
    # drop-in host path: kmg_gram with a host float64 output (what kernels.get_spectrum_K
    # returns), PCIe D2H included; never `value`
    codes, lens = E.synthetic(20000, 101, seed=2)
    p8 = P.make(L.KMG_SPECTRUM, k=8)
    K = ctx.gram(p8, codes, lens, L.KMG_F64)
    t0 = time.perf_counter()
    K = ctx.gram(p8, codes, lens, L.KMG_F64, out=K)
    t = time.perf_counter() - t0
    out["host_path_spectrum_k8_n20000"] = {
        "ms": t * 1e3, "pairs_per_s": 20000 ** 2 / t,
        "note": "kmg_gram: H2D codes + device build + 3.2 GB float64 D2H into a numpy array"}
    del K
    try:
        out["host_path_config4"] = host_path_config4(ctx)
    except Exception as e:  # a host without 80 GB to pin: report, never fail the bench
        out["host_path_config4"] = {"error": repr(e)}
    out["run_py_kernels_n9000"] = run_py_workload(ctx)
    out["downstream"] = downstream(ctx)
    return out


def _hip():
    return ctypes.CDLL("libamdhip64.so")


def host_path_config4(ctx, n=100000, slab_rows=2500, f64=True):
    """SURVEY §8d's host legs at BASELINE configs[3] (get_spectrum_K returns the host array,
    kernels.py:47): H2D of the codes, then kmg_gram_to_host — device row slabs of one index
    build, each slab's D2H (second stream) overlapping the next slab's Gram — into one pinned
    host buffer, int32 (40 GB, exact counts) and float64 (80 GB, what the reference
    materialises).  Never `value`: PCIe-bound."""
    hip = _hip()
    codes, lens = E.synthetic(n, 101, seed=4)
    ldc = codes.shape[1]
    out = {"N": n, "slab_rows": slab_rows}
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    hp = ctypes.c_void_p()
    try:
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.synchronize()
        out["h2d_codes_ms"] = (time.perf_counter() - t0) * 1e3
        out["h2d_bytes"] = codes.nbytes + lens.nbytes
        p8 = P.make(L.KMG_SPECTRUM, k=8)
        total = n * n * (8 if f64 else 4)
        t0 = time.perf_counter()
        rc = hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(total), 0)
        out["pinned_alloc_s"] = time.perf_counter() - t0
        if rc != 0 or not hp.value:
            hp = ctypes.c_void_p()
            out["error"] = f"hipHostMalloc({total}) = {rc}"
            return out
        for dt, name in ((L.KMG_I32, "int32"), (L.KMG_F64, "float64")):
            if dt == L.KMG_F64 and not f64:
                continue
            esz = np.dtype(L.DTYPES[dt]).itemsize
            nbytes = n * n * esz
            buf = (ctypes.c_char * nbytes).from_address(hp.value)
            K = np.frombuffer(buf, dtype=L.DTYPES[dt]).reshape(n, n)
            ctx.gram_to_host(p8, d_codes, d_lens, n, ldc, dt, slab_rows, K)  # warm (index, slabs)
            t0 = time.perf_counter()
            ctx.gram_to_host(p8, d_codes, d_lens, n, ldc, dt, slab_rows, K)
            t = time.perf_counter() - t0
            import cref
            r = n // 2
            ok = bool(np.array_equal(K[r].astype(np.int64),
                                     cref.spectrum(codes, lens, 8, rows=(r, r + 1))[0]))
            out[name] = {"ms": t * 1e3, "bytes": nbytes, "d2h_GBps": nbytes / t / 1e9,
                         "pairs_per_s": n * n / t, "spot_check_row": r, "spot_check": ok}
            del K, buf
    finally:
        if hp.value:
            hip.hipHostFree(hp)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    out["note"] = ("kmg_gram_to_host into one hipHostMalloc'd buffer (pinning it is "
                   "pinned_alloc_s, outside the timings); the device build alone is the "
                   "headline ms_per_step (inputs resident)")
    return out


RUN_PY_METHODS = ["SP_k4", "SP_k5", "SP_k6", "MM_k4_m1", "MM_k5_m1", "MM_k6_m1", "WD_d4",
                  "WD_d5", "WD_d10"]


def run_py_workload(ctx, n=9000, reps=5):
    """run.py's nine Gram matrices (reference run.py:6, built by utils.get_training_datas,
    utils.py:149-153, over train+val+test = 9000 sequences), device-resident float64 K as
    the drop-in returns it: per-kernel device time, its HBM fraction (8 B per entry) and,
    for the int8-MFMA dense path, the MFMA fraction (2 * 4^k int ops per entry)."""
    codes, lens = E.synthetic(n, 101, seed=9000)
    ldc = codes.shape[1]
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    d_out = ctx.dmalloc(n * n * 8)
    out = {}
    try:
        for m in RUN_PY_METHODS:
            tok = m.split("_")
            if tok[0] == "SP":
                k = int(tok[1][1:])
                params = P.make(L.KMG_SPECTRUM, k=k)
            elif tok[0] == "MM":
                k = int(tok[1][1:])
                params = P.make(L.KMG_MISMATCH, k=k, m=int(tok[2][1:]), window=101, normalize=1)
            else:
                k = None
                params = P.make(L.KMG_WD, d=int(tok[1][1:]))
            ctx.gram_device(params, d_codes, d_lens, n, ldc, 0, n, L.KMG_F64, d_out, n)
            ctx.synchronize()
            ctx.set_timing(True)
            ctx.timing_reset()
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.gram_device(params, d_codes, d_lens, n, ldc, 0, n, L.KMG_F64, d_out, n)
            ctx.synchronize()
            wall = (time.perf_counter() - t0) / reps
            ctx.set_timing(False)
            st = stage_means(ctx)
            g = st.get("gram")
            rec = {"ms_per_build": wall * 1e3, "stages_ms": st,
                   "gram_hbm_frac": 8.0 * n * n / (g / 1e3) / HBM_PEAK if g else None}
            if st.get("features") is not None and k is not None:
                dp = max(128, 4 ** k)
                rec["dense_int8_dp"] = dp
                rec["gram_mfma_frac"] = 2.0 * dp * n * n / (g / 1e3) / INT8_PEAK
            out[m] = rec
        out["total_ms"] = sum(v["ms_per_build"] for v in out.values())
    finally:
        ctx.dfree(d_out)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    return out


FP64_PEAK = 78.6e12  # MI355X dense fp64 (spec sheet)


def downstream(ctx, asym=True):
    """§8f consumers of the Gram on device-resident float64 matrices at the production size
    (n = 9000 = train + val + test of the 3 TFs, utils.py:151-153): NLCK combination
    (HBM-bound) and the KRR / KLR / C-SVM solves (fp64 factorisation)."""
    n, p, reps = 9000, 3, 5
    rng = np.random.default_rng(9)
    A = rng.standard_normal((n, 64))
    K = A @ A.T
    K += n * 1e-3 * np.eye(n)
    d = np.sqrt(np.diag(K))
    K = K / d[:, None] / d[None, :]
    # K / d_i / d_j rounds differently at (i, j) and (j, i) (about a third of the entries
    # differ by an ulp), which would send KRR / KLR to the per-column LU of an asymmetric K;
    # every Gram kmg_gram returns is bitwise symmetric, so the bench's K is made so too
    Ka = K
    K = (K + K.T) / 2.0
    nbytes = K.nbytes
    dK = [ctx.dmalloc(nbytes) for _ in range(p)]
    for x in dK:
        ctx.h2d(x, K)
    d_out = ctx.dmalloc(nbytes)
    d_u = ctx.dmalloc(8 * p)
    ctx.h2d(d_u, np.array([0.5, 0.3, 0.2]))
    y = np.where(rng.random(n) > 0.5, 1.0, -1.0)
    d_y, d_a = ctx.dmalloc(8 * n), ctx.dmalloc(8 * n)
    ctx.h2d(d_y, y)
    ptrs = (ctypes.c_void_p * p)(*[x.value for x in dK])
    out = {}
    try:
        ctx.set_timing(True)
        L.check(ctx.lib.kmg_combine_device(ctx.handle, ptrs, p, d_u, 2, n, n, d_out, n))
        ctx.synchronize()
        ctx.timing_reset()
        for _ in range(reps):
            L.check(ctx.lib.kmg_combine_device(ctx.handle, ptrs, p, d_u, 2, n, n, d_out, n))
        tot, cnt = ctx.stage_stats("combine")
        ms = tot / cnt
        alg = 8.0 * (p + 1) * n * n
        out["nlck_combine_n9000_p3_deg2"] = {
            "ms": ms, "alg_bytes": alg, "achieved_GBps": alg / (ms / 1e3) / 1e9,
            "hbm_frac": alg / (ms / 1e3) / HBM_PEAK, "source": "NLCKernels.py:52,97",
            "note": "(sum_m u_m K_m)**2 on 3 device-resident 9000x9000 fp64 K, 1 write"}
        for m_ in (n, 2000):
            L.check(ctx.lib.kmg_krr_solve_device(ctx.handle, dK[0], n, m_, d_y, 0.1, d_a))
            ctx.synchronize()
            ctx.timing_reset()
            for _ in range(reps):
                L.check(ctx.lib.kmg_krr_solve_device(ctx.handle, dK[0], n, m_, d_y, 0.1, d_a))
            tot, cnt = ctx.stage_stats("solve")
            ms = tot / cnt
            fl = m_ ** 3 / 3.0 + 2.0 * m_ * m_
            out[f"krr_solve_n{m_}"] = {
                "ms": ms, "alg_flops": fl, "achieved_TFLOPs": fl / (ms / 1e3) / 1e12,
                "fp64_frac": fl / (ms / 1e3) / FP64_PEAK, "source": "KRR.py:33",
                "factorisation": ctx.last_factorisation(),
                "note": "symmetry check + blocked Cholesky (kmg_solve.hip, rocBLAS GEMM / syrk updates) + substitution sweeps of K + lbda n I"}
        # the same solve on the ulp-asymmetric K / d_i / d_j: LU (rocSOLVER dgetrf, launch-bound
        # per column), what any user-normalised K not symmetrised costs (asym=False: skipped,
        # tools/trace_downstream.py's trace of the symmetric legs)
        if asym:
            ctx.h2d(dK[1], Ka)
            m_ = 2000
            L.check(ctx.lib.kmg_krr_solve_device(ctx.handle, dK[1], n, m_, d_y, 0.1, d_a))
            ctx.synchronize()
            ctx.timing_reset()
            for _ in range(reps):
                L.check(ctx.lib.kmg_krr_solve_device(ctx.handle, dK[1], n, m_, d_y, 0.1, d_a))
            tot, cnt = ctx.stage_stats("solve")
            out["krr_solve_asymmetric_K_n2000"] = {
                "ms": tot / cnt, "factorisation": ctx.last_factorisation(), "source": "KRR.py:33",
                "note": "K != K^T by ulps: symmetry check + LU (dgetrf / dgetrs)"}
            ctx.h2d(dK[1], K)
        it = ctypes.c_int32(0)
        m_ = 2000
        # one untimed fit first (first-use costs of the IRLS path), as every other leg warms up
        L.check(ctx.lib.kmg_klr_fit_device(ctx.handle, dK[0], n, m_, d_y, 0.1, 1e-5, 50, d_a,
                                           ctypes.byref(it)))
        ctx.synchronize()
        ctx.timing_reset()
        L.check(ctx.lib.kmg_klr_fit_device(ctx.handle, dK[0], n, m_, d_y, 0.1, 1e-5, 50, d_a,
                                           ctypes.byref(it)))
        tot, cnt = ctx.stage_stats("solve")
        out["klr_fit_n2000"] = {"ms": tot, "iterations": it.value,
                                "ms_per_iteration": tot / max(1, it.value),
                                "factorisation": ctx.last_factorisation(),
                                "source": "KLR.py:57-75",
                                "note": "IRLS: dgemv + HIP IRLS kernel + Cholesky per step"}
        for m_ in (2000, n):
            it, obj = ctypes.c_int32(0), ctypes.c_double(0.0)
            ctx.timing_reset()
            L.check(ctx.lib.kmg_svm_fit_device(ctx.handle, dK[0], n, m_, d_y, 1.0, 1e-10, 100,
                                               d_a, ctypes.byref(it), ctypes.byref(obj)))
            tot, cnt = ctx.stage_stats("solve")
            out[f"svm_fit_n{m_}"] = {
                "ms": tot, "iterations": it.value, "ms_per_iteration": tot / max(1, it.value),
                "objective": obj.value, "source": "SVM.py:78-89",
                "note": "C=1 QP by Mehrotra interior point: dgemv + Cholesky + 2 solves per step"}
    finally:
        ctx.set_timing(False)
        for x in dK + [d_out, d_u, d_y, d_a]:
            ctx.dfree(x)
    return out


def load_traffic(workload, n):
    """HBM bytes per launch from the committed PMC pass of this workload at this N
    (profiles/*pmc*.json, written by profiles/pmc_summary.py), if any."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("N") == n and d.get("hbm_bytes_per_launch"):
            best = d["hbm_bytes_per_launch"]
    return best


def gather_roofline(res, world, esz):
    """All-gather over xGMI: bytes each rank receives per step / the gather's time on its
    stream, against the per-GPU ingress peak."""
    st = res.get("stages_ms", {})
    if world <= 1 or "gather_total" not in st:
        return None
    n = res["N"]
    npad = rows_padded(n, world, res["block_rows"])
    if res.get("gather_mode") == 2:  # upper-triangle round slabs of raw 8/16-bit counts
        esz = res.get("wire_bytes") or esz  # (kmg_gram_blocks_wire: what actually travelled)
        r = world * res["block_rows"]
        recv = (world - 1) / world * sum(r * w for _, w in triangle_rounds(n, world, res["block_rows"])) * esz
    else:
        recv = (world - 1) / world * npad * n * esz
    launches_per_step = res["rounds"]
    t = st["gather"] * launches_per_step / 1e3  # gather seconds per step
    return {"bound": "xgmi", "bytes_received_per_step": recv, "gather_ms_per_step": t * 1e3,
            "achieved_GBps": recv / t / 1e9, "peak_GBps": XGMI_IN_PEAK / 1e9,
            "frac": recv / t / XGMI_IN_PEAK}


def mm_nbhd_roofline(n, rows, gram_ms, plan, esz, k=9, P=93):
    """HBM model of the neighbourhood-list Gram launch (kmg_nbhd.hip): a row window reads
    its list once per column chunk, (1 + 3k) x (chunk x P / 4^k) uint16 entries in segments
    0 / 1 and 9k(k-1)/2 x (chunk x P / 4^k) in segment 2 -- packed, 16 B a 15 entries (the
    0.5 % of 15-entry runs that spill, measured on this data, ~1.078 B an entry), or 2 B --
    plus the segments' padding to 8, and the row writes its K row (a square K built by its
    upper block triangle: (nch + 1) / (2 nch) of both on average)."""
    nch, ch = max(1, plan["nchunks"]), max(8, plan["chunk"])
    n01, n2 = 1 + 3 * k, 9 * k * (k - 1) // 2
    b2 = 1.078 if plan.get("packed") else 2.0
    f = (nch + 1) / (2.0 * nch) if plan["triangle"] else 1.0
    occ = n * P / 4.0 ** k  # occurrences of a k-mer over all chunks
    per_window = (2.0 * n01 + b2 * n2) * occ + 2.0 * 10.5 * nch  # bytes over all chunks
    reads = rows * P * per_window * f
    writes = rows * n * esz * f
    alg = reads + writes
    return {"bound": "hbm", "table": "neighbourhood lists (%s segment 2; %d chunk(s) of %d "
                                     "columns%s; %d-thread workgroups)"
                                     % ("packed" if plan.get("packed") else "16-bit", nch, ch,
                                        ", upper block triangle" if plan["triangle"] else "",
                                        plan["threads"]),
            "list_bytes_per_window": per_window, "list_bytes_per_launch": reads,
            "k_bytes_per_launch": writes, "achieved_GBps": alg / (gram_ms / 1e3) / 1e9,
            "peak_GBps": HBM_PEAK / 1e9, "frac": alg / (gram_ms / 1e3) / HBM_PEAK}


def mm_gather_roofline(n, rows, gram_ms, plan, k=9, P=93):
    """Random-line gather model of the MM(9,1) Gram launch (see the secondary line), for the
    chunking the library reports (kmg_last_plan): a row reads every column chunk, or (a
    square K built by its upper block triangle) (nch + 1) / 2 of them on average."""
    if plan["formulation"] == "neighbourhood":
        return mm_nbhd_roofline(n, rows, gram_ms, plan, 8)
    nch = max(1, plan["nchunks"])
    reads = (nch + 1) / 2.0 if plan["triangle"] else float(nch)
    per_chunk = 117.0
    form = ("slot table (117 one-line lists a window and chunk, %d chunks%s)"
            % (nch, ", upper block triangle" if plan["triangle"] else ""))
    per_window = per_chunk * reads
    lines = rows * P * per_window
    rate = lines / (gram_ms / 1e3)
    return {"bound": "infinity-cache random 128-B line gathers", "table": form,
            "lines_per_window": per_window, "lines_per_launch": lines,
            "achieved_Glines_per_s": rate / 1e9, "ceiling_Glines_per_s": GATHER_CEILING / 1e9,
            "frac": rate / GATHER_CEILING,
            "source": "profiles/r02_mall_gather.jsonl (78.6 MB table, 128-B lines); PMC of the "
                      "one-chunk launch profiles/r03l_mm_n20000_pmc.txt, of the two-chunk "
                      "triangle launch profiles/r03af_mm_n20000_pmc.txt"}


def _chunked(n, max_chunk):
    """Column chunk width of a posting-list build: n split evenly into ceil(n / max_chunk)."""
    nch = -(-n // max_chunk)
    return -(-n // nch)


def projection(sp, n, extra):
    """G = 2/4/8 predictions for configs 4 and 5 from THIS run's one-GPU stage times
    (kmgram.shard.scaling_projection): index and Gram device times, the measured
    fill rate, uint8 round slabs (spectrum: diagonal from each rank; mismatch: escape list),
    xGMI at 76.5 GB/s per link and direction with no efficiency loss (an upper bound)."""
    fill = sp.get("write_ceiling_GBps") or 6000.0
    st = sp["stages_ms"]
    t_index = sum(v for k, v in st.items() if k in ("count", "scan", "place", "fine", "pack"))
    out = {"model": "kmgram.shard.scaling_projection (DESIGN.md §5); not measured on >1 GPU",
           "assumptions": {"xgmi_link_GBps": XGMI_IN_PEAK / 7 / 1e9, "link_eff": 1.0,
                           "fill_GBps": fill, "wire_bytes": 1}}
    # the G > 1 headline (strong, N = n, each GPU its 1/G of the rows, no collective): the
    # replicated index plus 1/G of the Gram (kmgram.shard.scaling_projection collective_free)
    out["headline_strong_collective_free"] = {
        str(g): {"N": n, "ms_model": t_index + st["gram"] / g,
                 "value_model": n * n / ((t_index + st["gram"] / g) / 1e3),
                 "speedup_model": sp["ms_per_step"] / (t_index + st["gram"] / g)}
        for g in (2, 4, 8)}
    out["config4_spectrum_k8_n%d" % n] = {
        str(g): v for g, v in scaling_projection(
            n, sp["ms_per_step"], t_index, st["gram"], fill, 4, 1,
            chunk=_chunked(n, 24576)).items()}
    c5 = (extra or {}).get("config5_mismatch_k9_n200000_full_1gpu")
    if c5:
        s5 = c5["stages_ms"]
        t5_index = sum(v for k, v in s5.items() if k in ("count", "scan", "place", "fine", "pack",
                                                         "lists", "nbfill", "slots"))
        n5 = c5["N"]
        # the one-GPU build computes the upper block triangle ((nch + 1) / (2 nch) of the full
        # rows, nch from the plan the library reported) and mirrors the rest: the model wants
        # the full-row Gram time
        plan5 = c5.get("plan") or {}
        ch5 = plan5.get("chunk") or _chunked(n5, 28572)
        nch = -(-n5 // ch5)
        g_rows = s5["gram"] * (2.0 * nch) / (nch + 1) if s5.get("mirror") else s5["gram"]
        out["config5_mismatch_k9_n200000_raw_int32"] = {
            "one_gpu": {"gram_ms": s5["gram"],
                        "mirror_ms": s5.get("mirror_per_build", s5.get("mirror")),
                        "full_rows_gram_ms_model": g_rows},
            **{str(g): v for g, v in scaling_projection(
                n5, c5["ms_per_step"], t5_index, g_rows, fill, 4, 1, chunk=ch5).items()}}
        cb = (extra or {}).get("config5_mismatch_k9_n200000_colblock_raw_int32")
        if cb:  # a G=8 share measured on this GPU: the collective-free build, no model
            out["config5_mismatch_k9_n200000_raw_int32"]["8"]["collective_free_measured_ms"] = \
                cb["ms_per_step"]
            out["config5_mismatch_k9_n200000_raw_int32"]["8"]["collective_free_measured_speedup"] = \
                c5["ms_per_step"] / cb["ms_per_step"]
        ca = (extra or {}).get("config5_mismatch_k9_n200000_colblock_assembly_rehearsal_g8")
        if cb and ca:
            # K on every GPU from column blocks (gather 5): one rank's block (measured) + its
            # transpose (the rehearsal's mean) + the in-place all-gather of int32 row slabs,
            # (G - 1) / G x 4 N^2 bytes into every GPU over its 7 links, in sequence (one round)
            tr = ca["transpose_ms_per_step"] / max(1.0, ca["transposes_per_step"])
            recv = 7.0 / 8.0 * 4.0 * n5 * n5 / XGMI_IN_PEAK * 1e3
            tot = cb["ms_per_step"] + tr + recv
            out["config5_mismatch_k9_n200000_raw_int32"]["8"]["colblock_assembled"] = {
                "block_ms_measured": cb["ms_per_step"], "transpose_ms_measured": tr,
                "receive_ms_model": recv, "ms_model": tot,
                "speedup_model": c5["ms_per_step"] / tot,
                "note": "int32 row slabs: 4x the bytes of the uint8 upper-triangle round slabs "
                        "the row-block path sends (every_gpu above), so receive-bound further out"}
    return out


_STAGE_KEYS = ("count", "place", "fine", "pack", "lists", "nbfill", "slots", "diag", "gram",
               "mirror")


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, float) else x


def _compact_record(rec):
    """The few keys of a build record the stdout tail must carry."""
    out = {}
    for k in ("workload", "N", "ms_per_step", "value", "pairs_per_s", "spot_check"):
        if k in rec:
            out[k] = _r(rec[k]) if k != "workload" else rec[k][:60]
    st = rec.get("stages_ms") or {}
    out["stages_ms"] = {k: _r(st[k]) for k in _STAGE_KEYS if k in st}
    pl = rec.get("plan") or {}
    if pl:
        out["plan"] = {k: pl.get(k) for k in ("formulation", "nchunks", "chunk", "triangle", "packed")
                       if k in pl}
    for k in ("hbm_frac_of_gram_and_mirror", "gram_hbm_frac"):
        if k in rec:
            out[k] = _r(rec[k])
    if isinstance(rec.get("cpu_baseline"), dict):
        out["cpu_baseline"] = {k: _r(rec["cpu_baseline"].get(k)) for k in ("value", "cores")}
    return out


def _compact_configs(extra):
    """The configs' times for the stdout tail: no workload text (bench_details.json has it),
    the stages that carry the time, the plan's shape."""
    out = {}
    for k, v in extra.items():
        if k.startswith("config") and isinstance(v, dict):
            rec = {kk: _r(v[kk]) for kk in ("ms_per_step", "spot_check", "gram_hbm_frac") if kk in v}
            st = v.get("stages_ms") or {}
            rec["stages_ms"] = {kk: _r(st[kk], 3) for kk in ("nbfill", "diag", "gram", "mirror")
                                if kk in st}
            if "mirror_per_build" in st:  # (one mirror launch per row chunk)
                rec["stages_ms"]["mirror"] = _r(st["mirror_per_build"], 3)
            pl = v.get("plan") or {}
            if pl:
                rec["plan"] = {kk: pl.get(kk) for kk in ("formulation", "nchunks", "packed") if kk in pl}
            out[k] = rec
    if isinstance(extra.get("run_py_kernels_n9000"), dict):
        out["run_py_kernels_n9000_total_ms"] = _r(extra["run_py_kernels_n9000"].get("total_ms"))
    return out


def _projection_summary(proj):
    """G = 8 speedup models per line of projection() (the full tables: bench_details.json)."""
    out = {}
    h = proj.get("headline_strong_collective_free", {}).get("8")
    if h:
        out["headline_collective_free"] = _r(h["speedup_model"], 3)
    for k, v in proj.items():
        if k.startswith("config") and isinstance(v, dict) and "8" in v:
            g8 = v["8"]
            out[k.split("_")[0]] = {"every_gpu": _r(g8.get("every_gpu_speedup"), 3),
                                   "collective_free": _r(g8.get("collective_free_speedup"), 3)}
            if "collective_free_measured_speedup" in g8:
                out[k.split("_")[0]]["collective_free_measured_share"] = _r(
                    g8["collective_free_measured_speedup"], 3)
            if "colblock_assembled" in g8:
                out[k.split("_")[0]]["colblock_assembled"] = _r(
                    g8["colblock_assembled"]["speedup_model"], 3)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=100000, help="spectrum N (headline)")
    ap.add_argument("--mm-n", type=int, default=20000, help="mismatch N (secondary)")
    ap.add_argument("--gather-mode", type=int, default=2, choices=(1, 2),
                    help="G > 1 assembly: 2 upper-triangle slabs + mirror, 1 full rows")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-mismatch", action="store_true")
    ap.add_argument("--no-weak", action="store_true",
                    help="skip the weak-scaled G > 1 build (N = n sqrt(G)): for rehearsals with "
                         "several ranks on one GPU, whose HBM the G weak shares would overfill")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the config 4 / 5, host-path, run.py and downstream lines")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    # `--gpus G` alone (no launcher environment): this process starts the G ranks itself,
    # before anything here touches the GPU, and relays rank 0's line
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={world} (launched with a different "
                 "number of ranks)")
    global GATHER_MODE
    GATHER_MODE = args.gather_mode
    # stdout carries exactly one JSON line: everything else written to fd 1 (gloo's
    # connection banner, runtime chatter) is sent to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    dist = Dist()
    if os.environ.get("KMG_BENCH_DRYRUN") == "1":
        # launcher plumbing only (tests/test_distributed_cpu.py): the rank layout of the
        # headline and one barrier / max-over-ranks round, no library, no GPU
        # (KMG_BENCH_FAIL_RANK=r: rank r exits with status 3, the launcher's failure path)
        if os.environ.get("KMG_BENCH_FAIL_RANK") == str(dist.rank):
            sys.exit(3)
        n = args.n
        rows = sum(b - a for a, b in block_cyclic_ranges(n, dist.world, dist.rank,
                                                          (-(-n // dist.world) + 7) // 8 * 8))
        dist.barrier()
        slowest = dist.max(float(dist.rank))
        per_rank = dist.gather(rows)
        if dist.rank == 0:
            print(json.dumps({"metric": METRIC, "dryrun": True, "n_gpus": dist.world,
                              "rank": dist.rank, "rows_this_rank": rows,
                              "rows_per_rank": per_rank, "max_over_ranks": slowest,
                              "local_rank": dist.local,
                              "launched": os.environ.get("KMG_BENCH_LAUNCHED") == "1"}),
                  file=json_out, flush=True)
        dist.close()
        return
    n1 = args.n
    sp_seed = 4 if n1 == 100000 else 2
    # the CPU baseline runs FIRST, before this process makes any HIP call: its workers are
    # forked, and a fork of a process holding a HIP context is unsafe (round 3's r03s
    # benchprof saw the forked workers crash in rocprofv3's signal handler)
    cpu = {}
    if dist.world == 1 and not args.no_cpu:
        cpu["spectrum_k8"] = cpu_baseline("spectrum_k8", n1, args.cpu_budget, sp_seed)
        if not args.no_mismatch:
            cpu["mismatch_k9_m1"] = cpu_baseline("mismatch_k9_m1", args.mm_n, args.cpu_budget / 2, 3)
    dev = os.environ.get("KMG_BENCH_DEVICE")
    ctx = L.Context(int(dev) if dev is not None else dist.local)
    # KMG_BENCH_NO_RCCL=1: the collective-free lines only (a rehearsal of the G > 1 headline
    # with several ranks on one GPU, where RCCL refuses duplicate devices)
    rccl = dist.world > 1 and os.environ.get("KMG_BENCH_NO_RCCL") != "1"
    rccl_error = None
    if rccl:
        # the communicator is the only RCCL step every G > 1 line needs; if it cannot be
        # built on every rank, the collective-free lines (the headline) still run
        comm_ok = False
        try:
            uid = dist.bcast_bytes(L.Context.unique_id() if dist.rank == 0 else None)
            ctx.comm_init(uid, dist.world, dist.rank)
            comm_ok = True
        except L.KmgError as e:
            rccl_error = repr(e)
            print(f"rank {dist.rank}: RCCL communicator failed: {e}", file=sys.stderr)
        if not dist.all_true(comm_ok):
            if comm_ok:
                ctx.comm_destroy()
            rccl = False
            rccl_error = rccl_error or "another rank's ncclCommInitRank failed"
    # headline at every G: the named N = n1 (strong scaling), K sharded over the ranks with
    # no data-path collective (the rows of K are independent, and K is symmetric: SURVEY
    # §8e) -- a rank's 1/G of the rows, or at G >= 4 its 1/G of the columns as one column
    # chunk (share_mode: the faster shape there); the other shape is `other_share`.  At
    # G > 1 the north-star's final RCCL all-gather (K assembled on every GPU) is `assembled`
    # and the weak-scaled build (N = n1 sqrt(G)) `weak_scaled`
    n = n1
    mode = share_mode(n, dist.world)
    sp_rows = run_build(ctx, dist, "spectrum_k8", P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32, n,
                        sp_seed, args.steps, args.warmup, check_spectrum, gather=0)
    sp_rows["share"] = "rows"
    sp_rows["rows_per_rank"] = dist.gather(sp_rows["rows_this_rank"])
    sp_cols = None
    if dist.world > 1:
        sp_cols = run_colshare(ctx, dist, "spectrum_k8", P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32,
                               n, sp_seed, args.steps, args.warmup, spectrum_row)
        sp_cols["cols_per_rank"] = dist.gather(sp_cols["cols_this_rank"])
    sp, sp_other = (sp_cols, sp_rows) if mode == "cols" else (sp_rows, sp_cols)
    sp["devices_per_rank"] = dist.gather(ctx.device)
    shares = None
    if dist.world == 1 and not args.no_extra:
        shares = measured_shares(ctx, dist, n, sp_seed, max(10, args.steps), args.warmup,
                                 sp["ms_per_step"])
    asm = None
    if rccl:
        asm = run_build(ctx, dist, "spectrum_k8", P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32, n1,
                        sp_seed, args.steps, args.warmup, check_spectrum)
    weak = None
    if dist.world > 1 and not args.no_weak:
        nw = weak_scaled_n(n1, dist.world)
        weak = run_build(ctx, dist, "spectrum_k8", P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32, nw,
                         2, args.steps, args.warmup, check_spectrum, gather=0)
    mm = None
    if not args.no_mismatch:
        mm = run_build(ctx, dist, "mismatch_k9_m1",
                       P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), L.KMG_F64,
                       args.mm_n, 3, max(10, args.steps), 2, check_mismatch,
                       gather=None if (rccl or dist.world == 1) else 0)
    c5 = None
    if rccl and not args.no_extra:
        # config-5 strong scaling: the full 200000^2 raw int32 K (160 GB) on every GPU
        c5 = run_build(ctx, dist, "mismatch_k9_m1_raw",
                       P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), L.KMG_I32,
                       200000, 5, 2, 1, check_mismatch_raw)
    c5ca = None
    if rccl and not args.no_extra:
        # config 5 assembled from column blocks (gather 5): K on every GPU, int32 all-gather
        import cref
        c5ca = run_colblock_assembly(ctx, dist, P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0),
                                     L.KMG_I32, 200000, 5, 2, 1,
                                     lambda c, l, r: cref.mismatch_raw(c, l, 9, 1, rows=(r, r + 1))[0])
    c5cb = None
    if dist.world > 1 and not args.no_extra:
        # config 5 collective-free at G > 1: each GPU its column block of the raw int32 K
        import cref
        c5cb = run_colblock_dist(ctx, dist, P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0),
                                 L.KMG_I32, 200000, 5, 2, 1,
                                 lambda c, l, r: cref.mismatch_raw(c, l, 9, 1, rows=(r, r + 1))[0])
    extra = None
    if dist.world == 1 and not args.no_extra:
        extra = extras(ctx, {k: v["value"] for k, v in cpu.items()}, max(20, args.steps))
    if rccl:
        ctx.comm_destroy()
    ctx.close()

    # roofline of the dominant kernel: gram_sp_kernel, one launch per round
    st = sp["stages_ms"]
    launches = max(1, st.get("gram_launches", 1) / max(1, args.steps))
    # K entries a launch writes: rows x all N (row share) or all N rows x the rank's columns
    out_per_launch = (sp["rows_this_rank"] * n if mode == "rows" else n * sp["cols_this_rank"]) / launches
    alg_bytes = 4.0 * out_per_launch + 52.0 * n  # int32 K write + packed input read
    kern_s = st["gram"] / 1e3
    achieved = alg_bytes / kern_s
    roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK,
            "traffic": load_traffic("spectrum_k8", n) if dist.world == 1 else None,
            "kernel": sp_kernel_name(sp.get("plan") or {}),
            "kernel_ms": st["gram"],
            "alg_bytes_per_launch": alg_bytes,
            # hipMemsetAsync over the same K buffer in the same run: a reference rate, not a
            # ceiling (the Gram kernel's own stores run faster than it)
            "memset_GBps": sp.get("write_ceiling_GBps"),
            "ratio_to_memset": (achieved / 1e9 / sp["write_ceiling_GBps"]
                                if sp.get("write_ceiling_GBps") else None)}

    line = {
        "metric": METRIC, "value": sp["pairs_per_s"], "unit": "Gram pairs/s",
        "n_gpus": dist.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": sp["ms_per_step"], "higher_is_better": True,
        # strong: the named N at every G, each GPU its 1/G of the rows (no data-path
        # collective); the all-gather assembly is `assembled`, the weak-scaled build
        # `weak_scaled`
        "scaling": "strong",
        "vs_baseline": None, "dtype": "int32",
        "data": "synthetic i.i.d. uniform ACGT, L=101, numpy default_rng(%d)" % (4 if n == 100000 else 2),
        "config": {"workload": "spectrum k=8 full-K build, N=%d x L=101 (BASELINE configs[3], the "
                               "north_star's target config; G>1: each GPU its 1/G share of K -- "
                               "rows K[R_g, :] at G=2, columns K[:, C_g] as one column chunk at "
                               "G>=4 -- no data-path collective, K assembled over RCCL measured "
                               "as `assembled`)" % n,
                   "N": n, "L": 101, "k": 8, "share": mode,
                   **({"rows_this_rank": sp["rows_this_rank"],
                       "rows_per_rank": sp["rows_per_rank"], "block_rows": sp["block_rows"]}
                      if mode == "rows" else
                      {"cols_this_rank": sp["cols_this_rank"],
                       "cols_per_rank": sp["cols_per_rank"]}),
                   "devices_per_rank": sp["devices_per_rank"],
                   "rccl": rccl, "rccl_error": rccl_error,
                   "parallelism": f"{'row' if mode == 'rows' else 'column'}-blocks x{dist.world}",
                   "out_dtype": "int32", "full_k_build_ms": sp["ms_per_step"]},
        "stages_ms": sp["stages_ms"], "roofline": roof, "spot_check": sp["spot_check"],
    }
    if shares:
        # the G-rank headline's per-rank share, timed here (collective-free: its time is the
        # job's); speedup = the one-GPU full build / the share
        line["shares_measured"] = {g: {"share": v["share"], "ms": _r(v["ms"]),
                                       "speedup": _r(v["speedup"], 3), "spot_check": v["spot_check"]}
                                   for g, v in shares.items()}
    if sp_other:
        line["other_share"] = {"share": sp_other["share"], "ms_per_step": sp_other["ms_per_step"],
                               "pairs_per_s": sp_other["pairs_per_s"],
                               "gram_ms": sp_other["stages_ms"].get("gram"),
                               "spot_check": sp_other["spot_check"]}
    if asm:
        # the north-star's assembly: N = n1, block-cyclic rows, upper-triangle uint8 round
        # slabs (escape list) all-gathered in place over RCCL + local unpack / mirror, so
        # every GPU ends with the whole K (bound by writing it: DESIGN §5)
        line["assembled"] = {
            "workload": "spectrum k=8, N=%d: K assembled on every GPU (RCCL all-gather)" % n1,
            "scaling": "strong", **{k: asm[k] for k in ("ms_per_step", "pairs_per_s", "stages_ms",
                                                        "block_rows", "rounds", "wire_bytes",
                                                        "spot_check") if k in asm},
            "collective_free": asm.get("collective_free"),
            "other_gather_mode": asm.get("other_gather_mode"),
            "gather_roofline": gather_roofline(asm, dist.world, 4)}
    if weak:
        line["weak_scaled"] = {
            "workload": "spectrum k=8, N=%d = 100000 sqrt(G): each GPU its 1/G of the rows x "
                        "all N columns (~1e10 Gram pairs per GPU), no data-path collective"
                        % weak["N"],
            "scaling": "weak", "N": weak["N"], "value": weak["pairs_per_s"],
            **{k: weak[k] for k in ("ms_per_step", "stages_ms", "rows_this_rank", "spot_check")}}
    if mm:
        mm_rows_launch = mm["rows_this_rank"] / max(1, mm["rounds"])
        mm_bytes = 8.0 * mm_rows_launch * args.mm_n + 52.0 * args.mm_n
        # Gram launch + (a square K built by its upper block triangle) the mirror of the rest
        mm_k_ms = mm["stages_ms"]["gram"] + mm["stages_ms"].get("mirror", 0.0)
        line["secondary"] = {
            "workload": "mismatch (k=9,m=1) full-K build, float64 normalised (BASELINE configs[2])",
            "N": args.mm_n, "value": mm["pairs_per_s"], "unit": "Gram pairs/s",
            "ms_per_step": mm["ms_per_step"], "stages_ms": mm["stages_ms"], "plan": mm["plan"],
            "hbm_frac_of_gram_and_mirror": mm_bytes / (mm_k_ms / 1e3) / HBM_PEAK,
            # the Gram launch against HBM: the neighbourhood lists' bytes (mm_nbhd_roofline;
            # the slot table's model, random 128-B lines, if a KMG_MM_FORM forces it)
            "gather_roofline": mm_gather_roofline(args.mm_n, mm_rows_launch,
                                                  mm["stages_ms"]["gram"], mm["plan"]),
            "spot_check": mm["spot_check"],
        }
        if "collective_free" in mm:
            line["secondary"]["collective_free"] = mm["collective_free"]
    if c5:
        line["config5_strong"] = {
            "workload": "BASELINE configs[4]: mismatch (9,1), N=200000, raw int32 K (160 GB) "
                        "assembled on every GPU (block-cyclic + in-place RCCL all-gather)",
            **{k: c5[k] for k in ("ms_per_step", "pairs_per_s", "stages_ms", "block_rows",
                                  "rounds", "spot_check", "collective_free")},
            "gather_roofline": gather_roofline(c5, dist.world, 4)}
    if c5ca:
        line["config5_colblock_assembled"] = {
            "workload": "BASELINE configs[4]: mismatch (9,1), N=200000, raw int32 K on every GPU "
                        "from G column blocks, each transposed into its row slab, one in-place "
                        "RCCL all-gather (kmg_gram_blocks gather 5)",
            "scaling": "strong", **c5ca}
    if c5cb:
        line["config5_colblock_collective_free"] = {
            "workload": "BASELINE configs[4]: mismatch (9,1), N=200000, raw int32 K as G column "
                        "blocks, each GPU K[:, C_g] of all rows (no collective; the G=1 point is "
                        "configs.config5_mismatch_k9_n200000_full_1gpu)",
            "scaling": "strong", **c5cb}
    if cpu:
        line["cpu_baseline"] = {k: v for k, v in cpu["spectrum_k8"].items() if k != "one_process"}
        line["cpu_baseline_one_process"] = cpu["spectrum_k8"]["one_process"]
        line["reference_model"] = {
            "s": reference_model_s("spectrum_k8", n),
            "speedup_vs_model": reference_model_s("spectrum_k8", n) / (sp["ms_per_step"] / 1e3),
            "note": "reference kernels.py cost model (BASELINE.md), survey container 8-core Xeon"}
        if mm:
            line["secondary"]["cpu_baseline"] = cpu["mismatch_k9_m1"]
    # The full records (every config's stages, run.py's kernels, the downstream solvers, the
    # G > 1 projection, the secondary's gather model) go to bench_details.json; the JSON line
    # keeps compact forms and ends with the configs 2 / 5 and configs[2] (secondary) numbers,
    # so the driver's 2000-character stdout tail holds them.
    details = {"configs": extra, "secondary": line.get("secondary")}
    if dist.world == 1:
        details["projection"] = projection(sp, n, extra)
        line["projection_g8"] = _projection_summary(details["projection"])
    if extra:
        line["configs"] = _compact_configs(extra)
    if "secondary" in line:
        line["secondary"] = _compact_record(line.pop("secondary"))
    line["details_file"] = "bench_details.json"
    if dist.rank == 0:
        try:
            with open(os.path.join(ROOT, "bench_details.json"), "w") as f:
                json.dump(details, f, indent=1, default=str)
        except OSError as e:
            line["details_file"] = "unwritable: %r" % (e,)
        print(json.dumps(line), file=json_out, flush=True)
    dist.close()


if __name__ == "__main__":
    main()
