#!/usr/bin/env python3
"""bench.py — Gram pairs/s of the MI355X string-kernel Gram engine.

Workload (BASELINE.json configs[1]): spectrum k=8 Gram of N=20000 synthetic DNA
sequences of length L=101 on one MI355X, int32 exact counts, device-resident
(input codes already in HBM when the timed region starts).  A "step" is one full
Gram build: k-mer extraction + posting-index build + Gram kernel over the rank's rows.

Multi-GPU (`python -m torch.distributed.run --nproc-per-node G bench.py --gpus G`):
one process per GPU, rows of K sharded across ranks with no data-path collective;
weak scaling — N = 20000*sqrt(G) so every rank computes the same 20000^2 Gram pairs
(rows N/G x N columns).  `value` = N^2 / max-over-ranks time.  `--allgather` adds the
RCCL all-gather that assembles K on every GPU (reported separately).

Also reported: the mismatch (k=9, m=1) Gram at the same N (BASELINE configs[2],
float64 normalised, exact), per-stage device times from HIP events, the HBM roofline
of the dominant kernel and the oracle timed on the host cores (cpu_baseline).
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
from kmgram.shard import even_splits, weak_scaled_n  # noqa: E402

HBM_PEAK = 8.0e12  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = ("Gram pairs/sec (N×N) + full-K build time, spectrum k=8 and mismatch "
          "(k=9,m=1), 1/2/4/8 GPUs")


class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")  # barrier / max on the host, no device traffic
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

    def bcast_bytes(self, b):
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def run_workload(ctx, dist, name, params, out_dtype, n, seed, steps, warmup, allgather):
    codes, lens = E.synthetic(n, 101, seed=seed)
    ldc = codes.shape[1]
    splits = even_splits(n, dist.world)
    r0, r1 = splits[dist.rank], splits[dist.rank + 1]
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    d_codes = ctx.dmalloc(codes.nbytes)
    d_lens = ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    full_rows = n if allgather else (r1 - r0)
    d_out = ctx.dmalloc(full_rows * n * esz)
    out_rows = ctypes.c_void_p(d_out.value + (r0 * n * esz if allgather else 0))

    def step():
        ctx.gram_device(params, d_codes, d_lens, n, ldc, r0, r1, out_dtype, out_rows, n)

    for _ in range(warmup):
        step()
    ctx.synchronize()
    ctx.set_timing(True)
    ctx.timing_reset()
    dist.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.synchronize()
    dist.barrier()
    t1 = time.perf_counter()
    ctx.set_timing(False)
    wall = dist.max(t1 - t0)
    stages = {}
    for st in ("count", "scan", "place", "fine", "pack", "extract", "features", "diag", "gram", "mirror"):
        tot, cnt = ctx.stage_stats(st)
        if cnt:
            stages[st] = round(tot / cnt, 5)
    res = {
        "name": name, "n": n, "rows": r1 - r0, "wall_s": wall, "steps": steps,
        "ms_per_step": wall / steps * 1e3, "pairs_per_s": n * n / (wall / steps),
        "stages_ms": stages, "gram_kernel_ms": stages.get("gram"),
    }
    if allgather and dist.world > 1:
        uid = dist.bcast_bytes(L.Context.unique_id() if dist.rank == 0 else None)
        ctx.comm_init(uid, dist.world, dist.rank)
        ctx.allgather_rows(d_out, n, n, out_dtype, splits)  # warm
        ctx.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
            ctx.allgather_rows(d_out, n, n, out_dtype, splits)
        ctx.synchronize()
        dist.barrier()
        ag = dist.max(time.perf_counter() - t0)
        res["with_allgather_ms_per_step"] = ag / steps * 1e3
        res["with_allgather_pairs_per_s"] = n * n / (ag / steps)
        ctx.comm_destroy()
    # small parity spot-check of the measured output (first row of this rank vs oracle)
    res["spot_check"] = spot_check(ctx, name, codes, lens, n, r0, out_rows, out_dtype, r1)
    if name == "spectrum_k8":
        res["write_ceiling_GBps"] = write_ceiling(ctx, out_rows, (r1 - r0) * n * esz)
    ctx.dfree(d_out)
    ctx.dfree(d_codes)
    ctx.dfree(d_lens)
    return res


def spot_check(ctx, name, codes, lens, n, r0, d_rows, out_dtype, r1=None):
    """Rows r0 and r1-1 of the measured output vs the oracle (the last row of a full K
    lies in the mirrored lower triangle of the mismatch path)."""
    try:
        import cref
    except Exception:
        return None
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    ok = True
    for r in sorted({r0, (r1 or r0 + 1) - 1}):
        row = np.empty(n, dtype=L.DTYPES[out_dtype])
        ctx.d2h(row, ctypes.c_void_p(d_rows.value + (r - r0) * n * esz))
        if name == "spectrum_k8":
            ref = cref.spectrum(codes, lens, 8, rows=(r, r + 1))[0]
            ok &= bool(np.array_equal(row.astype(np.int64), ref))
        else:
            ref = cref.mismatch_rows(codes, lens, 9, 1, rows=(r, r + 1))[0]
            ok &= bool(np.array_equal(row, ref))
    return ok


def write_ceiling(ctx, d_out, nbytes, reps=10):
    """Measured HBM write ceiling on this box: hipMemsetAsync over the same K buffer
    (context stream, HIP events) -> GB/s.  Reported beside the 8 TB/s spec peak."""
    ctx.memset(d_out, 0, nbytes)
    ctx.synchronize()
    ctx.set_timing(True)
    ctx.timing_reset()
    for _ in range(reps):
        ctx.memset(d_out, 0, nbytes)
    ctx.synchronize()
    tot, cnt = ctx.stage_stats("memset")
    ctx.set_timing(False)
    if not cnt:
        return None
    return nbytes / (tot / cnt / 1e3) / 1e9


def cpu_baseline(name, n, budget_s):
    """The strongest CPU restatement of the reference we have, timed on this box's host
    cores: scipy-sparse Phi Phi^T (oracle/cpu_ref.py spectrum_phi / mismatch_phi; the
    reference's own get_phi_u / get_phi_km feature maps, kernels.py:12-25, 161-175, and its
    np.dot pair loop, kernels.py:41-45, 211-215, as one sparse product).  Phi is built for
    all N (timed); the product runs on a bounded row sample and the whole job is
    extrapolated as t_phi + (N / rows) * t_rows.  Single-threaded (scipy's sparse product)."""
    import cpu_ref
    seed = 2 if name == "spectrum_k8" else 3
    codes, lens = E.synthetic(n, 101, seed=seed)
    t0 = time.perf_counter()
    F = (cpu_ref.spectrum_phi(codes, lens, 8) if name == "spectrum_k8"
         else cpu_ref.mismatch_phi(codes, lens, 9, 1))
    FT = F.T.tocsr()
    t_phi = time.perf_counter() - t0
    r = 16
    while True:
        t0 = time.perf_counter()
        (F[:r] @ FT).toarray()
        t = time.perf_counter() - t0
        if t >= budget_s / 4 or r >= n:
            break
        r = min(n, max(r * 2, int(r * (budget_s / 4) / max(t, 1e-3))))
    rows = min(n, max(r, int(r * (budget_s / 2) / max(t, 1e-6))))
    t0 = time.perf_counter()
    (F[:rows] @ FT).toarray()
    t_rows = time.perf_counter() - t0
    t_job = t_phi + (n / rows) * t_rows
    return {"value": n * n / t_job, "unit": "Gram pairs/s", "cores": 1, "kind": "port",
            "sample": f"scipy-sparse Phi Phi^T (oracle/cpu_ref.py {'spectrum_phi' if name == 'spectrum_k8' else 'mismatch_phi'}): "
                      f"Phi of all {n} sequences {t_phi:.2f} s + rows 0..{rows} x {n} in "
                      f"{t_rows:.2f} s, whole job extrapolated to {t_job:.1f} s, 1 thread"}


def cpu_baseline_openmp(name, n, budget_s):
    """The C oracle (oracle/kmg_oracle.c, pairwise merge / Hamming, OpenMP) on a bounded row
    sample of the same workload, on this box's host cores."""
    import cref
    cref.load()
    cores = int(os.environ.get("OMP_NUM_THREADS") or (os.cpu_count() or 1))
    seed = 2 if name == "spectrum_k8" else 3
    codes, lens = E.synthetic(n, 101, seed=seed)
    fn = ((lambda r: cref.spectrum(codes, lens, 8, rows=(0, r))) if name == "spectrum_k8"
          else (lambda r: cref.mismatch_raw(codes, lens, 9, 1, rows=(0, r))))
    r = 8
    while True:
        t0 = time.perf_counter()
        fn(r)
        t = time.perf_counter() - t0
        if t >= budget_s / 4 or r >= n:
            break
        r = min(n, max(r * 2, int(r * (budget_s / 4) / max(t, 1e-3))))
    rows = min(n, max(r, int(r * budget_s / max(t, 1e-6))))
    t0 = time.perf_counter()
    fn(rows)
    t = time.perf_counter() - t0
    return {"value": rows * n / t, "unit": "Gram pairs/s", "cores": cores, "kind": "port",
            "sample": f"oracle/kmg_oracle.c {'kmo_spectrum' if name == 'spectrum_k8' else 'kmo_mismatch_raw'}"
                      f" rows 0..{rows} x {n} columns ({rows * n} pairs) in {t:.2f} s, "
                      f"{cores} OpenMP threads"}


# reference kernels.py cost model (measured in the survey container: 8-core
# Xeon, numpy/OpenBLAS; not this box): seconds for the whole Gram build
def reference_model_s(kind, n):
    if kind == "spectrum_k8":
        return 1.10 * n + 10.0e-6 * n * (n + 1) / 2
    return 78.0 * n + 35e-6 * n * (n + 1) / 2 + 0.46e-6 * n * n / 2


def run_slab(ctx, params, out_dtype, n, seed, r0, r1, steps, warmup, spot_rows, oracle_row):
    """One workload on rows [r0, r1) x all n columns, device-resident, this rank only."""
    codes, lens = E.synthetic(n, 101, seed=seed)
    ldc = codes.shape[1]
    esz = np.dtype(L.DTYPES[out_dtype]).itemsize
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    d_out = ctx.dmalloc((r1 - r0) * n * esz)
    try:
        def step():
            ctx.gram_device(params, d_codes, d_lens, n, ldc, r0, r1, out_dtype, d_out, n)

        for _ in range(warmup):
            step()
        ctx.synchronize()
        ctx.set_timing(True)
        ctx.timing_reset()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        ctx.synchronize()
        wall = time.perf_counter() - t0
        ctx.set_timing(False)
        stages = {}
        for st in ("count", "scan", "place", "fine", "pack", "extract", "features", "diag", "gram", "mirror"):
            tot, cnt = ctx.stage_stats(st)
            if cnt:
                stages[st] = round(tot / cnt, 4)
        ok = True
        for r in spot_rows:
            row = np.empty(n, dtype=L.DTYPES[out_dtype])
            ctx.d2h(row, ctypes.c_void_p(d_out.value + (r - r0) * n * esz))
            ref = oracle_row(codes, lens, r)
            ok &= bool(np.array_equal(row.astype(ref.dtype), ref))
    finally:
        ctx.dfree(d_out)
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    ms = wall / steps * 1e3
    return {"N": n, "rows": r1 - r0, "steps": steps, "ms_per_step": ms,
            "pairs_per_s": (r1 - r0) * n / (ms / 1e3), "stages_ms": stages,
            "spot_check_rows": list(spot_rows), "spot_check": ok}


def extras(ctx, cpu_rates):
    """BASELINE configs[3] and [4] and the drop-in host path, on this GPU (N=1 runs only)."""
    import cref
    out = {}
    sp = lambda c, l, r: cref.spectrum(c, l, 8, rows=(r, r + 1))[0]  # noqa: E731
    mm = lambda c, l, r: cref.mismatch_rows(c, l, 9, 1, rows=(r, r + 1))[0]  # noqa: E731
    n4 = 100000
    c4 = run_slab(ctx, P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32, n4, 4, 0, n4, 3, 1,
                  (0, 54321, n4 - 1), sp)
    c4["workload"] = ("BASELINE configs[3]: spectrum k=8, N=100000 x L=101, full K on 1 GPU, "
                      "int32 (40 GB), posting-list formulation (DESIGN.md: why not the fp32 GEMM)")
    c4["gram_hbm_frac"] = (4.0 * n4 * n4 + 26.0 * n4) / (c4["stages_ms"]["gram"] / 1e3) / HBM_PEAK
    c4["reference_model_s"] = reference_model_s("spectrum_k8", n4)
    c4["speedup_vs_reference_model"] = c4["reference_model_s"] / (c4["ms_per_step"] / 1e3)
    if cpu_rates.get("spectrum_k8"):
        c4["speedup_vs_cpu_baseline"] = c4["pairs_per_s"] / cpu_rates["spectrum_k8"]
    out["config4_spectrum_k8_n100000"] = c4
    n5 = 200000
    c5 = run_slab(ctx, P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), L.KMG_F64, n5,
                  5, 0, n5 // 8, 2, 1, (0, n5 // 8 - 1), mm)
    c5["workload"] = ("BASELINE configs[4] per-GPU share: mismatch (9,1), N=200000, rows "
                      "0..25000 (one of 8 ranks) x 200000 columns, float64 normalised (40 GB)")
    c5["projected_8gpu_ms_per_step"] = c5["ms_per_step"]
    c5["projected_8gpu_pairs_per_s"] = 8 * c5["pairs_per_s"]
    c5["reference_model_s"] = reference_model_s("mismatch_k9_m1", n5)
    out["config5_mismatch_k9_n200000_rank_slab"] = c5
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
    out["downstream"] = downstream(ctx)
    return out


FP64_PEAK = 78.6e12  # MI355X dense fp64 (spec sheet)


def downstream(ctx):
    """§8f consumers of the Gram on device-resident float64 matrices at the production size
    (n = 9000 = train + val + test of the 3 TFs, utils.py:151-153): NLCK combination
    (HBM-bound) and the KRR / KLR solves (fp64 factorisation)."""
    import ctypes
    n, p, reps = 9000, 3, 5
    rng = np.random.default_rng(9)
    A = rng.standard_normal((n, 64))
    K = A @ A.T
    K += n * 1e-3 * np.eye(n)
    d = np.sqrt(np.diag(K))
    K = K / d[:, None] / d[None, :]
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
                "note": "Cholesky (rocSOLVER dpotrf) + dpotrs of K + lbda n I, fp64"}
        it = ctypes.c_int32(0)
        m_ = 2000
        ctx.timing_reset()
        L.check(ctx.lib.kmg_klr_fit_device(ctx.handle, dK[0], n, m_, d_y, 0.1, 1e-5, 50, d_a,
                                           ctypes.byref(it)))
        tot, cnt = ctx.stage_stats("solve")
        out["klr_fit_n2000"] = {"ms": tot, "iterations": it.value,
                                "ms_per_iteration": tot / max(1, it.value),
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


def load_traffic(workload):
    """HBM bytes per launch from the committed PMC pass (profiles/*pmc*.json), if any."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("hbm_bytes_per_launch"):
            best = d["hbm_bytes_per_launch"]
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=20000, help="sequences at 1 GPU (weak-scaled)")
    ap.add_argument("--allgather", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-mismatch", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=8.0)
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the N=100000 / N=200000 slab / host-path lines (N=1 only)")
    args = ap.parse_args()
    # stdout carries exactly one JSON line: everything else written to fd 1 (gloo's
    # connection banner, runtime chatter) is sent to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    dist = Dist()
    if dist.world != args.gpus and dist.rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={dist.world}", file=sys.stderr)
    # KMG_BENCH_DEVICE: pin every rank to one device (rehearsing the multi-rank protocol
    # on a one-GPU box); by default rank r uses device LOCAL_RANK
    dev = os.environ.get("KMG_BENCH_DEVICE")
    ctx = L.Context(int(dev) if dev is not None else dist.local)
    n = weak_scaled_n(args.n, dist.world)

    sp = run_workload(ctx, dist, "spectrum_k8", P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32, n, 2,
                      args.steps, args.warmup, args.allgather)
    mm = None
    if not args.no_mismatch:
        mm = run_workload(ctx, dist, "mismatch_k9_m1",
                          P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), L.KMG_F64,
                          n, 3, max(3, args.steps // 4), 1, args.allgather)
    cpu = {}
    if dist.world == 1 and dist.rank == 0 and not args.no_cpu:
        cpu["spectrum_k8"] = cpu_baseline("spectrum_k8", n, args.cpu_budget)
        cpu["spectrum_k8_openmp"] = cpu_baseline_openmp("spectrum_k8", n, args.cpu_budget / 2)
        if mm:
            cpu["mismatch_k9_m1"] = cpu_baseline("mismatch_k9_m1", n, args.cpu_budget / 2)
            cpu["mismatch_k9_m1_openmp"] = cpu_baseline_openmp("mismatch_k9_m1", n,
                                                               args.cpu_budget / 4)
    extra = None
    if dist.world == 1 and not args.no_extra:
        extra = extras(ctx, {k: v["value"] for k, v in cpu.items()})
    ctx.close()

    rows = sp["rows"]
    alg_bytes = 4.0 * rows * n + 26.0 * n  # int32 K write + 2-bit packed input
    kern_s = sp["gram_kernel_ms"] / 1e3
    achieved = alg_bytes / kern_s
    traffic = load_traffic("spectrum_k8")
    roof = {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": achieved / HBM_PEAK, "traffic": traffic,
            "kernel": "kmg::gram_sp_kernel<true,1,true,1>", "kernel_ms": sp["gram_kernel_ms"],
            "alg_bytes_per_launch": alg_bytes,
            "measured_write_ceiling_GBps": sp.get("write_ceiling_GBps"),
            "frac_of_measured_ceiling": (achieved / 1e9 / sp["write_ceiling_GBps"]
                                         if sp.get("write_ceiling_GBps") else None)}

    line = {
        "metric": METRIC, "value": sp["pairs_per_s"], "unit": "Gram pairs/s",
        "n_gpus": dist.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": sp["ms_per_step"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int32",
        "data": "synthetic i.i.d. uniform ACGT, L=101, numpy default_rng(2)",
        "config": {"workload": "spectrum k=8 Gram, N=20000 x L=101 per GPU-share "
                               "(BASELINE configs[1]); weak-scaled N=20000*sqrt(G)",
                   "N": n, "L": 101, "k": 8, "rows_per_rank": rows,
                   "parallelism": f"row-shard x{dist.world}", "out_dtype": "int32",
                   "full_k_build_ms": sp["ms_per_step"]},
        "stages_ms": sp["stages_ms"], "roofline": roof, "spot_check": sp["spot_check"],
    }
    if "with_allgather_ms_per_step" in sp:
        line["allgather"] = {k: sp[k] for k in ("with_allgather_ms_per_step",
                                                "with_allgather_pairs_per_s")}
    if mm:
        mm_rows = mm["rows"]
        mm_bytes = 8.0 * mm_rows * n + 26.0 * n
        line["secondary"] = {
            "workload": "mismatch (k=9,m=1) Gram, float64 normalised (BASELINE configs[2])",
            "N": n, "value": mm["pairs_per_s"], "unit": "Gram pairs/s",
            "ms_per_step": mm["ms_per_step"], "stages_ms": mm["stages_ms"],
            "hbm_frac_of_gram_kernel": (mm_bytes / (mm["gram_kernel_ms"] / 1e3)) / HBM_PEAK,
            # the kernel's actual bound: one 128-byte slot line per posting
            # list, (101-9+1) windows x (9 + 3*9*8/2) lists per row
            "slot_line_GBps": 128.0 * mm_rows * 93 * 117 / (mm["gram_kernel_ms"] / 1e3) / 1e9,
            "spot_check": mm["spot_check"],
        }
    if cpu:
        line["cpu_baseline"] = cpu["spectrum_k8"]
        line["cpu_baseline_alt"] = cpu["spectrum_k8_openmp"]
        line["reference_model"] = {
            "s": reference_model_s("spectrum_k8", n),
            "note": "reference kernels.py cost model (BASELINE.md), survey container 8-core Xeon"}
        if mm:
            line["secondary"]["cpu_baseline"] = cpu["mismatch_k9_m1"]
            line["secondary"]["cpu_baseline_alt"] = cpu["mismatch_k9_m1_openmp"]
    if extra:
        line["configs"] = extra
    if dist.rank == 0:
        print(json.dumps(line), file=json_out, flush=True)
    dist.close()


if __name__ == "__main__":
    main()
