"""kmgram.shard.scaling_projection: the G-GPU model bench.py emits at N=1."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kernel-methods-for-genomics_amd"))

from kmgram.shard import default_block, scaling_projection, triangle_rounds  # noqa: E402


def test_projection_bytes_and_bounds():
    n = 100000
    p = scaling_projection(n, 6.5, 0.15, 6.35, 6100.0, 4, 1, chunk=20000)
    for g, v in p.items():
        b = default_block(n, g, n * 4)
        assert v["block_rows"] == b
        slab = sum(g * b * w for _, w in triangle_rounds(n, g, b))
        assert abs(v["bytes_received_per_gpu"] - slab * (g - 1) / g) < 1
        # the slabs cover the upper triangle at least once
        assert slab >= n * (n + 1) / 2
        # receive: the (G-1)/G share over G-1 links of 76.5 GB/s
        assert abs(v["receive_ms"] - slab / (g * 76.5e9) * 1e3) < 1e-9
        # every GPU writes the whole int32 K: never below n^2 * 4 / fill
        assert v["unpack_ms"] >= n * n * 4 / 6100e9 * 1e3
        assert v["every_gpu_ms"] >= max(v["compute_ms"], v["receive_ms"], v["unpack_ms"])
        assert v["collective_free_ms"] == 0.15 + 6.35 / g
    # config 4 with K on every GPU cannot beat the single-GPU build
    assert all(v["every_gpu_speedup"] < 1.0 for v in p.values())
    assert p[8]["collective_free_speedup"] > p[4]["collective_free_speedup"] > p[2]["collective_free_speedup"]


def test_projection_chunk_granularity():
    """Whole column chunks left of a round's first row are skipped, so the Gram share lies
    between the exact upper triangle and the full rows."""
    n = 200000
    fine = scaling_projection(n, 277.7, 2.8, 274.9, 6100.0, 4, 1, chunk=1, worlds=(8,))[8]
    coarse = scaling_projection(n, 277.7, 2.8, 274.9, 6100.0, 4, 1, chunk=n, worlds=(8,))[8]
    mid = scaling_projection(n, 277.7, 2.8, 274.9, 6100.0, 4, 1, chunk=28572, worlds=(8,))[8]
    assert fine["compute_ms"] < mid["compute_ms"] < coarse["compute_ms"]
    assert abs(coarse["compute_ms"] - (2.8 + 274.9 / 8)) < 1e-6


def test_bench_list_model_matches_pmc():
    """bench.mm_nbhd_roofline's byte model of the neighbourhood-list Gram at N=20000 (one
    chunk, float64 K) against the PMC of the same launch: 2 FETCH_SIZE + WRITE_SIZE.
    16-bit lists: 13.24 GB (profiles/r04p_mm_n20000_pmc.json); packed segment 2: 9.57 GB
    (profiles/r05b_mm_n20000_pmc.txt: FETCH 3142748 KiB, WRITE 3125482 KiB).  The packed
    lists fetch ~11 % over the model (2.9 KB lists: the partial 128-byte lines at a list's
    two ends weigh more than at 5 KB)."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    import bench
    for packed, pmc in ((False, 13.24e9), (True, (2 * 3142747.8 + 3125482.2) * 1024)):
        one = {"formulation": "neighbourhood", "chunk": 20000, "nchunks": 1, "triangle": False,
               "threads": 1024, "packed": packed}
        g = bench.mm_gather_roofline(20000, 20000, 2.0, one)
        alg = g["list_bytes_per_launch"] + g["k_bytes_per_launch"]
        assert abs(alg - pmc) / pmc < (0.13 if packed else 0.06), (packed, alg, pmc)
    # the weak-scaled headline N keeps every GPU at ~n1^2 pairs
    from kmgram.shard import weak_scaled_n
    for w in (2, 4, 8):
        n = weak_scaled_n(100000, w)
        assert abs(n * n / w - 1e10) / 1e10 < 1e-3


def test_bench_headline_projection_is_strong_at_named_n():
    """At G > 1 the headline keeps N = 100000 (strong scaling): the projection bench.py
    emits for it is index + gram / G at that N."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    import bench
    sp = {"ms_per_step": 6.5, "write_ceiling_GBps": 6100.0,
          "stages_ms": {"count": 0.05, "scan": 0.01, "place": 0.04, "fine": 0.03, "pack": 0.0,
                        "gram": 6.3}}
    p = bench.projection(sp, 100000, None)["headline_strong_collective_free"]
    for g in ("2", "4", "8"):
        assert p[g]["N"] == 100000
        assert abs(p[g]["ms_model"] - (0.13 + 6.3 / int(g))) < 1e-9
    assert p["8"]["speedup_model"] > 6.0


def test_bench_headline_share_shapes():
    """The G-rank headline's per-rank share (bench.share_mode): rows at G = 1 and 2; at G >= 4
    a column block, which the library makes ONE column chunk (KMG_SP_CB_CHUNK = 32768), so
    every rank's columns fit it; sp_kernel_name names the gram_sp_kernel instance the plan
    launches (int32 K: plain stores for one chunk; two rows a workgroup at chunks <= 16384)."""
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
    import bench
    from kmgram.shard import rank_rows
    assert bench.share_mode(100000, 1) == "rows"
    assert bench.share_mode(100000, 2) == "rows"
    assert bench.share_mode(100000, 3) == "rows"  # 33334 columns: past one chunk
    for g in (4, 5, 8, 16):
        assert bench.share_mode(100000, g) == "cols"
        widths = [b - a for a, b in (rank_rows(100000, g, r) for r in range(g))]
        assert sum(widths) == 100000 and max(widths) <= bench.SP_COLSHARE_MAX
    assert bench.sp_kernel_name({"chunk": 20000, "nchunks": 5}) == "kmg::gram_sp_kernel<true,1,true,1>"
    assert bench.sp_kernel_name({"chunk": 25000, "nchunks": 1}) == "kmg::gram_sp_kernel<true,1,false,1>"
    assert bench.sp_kernel_name({"chunk": 12504, "nchunks": 1}) == "kmg::gram_sp_kernel<true,1,false,2>"
