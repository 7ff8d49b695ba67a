"""GPU tests of the multi-GPU build path on one device: kmg_gram_blocks (block-cyclic rows,
index built once, Gram launched per round) and its in-place RCCL all-gather on a 1-rank
communicator.  Two ranks' block sets written into one buffer must assemble the full K
exactly (the rows each rank owns are disjoint and cover K).  Argument checks of the
device entry points ride along."""
import ctypes

import numpy as np
import pytest

from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P
from kmgram.shard import block_cyclic_ranges, rows_padded

pytestmark = pytest.mark.gpu

CASES = [
    (P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32),
    (P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), L.KMG_F64),
    (P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), L.KMG_I32),
    (P.make(L.KMG_WD, d=5), L.KMG_F64),
]


@pytest.fixture(scope="module")
def data(ctx):
    codes, lens = E.synthetic(1500, 101, seed=71)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    yield codes, lens, d_codes, d_lens
    ctx.dfree(d_codes)
    ctx.dfree(d_lens)


def _run_blocks(ctx, data, params, dt, world, ranks, block, gather):
    codes, lens, d_codes, d_lens = data
    n, ldc = codes.shape
    npad = rows_padded(n, world, block)
    assert npad == L.load().kmg_rows_padded(n, world, block)
    esz = np.dtype(L.DTYPES[dt]).itemsize
    d_out = ctx.dmalloc(npad * n * esz)
    try:
        ctx.memset(d_out, 0xA5, npad * n * esz)
        for r in ranks:
            ctx.gram_blocks(params, d_codes, d_lens, n, ldc, dt, d_out, n, world, r, block, gather)
        ctx.synchronize()
        out = np.empty((n, n), dtype=L.DTYPES[dt])
        ctx.d2h(out, d_out)
        return out
    finally:
        ctx.dfree(d_out)


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world,block", [(1, 1500), (1, 333), (2, 256), (3, 100), (8, 64)])
def test_blocks_union_equals_full(ctx, data, case, world, block):
    params, dt = CASES[case]
    codes, lens = data[0], data[1]
    full = ctx.gram(params, codes, lens, dt)
    got = _run_blocks(ctx, data, params, dt, world, range(world), block, gather=False)
    assert np.array_equal(got, full)


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world,rank,block", [(1, 0, 1500), (3, 1, 100), (8, 7, 64), (2, 0, 256)])
def test_blocks_packed_rank_share(ctx, data, case, world, rank, block):
    """gather = 4 (the multi-GPU bench's collective-free build): this rank's blocks packed
    in its own buffer, row t*block + y = K row t*world*block + rank*block + y."""
    params, dt = CASES[case]
    codes, lens, d_codes, d_lens = data
    n, ldc = codes.shape
    full = ctx.gram(params, codes, lens, dt)
    rounds = block_cyclic_ranges(n, world, rank, block)
    esz = np.dtype(L.DTYPES[dt]).itemsize
    d_out = ctx.dmalloc(len(rounds) * block * n * esz)
    try:
        ctx.memset(d_out, 0xA5, len(rounds) * block * n * esz)
        ctx.gram_blocks(params, d_codes, d_lens, n, ldc, dt, d_out, n, world, rank, block, 4)
        ctx.synchronize()
        got = np.empty((len(rounds) * block, n), dtype=L.DTYPES[dt])
        ctx.d2h(got, d_out)
    finally:
        ctx.dfree(d_out)
    for t, (a, b) in enumerate(rounds):
        assert np.array_equal(got[t * block:t * block + (b - a)], full[a:b]), (t, a, b)


@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("world,block", [(1, 1500), (1, 336), (2, 256), (3, 100), (8, 64),
                                         (4, 50)])
def test_upper_triangle_assembly_equals_full(ctx, data, case, world, block):
    """gather = 3: every rank's upper-triangle round slabs (columns >= the round's first row)
    computed on this GPU, copied into K and mirrored into the lower triangle: exactly the
    single-call K, every element written (the buffer starts poisoned).  Blocks that are not
    multiples of 8 and the WD kernel take the full-row scratch + copy-out path."""
    params, dt = CASES[case]
    codes, lens = data[0], data[1]
    full = ctx.gram(params, codes, lens, dt)
    got = _run_blocks(ctx, data, params, dt, world, [0], block, gather=3)
    assert np.array_equal(got, full)


@pytest.fixture(scope="module")
def data_repeats(ctx):
    """Every 97th row a homopolymer: its raw mismatch (9,1) self-count is 93 * 93 * 28 =
    242172, past the 16-bit round slabs (the build must notice and redo with 32 bits); the
    spectrum counts stay <= 94^2."""
    codes, lens = E.synthetic(600, 101, seed=72)
    codes[::97] = 0
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    yield codes, lens, d_codes, d_lens
    ctx.dfree(d_codes)
    ctx.dfree(d_lens)


@pytest.mark.parametrize("case", [0, 1, 2])
@pytest.mark.parametrize("world,block", [(2, 128), (3, 64)])
def test_upper_triangle_8bit_slabs_escapes(ctx, data_repeats, case, world, block):
    """Round slabs travel as uint8 counts; an off-diagonal count >= 255 (homopolymer pairs:
    94^2 spectrum, 242172 raw mismatch) goes to the escape list, which is patched into K
    after the unpack: the assembled K equals the single-call K."""
    params, dt = CASES[case]
    codes, lens = data_repeats[0], data_repeats[1]
    full = ctx.gram(params, codes, lens, dt)
    if case == 2:
        assert full.max() > 65535
    got = _run_blocks(ctx, data_repeats, params, dt, world, [0], block, gather=3)
    assert np.array_equal(got, full)
    assert ctx.blocks_wire() == 1


@pytest.mark.parametrize("case", [0, 1, 2])
def test_upper_triangle_escape_list_full_ladder(ctx, tune, data_repeats, case):
    """An escape list too small for the build (KMG_ESC_CAP=4) raises the overflow flag and
    the build is redone one width up: spectrum at 16 bits (its counts <= 94^2), raw mismatch
    at the output dtype's width (242172 > 65535).  The K is exact either way."""
    tune(KMG_ESC_CAP=4)
    params, dt = CASES[case]
    codes, lens = data_repeats[0], data_repeats[1]
    full = ctx.gram(params, codes, lens, dt)
    got = _run_blocks(ctx, data_repeats, params, dt, 2, [0], 128, gather=3)
    assert np.array_equal(got, full)
    assert ctx.blocks_wire() == (2 if case == 0 else np.dtype(L.DTYPES[dt]).itemsize)


@pytest.mark.parametrize("form", ["0", "1", "4"])
def test_upper_triangle_escapes_n20000(ctx, tune, form):
    """N=20000 MM(9,1), normalised float64 K, uint8 round slabs of 8 ranks rehearsed on one
    GPU: 40 row pairs share an injected 30-mer (counts far past 255, so escapes are taken on
    top of the random pairs' own); the assembled K equals the one-call K byte for byte."""
    tune(KMG_MM_FORM=form)
    codes, lens = E.synthetic(20000, 101, seed=74)
    rng = np.random.default_rng(75)
    motif = rng.integers(0, 4, size=30, dtype=np.uint8)
    for _ in range(40):
        i, j = rng.choice(20000, size=2, replace=False)
        codes[i, 10:40] = motif
        codes[j, 50:80] = motif
    params = P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1)
    full = ctx.gram(params, codes, lens, L.KMG_F64)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        got = _run_blocks(ctx, (codes, lens, d_codes, d_lens), params, L.KMG_F64, 8, [0], 1024,
                          gather=3)
    finally:
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    assert ctx.blocks_wire() == 1
    assert np.array_equal(got, full)


@pytest.mark.parametrize("case", [0, 1, 2])
def test_upper_triangle_8bit_slabs(ctx, data, case):
    """Random sequences: round slabs of spectrum and mismatch counts travel as uint8 with the
    diagonal left out (K_ii from the locally computed diagonal)."""
    params, dt = CASES[case]
    codes, lens = data[0], data[1]
    full = ctx.gram(params, codes, lens, dt)
    got = _run_blocks(ctx, data, params, dt, 3, [0], 104, gather=3)
    assert np.array_equal(got, full)
    assert ctx.blocks_wire() == 1


def test_upper_triangle_one_rank_gather2(ctx, data):
    """gather = 2 on one rank needs no communicator and assembles the same K."""
    params, dt = CASES[1]
    codes, lens = data[0], data[1]
    full = ctx.gram(params, codes, lens, dt)
    got = _run_blocks(ctx, data, params, dt, 1, [0], 256, gather=2)
    assert np.array_equal(got, full)


def test_block_cyclic_ranges_match_library(ctx, data):
    """The Python layout helper (used by bench.py) and the library agree: rank 1 of 3 writes
    exactly the rows block_cyclic_ranges lists, nothing else."""
    params, dt = CASES[0]
    codes, lens = data[0], data[1]
    n = codes.shape[0]
    full = ctx.gram(params, codes, lens, dt)
    got = _run_blocks(ctx, data, params, dt, 3, [1], 100, gather=False)
    mine = np.zeros(n, dtype=bool)
    for a, b in block_cyclic_ranges(n, 3, 1, 100):
        mine[a:b] = True
    assert np.array_equal(got[mine], full[mine])
    assert np.all(got[~mine].view(np.uint32) == 0xA5A5A5A5)


def test_blocks_gather_single_rank_comm(ctx, data):
    """gather = 1 (full rows) and 2 (upper-triangle uint16 slabs, unpacked on their own
    stream) on a 1-rank RCCL communicator: the comm-stream / unpack-stream / event ordering
    path with an in-place ncclAllGather per round; the result is the full K on the context
    stream."""
    uid = L.Context.unique_id()
    ctx.comm_init(uid, 1, 0)
    try:
        for params, dt in CASES[:3]:
            full = ctx.gram(params, data[0], data[1], dt)
            for gather, block in ((1, 200), (2, 200), (2, 96)):
                got = _run_blocks(ctx, data, params, dt, 1, [0], block, gather=gather)
                assert np.array_equal(got, full), (gather, block)
        with pytest.raises(L.KmgError):  # communicator size must match
            _run_blocks(ctx, data, CASES[0][0], CASES[0][1], 2, [0], 200, gather=True)
    finally:
        ctx.comm_destroy()


def test_allgather_rows_validates_splits(ctx):
    uid = L.Context.unique_id()
    ctx.comm_init(uid, 1, 0)
    d = ctx.dmalloc(64 * 64 * 4)
    try:
        for bad in ([1, 64], [0, 63], [0, 65]):
            with pytest.raises(L.KmgError):
                ctx.allgather_rows(d, 64, 64, L.KMG_I32, bad)
        with pytest.raises(L.KmgError):
            ctx.allgather_rows(d, 64, 32, L.KMG_I32, [0, 64])  # ld < n
        ctx.allgather_rows(d, 64, 64, L.KMG_I32, [0, 64])
        ctx.synchronize()
    finally:
        ctx.dfree(d)
        ctx.comm_destroy()


def test_mismatch_device_rows_narrower_than_window(ctx):
    """kmg_gram_device with code rows of 100 < the 101 window: EINVAL, no kernel reads past
    a row."""
    codes, lens = E.synthetic(16, 100, seed=3)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(16 * 16 * 8)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        for params in (P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1),
                       P.make(L.KMG_GAPPY, k=1, g=0)):
            with pytest.raises(L.KmgError) as e:
                ctx.gram_device(params, d_codes, d_lens, 16, 100, 0, 16, L.KMG_F64, d_out, 16)
            assert e.value.status == L.KMG_EINVAL
    finally:
        for p in (d_out, d_codes, d_lens):
            ctx.dfree(p)


@pytest.mark.parametrize("params,dt,wire", [
    (P.make(L.KMG_MISMATCH, k=10, m=1, window=101, normalize=1), L.KMG_F64, 1),  # pair table
    (P.make(L.KMG_MISMATCH, k=8, m=1, window=101, normalize=0), L.KMG_I32, 1),   # slot table
    (P.make(L.KMG_SPECTRUM, k=12), L.KMG_I32, 1),
    (P.make(L.KMG_SPECTRUM, k=5), L.KMG_I32, 4),  # dense path: full-width slabs
])
def test_upper_triangle_slabs_other_formulations(ctx, params, dt, wire):
    """The narrow round slabs through the other posting-list kernels (drop-two pair table
    at k = 10, slot table at k = 8, spectrum k = 12) and the full-width fallback of the
    dense formulation: the assembled K equals the single-call K."""
    codes, lens = E.synthetic(400, 101, seed=73)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        full = ctx.gram(params, codes, lens, dt)
        got = _run_blocks(ctx, (codes, lens, d_codes, d_lens), params, dt, 3, [0], 48, gather=3)
    finally:
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    assert np.array_equal(got, full)
    assert ctx.blocks_wire() == wire


# ---------------------------------------------------------------- column-block assembly
def _colblock_assembly(ctx, data, params, dt, world, block, gather):
    codes, lens, d_codes, d_lens = data
    n, ldc = codes.shape
    esz = np.dtype(L.DTYPES[dt]).itemsize
    npad = world * block
    d_out = ctx.dmalloc(npad * n * esz)
    try:
        ctx.memset(d_out, 0xA5, npad * n * esz)
        ctx.gram_blocks(params, d_codes, d_lens, n, ldc, dt, d_out, n, world, 0, block, gather)
        ctx.synchronize()
        out = np.empty((n, n), dtype=L.DTYPES[dt])
        ctx.d2h(out, d_out)
        return out
    finally:
        ctx.dfree(d_out)


@pytest.mark.parametrize("case", [0, 1, 2])
@pytest.mark.parametrize("world", [2, 3, 8])
def test_column_block_assembly_equals_full(ctx, data, case, world):
    """gather = 6 (the one-GPU rehearsal of gather = 5): every rank's column block K[:, C_q]
    (lists / postings over its own sequences) computed, transposed into K's rows C_q:
    exactly the single-call K (the buffer starts poisoned), spectrum and mismatch."""
    params, dt = CASES[case]
    codes, lens = data[0], data[1]
    n = codes.shape[0]
    full = ctx.gram(params, codes, lens, dt)
    block = -(-n // world)
    got = _colblock_assembly(ctx, data, params, dt, world, block, 6)
    assert np.array_equal(got, full)
    assert ctx.last_plan()["formulation"] == ("posting" if case == 0 else "neighbourhood")


def test_column_block_assembly_single_rank_comm(ctx, data):
    """gather = 5 on a 1-rank RCCL communicator (the in-place all-gather after the transpose,
    comm-stream ordering), and the argument checks: nranks * block must cover n, and a
    communicator of another size is refused."""
    params, dt = CASES[1]
    codes, lens = data[0], data[1]
    n = codes.shape[0]
    full = ctx.gram(params, codes, lens, dt)
    uid = L.Context.unique_id()
    ctx.comm_init(uid, 1, 0)
    try:
        got = _colblock_assembly(ctx, data, params, dt, 1, n, 5)
        assert np.array_equal(got, full)
        with pytest.raises(L.KmgError):  # communicator size must match
            _colblock_assembly(ctx, data, params, dt, 2, -(-n // 2), 5)
    finally:
        ctx.comm_destroy()
    with pytest.raises(L.KmgError):  # 3 x 400 rows do not cover n = 1500
        _colblock_assembly(ctx, data, params, dt, 3, 400, 6)
    with pytest.raises(L.KmgUnsupported):  # column blocks: the posting-list paths only
        _colblock_assembly(ctx, data, CASES[3][0], CASES[3][1], 2, 750, 6)


@pytest.mark.parametrize("world", [2, 8])
def test_column_block_assembly_n20000(ctx, world):
    """BASELINE configs[2]'s K (N=20000, float64 normalised) assembled from column blocks
    (gather = 6) equals the single-call K bit for bit."""
    n = 20000
    codes, lens = E.synthetic(n, 101, seed=3)
    params = P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        full = ctx.gram(params, codes, lens, L.KMG_F64)
        got = _colblock_assembly(ctx, (codes, lens, d_codes, d_lens), params, L.KMG_F64, world,
                                 -(-n // world), 6)
    finally:
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
    assert np.array_equal(got, full)


@pytest.mark.parametrize("n,world", [(1, 1), (3, 8), (17, 4)])
def test_column_block_assembly_tiny(ctx, n, world):
    """Column-block assembly at sizes where some ranks hold no column (n < world) and a
    single row: still the one-call K, spectrum and mismatch."""
    codes, lens = E.synthetic(n, 101, seed=90 + n)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        for params, dt in (CASES[0], CASES[1]):
            full = ctx.gram(params, codes, lens, dt)
            got = _colblock_assembly(ctx, (codes, lens, d_codes, d_lens), params, dt, world,
                                     -(-n // world), 6)
            assert np.array_equal(got, full), (n, world)
    finally:
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)
