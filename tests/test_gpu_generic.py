"""GPU parity of the generic per-pair kernels (kmg_generic.hip) that lift round 2's parameter
limits: spectrum and mismatch k > 16 (the packed kernels hold a k-mer in 32 bits), WDS
S > 15 and WD / WDS rows longer than 256 symbols.  Bit-exact against the oracle.

For spectrum / mismatch past k = 16 the reference itself cannot run (get_spectrum_K /
get_mismatch_K build all 4^k betas: 17e9 strings at k = 17), so parity there is pinned
through the oracle restatements only: cpu_ref.spectrum_windows equals the golden-pinned
Phi Phi^T form for k <= 12 (tests/test_oracle_generic.py), and cpu_ref.mismatch_raw is
the golden-pinned closed form, checked against explicit window pairs at k = 17."""
import numpy as np
import pytest

import cpu_ref
import cref
from golden_io import load_xtr0
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P

pytestmark = pytest.mark.gpu


def _related(n, L_, seed, nsub=3):
    """Rows that share long stretches (mutated copies of a few parents), so k > 16 windows
    actually match across rows."""
    rng = np.random.default_rng(seed)
    parents = rng.integers(0, 4, size=(4, L_)).astype(np.uint8)
    codes = parents[rng.integers(0, 4, size=n)].copy()
    for r in range(n):
        pos = rng.integers(0, L_, size=nsub)
        codes[r, pos] = rng.integers(0, 4, size=nsub)
    return codes, np.full(n, L_, dtype=np.int32)


@pytest.mark.parametrize("k", [17, 24, 40, 101])
def test_spectrum_k_past_16(ctx, k):
    codes, lens = _related(40, 101, seed=k)
    codes[3, 50] = 9            # a non-ACGT symbol: windows over it match nothing
    lens[6], lens[7] = 60, 16   # ragged rows (one shorter than k for k > 16)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=k), codes, lens, L.KMG_I32)
    ref = cpu_ref.spectrum_windows(codes, lens, k)
    assert np.array_equal(K.astype(np.int64), ref)
    assert ref[0, 1:].any() or k == 101  # the test rows do share windows
    # rows of another call (no mirror): the same values
    n, ldc = codes.shape
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(9 * n * 4)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(P.make(L.KMG_SPECTRUM, k=k), d_codes, d_lens, n, ldc, 11, 20, L.KMG_I32,
                        d_out, n)
        ctx.synchronize()
        rows = np.empty((9, n), dtype=np.int32)
        ctx.d2h(rows, d_out)
    finally:
        for x in (d_codes, d_lens, d_out):
            ctx.dfree(x)
    assert np.array_equal(rows, K[11:20])


@pytest.mark.parametrize("k,m", [(17, 1), (20, 2), (24, 3)])
def test_mismatch_k_past_16(ctx, k, m):
    codes, lens = _related(30, 101, seed=100 + k)
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=0), codes, lens,
                   L.KMG_I32)
    ref = cpu_ref.mismatch_raw(codes, lens, k, m)
    assert np.array_equal(raw.astype(np.int64), ref)
    Kn = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=1), codes, lens,
                  L.KMG_F64)
    assert np.array_equal(Kn, cpu_ref.normalize(ref.astype(np.float64)))


@pytest.mark.parametrize("d,S", [(4, 16), (5, 25), (3, 40)])
def test_wds_shifts_past_15(ctx, d, S):
    codes, lens = load_xtr0()
    codes, lens = codes[:40].copy(), lens[:40].copy()
    lens[4] = 101 - 3   # ragged: the clipped-suffix matches of len(y) = len(x) - s
    codes[4, :98] = codes[5, 3:101]
    K = ctx.gram(P.make(L.KMG_WDS, d=d, S=S), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.wds(codes, lens, d, S))


@pytest.mark.parametrize("kind", ["wd", "wds"])
def test_wd_wds_rows_past_256(ctx, kind):
    codes, lens = _related(24, 300, seed=7, nsub=20)
    lens[2] = 290
    if kind == "wd":
        K = ctx.gram(P.make(L.KMG_WD, d=6), codes, lens, L.KMG_F64)
        assert np.array_equal(K, cref.wd(codes, lens, 6))
    else:
        K = ctx.gram(P.make(L.KMG_WDS, d=4, S=5), codes, lens, L.KMG_F64)
        assert np.array_equal(K, cref.wds(codes, lens, 4, 5))
