"""GPU parity of the reference's module-level feature maps and the substring auxiliary
through the drop-in kernels.py (kmg_features, KMG_MODE_SS_B): get_phi_u, get_phi_km,
gappy_k, B_k / rec (kernels.py:12-25, 161-175, 308-342, 420-433).  Bit-exact against the
reference's own fixtures (tests/golden, round 4) and, at sizes the reference would take
minutes for, against the golden-pinned oracle restatements (tests/test_feature_maps_cpu.py).

Also the generic per-pair kernels (k > 16) on ragged rows and non-ACGT symbols, and
spectrum k > 16 with normalisation (round-3 advisor findings)."""
import numpy as np
import pytest

import cpu_ref
import feature_cases as F
import kernels as km
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prefix", F.PREFIXES)
def test_feature_fixtures_bit_exact(golden, prefix):
    done = 0
    for name in F.names(golden):
        if not name.startswith(prefix) or golden.entry(name)["error"]:
            continue
        got = np.asarray(F.call(km, golden, name), dtype=np.float64)
        ref = golden.K(name)
        assert got.shape == ref.shape and np.array_equal(got, ref), name
        done += 1
    assert done > 0


def test_phi_u_random_rows():
    rng = np.random.default_rng(41)
    betas = F.betas({"fn": "get_phi_u", "kwargs": {"k": 6, "betas": "canonical"}})
    for t in range(6):
        n = int(rng.integers(0, 300))
        x = "".join(rng.choice(list("ACGTN"), size=n, p=[0.24, 0.24, 0.24, 0.24, 0.04]))
        assert np.array_equal(km.get_phi_u(x, 6, betas), cpu_ref.phi_u(x, 6, betas)), t


@pytest.mark.parametrize("k,m", [(9, 1), (7, 2), (4, 0), (12, 3)])
def test_phi_km_random_rows(k, m):
    rng = np.random.default_rng(100 + k)
    x = rng.integers(1, 5, size=120)
    betas = rng.integers(1, 5, size=(3000, k))
    betas[:50] = np.stack([x[a:a + k] for a in range(50)])  # exact hits
    if k == 7:
        x[30] = 0  # a symbol outside 1..4 mismatches every letter
    got = km.get_phi_km(x, k, m, betas)
    assert np.array_equal(got, cpu_ref.phi_km(x, k, m, betas))
    assert got[:50].min() >= 1


def test_gappy_k_letters():
    x = F.fmt("ACCA" * 25 + "G" + "T" * 40)  # T only past x[0:101]
    b = np.array([[1], [2], [3], [4]])
    assert np.array_equal(km.gappy_k(x, 1, 0, b), np.array([1.0, 1.0, 1.0, 0.0]))


@pytest.mark.parametrize("lb,k", [(0.6, 5), (0.9, 9), (0.5, 12), (0.8, 1)])
def test_b_k_against_oracle(lb, k):
    rng = np.random.default_rng(k)
    for t in range(3):
        x = "".join(rng.choice(list("ACGT"), size=int(rng.integers(k, 70))))
        y = "".join(rng.choice(list("ACGT"), size=int(rng.integers(k, 70))))
        assert km.B_k(lb, k, x, y) == cpu_ref.ss_b(x, y, lb, k), (k, t)


def test_b_k_memoised_call_is_reused():
    a = km.B_k(0.5, 3, "ACGTTGCA", "GATTACA")
    assert km.B_k(0.5, 3, "ACGTTGCA", "GATTACA") is a


def test_mismatch_generic_ragged_and_non_acgt(ctx):
    """k > 16: rows shorter than the window and non-ACGT symbols make their windows invalid
    (weight 0), the same rule as the packed k <= 16 kernels; K_ii agrees with the
    off-diagonal entries (fused normalisation uses the same sums)."""
    rng = np.random.default_rng(7)
    parent = rng.integers(0, 4, size=101).astype(np.uint8)
    codes = np.tile(parent, (8, 1))
    for r in range(8):
        codes[r, rng.integers(0, 101, size=3)] = rng.integers(0, 4, size=3)
    lens = np.full(8, 101, dtype=np.int32)
    lens[2], lens[5] = 60, 20       # shorter than the window (and than k at row 5)
    codes[3, 40] = 11               # a non-ACGT symbol
    codes[2, 60:] = 0xEE            # padding bytes past the row must never be read
    for k, m in ((17, 1), (20, 2)):
        ref = cpu_ref.mismatch_raw_windows(codes, lens, k, m)
        # (the host path kmg_gram refuses rows shorter than the window, as the reference
        # does; the device-resident path takes them)
        raw = _gram_device(ctx, P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=0),
                           codes, lens, L.KMG_I32)
        assert np.array_equal(raw.astype(np.int64), ref), k
        assert ctx.last_plan()["formulation"] == "generic"
        Kn = _gram_device(ctx, P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=1),
                          codes, lens, L.KMG_F64)
        assert np.array_equal(Kn, cpu_ref.normalize(ref.astype(np.float64)), equal_nan=True)


def _gram_device(ctx, params, codes, lens, dt):
    n, ldc = codes.shape
    out = np.empty((n, n), dtype=L.DTYPES[dt])
    d_codes, d_lens, d_out = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes), ctx.dmalloc(out.nbytes)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(params, d_codes, d_lens, n, ldc, 0, n, dt, d_out, n)
        ctx.synchronize()
        ctx.d2h(out, d_out)
    finally:
        for x in (d_codes, d_lens, d_out):
            ctx.dfree(x)
    return out


def test_spectrum_generic_normalised(ctx):
    rng = np.random.default_rng(3)
    parent = rng.integers(0, 4, size=101).astype(np.uint8)
    codes = np.tile(parent, (10, 1))
    for r in range(10):
        codes[r, rng.integers(0, 101, size=4)] = rng.integers(0, 4, size=4)
    lens = np.full(10, 101, dtype=np.int32)
    raw = cpu_ref.spectrum_windows(codes, lens, 20)
    Kn = ctx.gram(P.make(L.KMG_SPECTRUM, k=20, normalize=1), codes, lens, L.KMG_F64)
    assert np.array_equal(Kn, cpu_ref.normalize(raw.astype(np.float64)))
    assert ctx.last_plan()["formulation"] == "generic"
