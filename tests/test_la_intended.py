"""Local-alignment kernel with the intended recurrence (KMG_LA_INTENDED; the reference's
affine_align / Smith_Waterman, kernels.py:226-270, with the one-array aliasing, the
range(1, n) loop bounds and the positive gap exponents fixed).  Parity unpinned: the
reference itself always returns zeros.  The oracle (cpu_ref.la_intended_pair) is checked
against a second, array-based restatement and a hand-computed case on the CPU; the
device kernel is checked against the oracle on the GPU."""
import math

import numpy as np
import pytest

import cpu_ref
from kmgram import encode as E

S = cpu_ref.LA_S


def _la_arrays(x, y, e, d, beta, smith):
    """Second restatement: the reference's code shape (five (n+1) x (n+1) arrays, double
    loop) with the three fixes, written independently of la_intended_pair."""
    nx, ny = len(x), len(y)
    M, X, Y, X2, Y2 = (np.zeros((nx + 1, ny + 1)) for _ in range(5))
    op, ex = math.exp(-beta * e), math.exp(-beta * d)
    for i in range(1, nx + 1):
        for j in range(1, ny + 1):
            f = math.exp(beta * float(S[x[i - 1], y[j - 1]]))
            if smith:
                M[i, j] = f * max(1.0, X[i - 1, j - 1], Y[i - 1, j - 1], M[i - 1, j - 1])
                X[i, j] = max(op * M[i - 1, j], ex * X[i - 1, j])
                Y[i, j] = max(op * M[i, j - 1], op * X[i, j - 1], ex * Y[i, j - 1])
                X2[i, j] = max(M[i - 1, j], X2[i - 1, j])
                Y2[i, j] = max(M[i, j - 1], X2[i, j - 1], Y2[i, j - 1])
            else:
                M[i, j] = f * (1.0 + X[i - 1, j - 1] + Y[i - 1, j - 1] + M[i - 1, j - 1])
                X[i, j] = op * M[i - 1, j] + ex * X[i - 1, j]
                Y[i, j] = op * (M[i, j - 1] + X[i, j - 1]) + ex * Y[i, j - 1]
                X2[i, j] = M[i - 1, j] + X2[i - 1, j]
                Y2[i, j] = M[i, j - 1] + X2[i, j - 1] + Y2[i, j - 1]
    v = (max(1.0, X2[nx, ny], Y2[nx, ny], M[nx, ny]) if smith
         else 1.0 + X2[nx, ny] + Y2[nx, ny] + M[nx, ny])
    return (1 / beta) * math.log(v)


def test_la_oracle_hand_case():
    # x = y = "A": only M[1,1] = exp(4 beta) is non-zero at the corner
    assert cpu_ref.la_intended_pair([0], [0], 11, 1, 0.5, 0) == (1 / 0.5) * math.log(1.0 + math.exp(2.0))
    assert cpu_ref.la_intended_pair([0], [0], 11, 1, 0.5, 1) == (1 / 0.5) * math.log(math.exp(2.0))
    assert cpu_ref.la_intended_pair([], [1, 2], 11, 1, 0.5, 0) == 0.0


@pytest.mark.parametrize("smith", [0, 1])
@pytest.mark.parametrize("e,d,beta", [(11, 1, 0.5), (5, 2, 0.2), (3, 3, 1.0)])
def test_la_oracle_two_restatements(smith, e, d, beta):
    rng = np.random.default_rng(5 + smith)
    for _ in range(6):
        x = rng.integers(0, 4, rng.integers(1, 30))
        y = rng.integers(0, 4, rng.integers(1, 30))
        a = cpu_ref.la_intended_pair(list(x), list(y), e, d, beta, smith)
        b = _la_arrays(x, y, e, d, beta, smith)
        assert a == b


def test_la_oracle_properties():
    codes, lens = E.synthetic(5, 60, seed=8)
    K = cpu_ref.la_intended(codes, lens)
    Ks = cpu_ref.la_intended(codes, lens, smith=1)
    assert np.all(Ks <= K + 1e-9)          # max over alignments <= log(1 + sum)
    assert np.all(np.diag(K) >= K.max(axis=1) - 1e-9)  # a sequence aligns best to itself here
    assert np.array_equal(K, K.T)


@pytest.mark.gpu
@pytest.mark.parametrize("smith", [0, 1])
@pytest.mark.parametrize("e,d,beta", [(11, 1, 0.5), (5, 2, 0.2)])
def test_gpu_la_intended_vs_oracle(engine, smith, e, d, beta):
    """Device DP = oracle to the last ulp of log (every DP sum is evaluated in the
    oracle's order without FMA; only the final log may differ by an ulp): rows of
    length 0..101 (ragged), an all-C row (large exponents)."""
    codes, lens = E.synthetic(11, 101, seed=31)
    lens[2], lens[5], lens[7] = 40, 1, 0
    codes[9, :] = 1
    seqs = E.decode(codes, lens)
    got = engine.local_alignment(seqs, e, d, beta, smith, eig=1, intended=True)
    ref = cpu_ref.la_intended(codes, lens, e, d, beta, smith)
    assert got.shape == ref.shape and np.all(np.isfinite(got))
    np.testing.assert_allclose(got, ref, rtol=4e-16, atol=0)


@pytest.mark.gpu
def test_gpu_la_intended_rows(engine, ctx):
    """A row range [row0, row1) of the intended LA (no mirror) equals those rows of the
    full build."""
    from kmgram import _lib as L
    from kmgram import params as P
    codes, lens = E.synthetic(40, 101, seed=32)
    lens[::7] = 77
    p = P.make(L.KMG_LOCALALIGN, smith=0, la_mode=L.KMG_LA_INTENDED, la_e=11, la_d=1,
               la_beta=0.5)
    full = ctx.gram(p, codes, lens, L.KMG_F64)
    n, ldc = codes.shape
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(13 * n * 8)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(p, d_codes, d_lens, n, ldc, 9, 22, L.KMG_F64, d_out, n)
        ctx.synchronize()
        rows = np.empty((13, n))
        ctx.d2h(rows, d_out)
    finally:
        for x in (d_codes, d_lens, d_out):
            ctx.dfree(x)
    assert np.array_equal(rows, full[9:22])


@pytest.mark.gpu
def test_gpu_la_intended_rejects_non_acgt(ctx):
    """The substitution matrix covers A/C/G/T only (kernels.py:223): a row holding another
    symbol is KMG_EINVAL through the C ABI (host and device-resident rows), not a read past
    the 16-entry table."""
    from kmgram import _lib as L
    from kmgram import params as P
    codes, lens = E.synthetic(9, 101, seed=33)
    codes[4, 50] = 4  # 'N'
    p = P.make(L.KMG_LOCALALIGN, smith=0, la_mode=L.KMG_LA_INTENDED, la_e=11, la_d=1,
               la_beta=0.5)
    with pytest.raises(L.KmgError) as ei:
        ctx.gram(p, codes, lens, L.KMG_F64)
    assert ei.value.status == L.KMG_EINVAL
    n, ldc = codes.shape
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(n * n * 8)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        with pytest.raises(L.KmgError) as ei:
            ctx.gram_device(p, d_codes, d_lens, n, ldc, 0, n, L.KMG_F64, d_out, n)
        assert ei.value.status == L.KMG_EINVAL
        lens[4] = 50  # the N is past the row's length: accepted
        ctx.h2d(d_lens, lens)
        ctx.gram_device(p, d_codes, d_lens, n, ldc, 0, n, L.KMG_F64, d_out, n)
        ctx.synchronize()
    finally:
        for x in (d_codes, d_lens, d_out):
            ctx.dfree(x)


@pytest.mark.gpu
@pytest.mark.parametrize("smith", [0, 1])
@pytest.mark.parametrize("lmin,lmax", [(60, 103), (104, 127), (128, 250)])
def test_gpu_la_intended_lengths(engine, smith, lmin, lmax):
    """Every launch shape against the oracle: the grouped sweep with 8-lane groups (rows up
    to 103), 16-lane groups (up to 127), and the 64-row strip kernel beyond."""
    rng = np.random.default_rng(40 + lmax + smith)
    seqs = ["".join(rng.choice(list("ACGT"), size=int(rng.integers(lmin, lmax + 1))))
            for _ in range(9)]
    codes, lens = E.encode(seqs)
    got = engine.local_alignment(seqs, 11, 1, 0.2, smith, eig=1, intended=True)
    ref = cpu_ref.la_intended(codes, lens, 11, 1, 0.2, smith)
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, ref, rtol=4e-16, atol=0)


@pytest.mark.gpu
def test_gpu_la_intended_past_1024(engine):
    """Lengths past round 2's 1024 limit: the strip kernel with fewer pairs a block (the
    boundary rows of 1300 columns take 42 KB of LDS per pair).  Max form, small beta so the
    values stay finite."""
    rng = np.random.default_rng(77)
    seqs = ["".join(rng.choice(list("ACGT"), size=n)) for n in (1100, 1300)]
    codes, lens = E.encode(seqs)
    got = engine.local_alignment(seqs, 11, 1, 0.05, 1, eig=1, intended=True)
    ref = cpu_ref.la_intended(codes, lens, 11, 1, 0.05, 1)
    assert np.all(np.isfinite(got))
    np.testing.assert_allclose(got, ref, rtol=4e-16, atol=0)
