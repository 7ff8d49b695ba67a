"""GPU parity of the kernel-combination consumers (kmg_combine.hip) against the oracle's
restatement of the reference expressions (NLCKernels.py:52,61-66,97; ALIGNF.py:43-58).
degree 1 and 2 are bit-exact; pow() for degree >= 3 is within 4 ulp (tolerance below);
the gradient and alignment sums reduce in a different order than BLAS / numpy, so they
are checked to 1e-12 relative (north_star's float bound is 1e-6)."""
import numpy as np
import pytest

import cpu_ref
from kmgram import combine as C

pytestmark = pytest.mark.gpu


def _kernels(n, p, seed):
    rng = np.random.default_rng(seed)
    out = []
    for m in range(p):
        A = rng.integers(1, 6, size=(n, 4 + m)).astype(np.float64)  # no zero rows: no 0/0
        out.append(cpu_ref.normalize(A @ A.T))
    return out


@pytest.mark.parametrize("n,p", [(1, 1), (97, 3), (300, 9), (257, 12)])
@pytest.mark.parametrize("degree", [1, 2])
def test_nlck_combine_bitexact(engine, n, p, degree):
    Ks = _kernels(n, p, n + p)
    u = np.random.default_rng(p).random(p)
    assert np.array_equal(C.nlck_combine(Ks, u, degree), cpu_ref.nlck_combine(Ks, u, degree))


@pytest.mark.parametrize("degree", [3, 4])
def test_nlck_combine_pow(engine, degree):
    """run.py uses degree 3 and 4 (run.py:14,21,28)."""
    Ks = _kernels(300, 9, 5)
    u = np.random.default_rng(7).random(9)
    got, ref = C.nlck_combine(Ks, u, degree), cpu_ref.nlck_combine(Ks, u, degree)
    assert np.allclose(got, ref, rtol=4 * np.finfo(np.float64).eps, atol=0)


@pytest.mark.parametrize("degree", [1, 2, 3])
def test_nlck_grad(engine, degree):
    Ks = _kernels(400, 9, 11)
    rng = np.random.default_rng(13)
    u, alpha = rng.random(9), rng.standard_normal(400)
    got, ref = C.nlck_grad(Ks, u, degree, alpha), cpu_ref.nlck_grad(Ks, u, degree, alpha)
    assert np.allclose(got, ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("n,p", [(64, 1), (333, 9), (200, 12)])
def test_alignf_stats(engine, n, p):
    Ks = _kernels(n, p, 17 + p)
    y = np.random.default_rng(19).integers(0, 2, size=n).astype(np.float64)  # Bound in {0,1}
    a, M = C.alignf_stats(Ks, y)
    ra, rM = cpu_ref.alignf_stats(Ks, y)
    scale = max(np.abs(rM).max(), 1.0)
    assert np.allclose(a, ra, rtol=1e-9, atol=1e-9 * scale)
    assert np.allclose(M, rM, rtol=1e-9, atol=1e-9 * scale)
    assert np.array_equal(M, M.T)


def test_combine_rejects_too_many_kernels(engine):
    from kmgram import _lib as L
    Ks = _kernels(10, 13, 1)
    with pytest.raises(L.KmgUnsupported):
        C.nlck_combine(Ks, np.ones(13), 1)
