"""CPU checks of the combination-consumer oracle (oracle/cpu_ref.py) that pin the fp64
operation order the device kernels reproduce (kmg_combine.hip)."""
import numpy as np
import pytest

import cpu_ref


def _kernels(n, p, seed):
    rng = np.random.default_rng(seed)
    out = []
    for m in range(p):
        A = rng.integers(1, 6, size=(n, 4 + m)).astype(np.float64)  # no zero rows: no 0/0
        out.append(cpu_ref.normalize(A @ A.T))
    return out


@pytest.mark.parametrize("degree", [1, 2])
def test_nlck_combine_is_sequential_slice_sum(degree):
    """np.sum(kernels * u[:, None, None], axis=0) (NLCKernels.py:52) adds the products
    slice after slice, and ** 2 is x * x: the order combine_kernel uses."""
    Ks = _kernels(70, 9, 1)
    u = np.random.default_rng(2).random(9)
    ref = cpu_ref.nlck_combine(Ks, u, degree)
    s = Ks[0] * u[0]
    for m in range(1, 9):
        s = s + Ks[m] * u[m]
    seq = s if degree == 1 else s * s
    assert np.array_equal(ref, seq)


def test_alignf_centring_identity():
    """(B K B)_ij = K_ij - r_i - c_j + t (center_K, kernels.py:387-395): the O(n^2) form
    alignf_rows_kernel uses, against the reference's multi_dot."""
    Ks = _kernels(50, 3, 3)
    for K in Ks:
        r = K.mean(axis=1)
        c = K.mean(axis=0)
        t = r.mean()
        fast = (K - (r - t)[:, None]) - c[None, :]
        assert np.allclose(fast, cpu_ref.center(K), rtol=0, atol=1e-12)


def test_sparse_comparator_matches_oracle():
    """The scipy-sparse Phi Phi^T CPU comparator (bench.py cpu_baseline) equals the C oracle."""
    import cref
    from kmgram import encode as E
    codes, lens = E.synthetic(120, 101, seed=4)
    F = cpu_ref.spectrum_phi(codes, lens, 8)
    assert np.array_equal((F @ F.T).toarray(), cref.spectrum(codes, lens, 8))
    G = cpu_ref.mismatch_phi(codes, lens, 9, 1)
    assert np.array_equal((G[:30] @ G.T).toarray(), cref.mismatch_raw(codes, lens, 9, 1, rows=(0, 30)))
    rng = np.random.default_rng(5)
    seqs = ["".join(rng.choice(list("ACGTN"), size=rng.integers(0, 60))) for _ in range(50)]
    c2, l2 = E.encode(seqs)
    F2 = cpu_ref.spectrum_phi(c2, l2, 3)
    assert np.array_equal((F2 @ F2.T).toarray(), cref.spectrum(c2, l2, 3))
