"""Gappy (k, g) with the semantics the reference intends (kernels.py:420-455, report §3.7).

The reference's get_gappy_K raises for every (k, g) but (1, 0) under numpy 2 (betas are
k-mers but gap_set holds (k-g)-tuples), so this kernel is PARITY UNPINNED: the CPU tests
pin the oracle restatement (oracle/cpu_ref.py gappy_intended) against a second
restatement that follows the reference's own loop with the single fix (betas over
(k-g)-mers, compared as tuples), and against the one case the reference does compute
(k=1, g=0, cpu_ref.gappy_k1g0, itself pinned to the reference's golden output).  The GPU
tests check the device path against the oracle bit for bit."""
from itertools import combinations, product

import numpy as np
import pytest

import cpu_ref
from kmgram import encode as E


def _reference_loop_fixed(codes, lens, k, g):
    """gappy_k / get_gappy_K (kernels.py:420-454) with betas = product('ACGT', k-g)."""
    seqs = [tuple(int(v) for v in codes[i, :lens[i]]) for i in range(len(lens))]
    betas = list(product(range(4), repeat=k - g))
    phis = []
    for x in seqs:
        gap_set = sum([list(combinations(x[i:i + k], k - g)) for i in range(101 - k + 1)], [])
        gs = set(gap_set)
        phis.append(np.array([1.0 if b in gs else 0.0 for b in betas]))
    n = len(seqs)
    K = np.zeros((n, n))
    for i in range(n):
        for j in range(i, n):
            K[i, j] = np.dot(phis[i], phis[j])
            K[j, i] = K[i, j]
    return cpu_ref.normalize(K)


@pytest.mark.parametrize("k,g", [(1, 0), (2, 1), (3, 1), (4, 2), (5, 1)])
def test_oracle_matches_fixed_reference_loop(k, g):
    codes, lens = E.synthetic(7, 101, seed=k * 10 + g)
    assert np.array_equal(cpu_ref.gappy_intended(codes, lens, k, g),
                          _reference_loop_fixed(codes, lens, k, g))


def test_oracle_k1g0_is_the_reference_gappy():
    codes, lens = E.synthetic(9, 120, seed=3)
    codes[2, :101] = 0  # a one-letter window set
    assert np.array_equal(cpu_ref.gappy_intended(codes, lens, 1, 0), cpu_ref.gappy_k1g0(codes, lens))


@pytest.mark.gpu
@pytest.mark.parametrize("k,g", [(1, 0), (3, 1), (5, 2), (6, 1), (8, 2), (9, 3)])
def test_gpu_gappy_intended_bitexact(engine, k, g):
    codes, lens = E.synthetic(70, 101, seed=k + 100 * g)
    codes[5] = 0  # homopolymer: a single feature
    K = engine.gappy(E.decode(codes, lens), k, g, intended=True)
    assert np.array_equal(K, cpu_ref.gappy_intended(codes, lens, k, g))


@pytest.mark.gpu
def test_gpu_gappy_intended_validation(engine):
    seqs = E.decode(*E.synthetic(4, 101, seed=1))
    with pytest.raises(ValueError):
        engine.gappy(seqs, 3, 3, intended=True)
    with pytest.raises(ValueError):
        engine.gappy(seqs[:3] + [seqs[3][:90]], 3, 1, intended=True)
    with pytest.raises(ValueError):  # reference semantics unchanged
        engine.gappy(seqs, 3, 1)
