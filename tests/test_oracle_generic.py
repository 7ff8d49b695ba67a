"""CPU checks of the oracle restatements behind the generic per-pair kernels (k > 16): the
window-counting spectrum equals the golden-pinned Phi Phi^T form where both apply."""
import numpy as np
import pytest

import cpu_ref
from golden_io import load_xtr0


@pytest.mark.parametrize("k", [1, 4, 8, 12])
def test_spectrum_windows_equals_phi_form(k):
    codes, lens = load_xtr0()
    codes, lens = codes[:24].copy(), lens[:24].copy()
    codes[3, 10] = 7   # a non-ACGT symbol: the windows over it match nothing
    lens[5] = 30       # a ragged row
    assert np.array_equal(cpu_ref.spectrum_windows(codes, lens, k), cpu_ref.spectrum(codes, lens, k))


def test_mismatch_raw_past_k16_matches_bruteforce_definition():
    """cpu_ref.mismatch_raw's closed form at k = 17 against sum_{a,b} w[ham] written out
    over explicit window pairs (the definition kernels.py:161-175 reduces to)."""
    rng = np.random.default_rng(5)
    codes = rng.integers(0, 4, size=(4, 101)).astype(np.uint8)
    codes[1, :60] = codes[0, :60]
    codes[1, 7] ^= 1
    lens = np.full(4, 101, dtype=np.int32)
    k, m = 17, 2
    w = cpu_ref.mismatch_weights(k, m)
    P = 101 - k + 1
    K = cpu_ref.mismatch_raw(codes, lens, k, m)
    for i in range(4):
        for j in range(4):
            Wi = np.stack([codes[i, a:a + k] for a in range(P)])
            Wj = np.stack([codes[j, b:b + k] for b in range(P)])
            H = (Wi[:, None, :] != Wj[None, :, :]).sum(axis=2)
            assert K[i, j] == int(w[H].sum())
