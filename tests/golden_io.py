"""Readers for the committed golden fixtures (tests/golden/, made by make_golden.py and
make_inputs.py from the unmodified reference kernels.py in the build container)."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha256_f64(K):
    return hashlib.sha256(np.ascontiguousarray(np.asarray(K, dtype=np.float64)).tobytes()).hexdigest()


class Golden:
    def __init__(self):
        self.meta = json.load(open(os.path.join(GOLDEN, "golden_meta.json")))
        z = np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False)
        self.arrays = {k: z[k] for k in z.files}

    def names(self, prefix=""):
        return sorted(k for k in self.meta if k.startswith(prefix))

    def seqs(self, name):
        return [str(s) for s in self.arrays[self.meta[name]["seqs"]]]

    def K(self, name):
        return self.arrays[name]

    def entry(self, name):
        return self.meta[name]


def load_xtr0():
    """Data/Xtr0.csv of the reference as uint8 codes (2000, 101)."""
    z = np.load(os.path.join(GOLDEN, "xtr0_codes.npz"), allow_pickle=False)
    n, L = int(z["n"]), int(z["L"])
    bits = np.unpackbits(z["packed"], axis=1)[:, : 2 * L].reshape(n, L, 2)
    codes = (bits[..., 0] * 2 + bits[..., 1]).astype(np.uint8)
    return codes, np.full(n, L, dtype=np.int32)
