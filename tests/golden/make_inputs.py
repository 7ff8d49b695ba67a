"""Store the reference's Data/Xtr0.csv sequences (2,000 x 101, ACGT only) as uint8 codes
(A,C,G,T = 0..3) so the config-1 parity test can run where /root/reference is absent.
Run by hand in the build container: python tests/golden/make_inputs.py"""
import hashlib
import os

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
CSV = "/root/reference/Data/Xtr0.csv"

df = pd.read_csv(CSV)
seqs = list(df["seq"])
L = {len(s) for s in seqs}
assert L == {101}, L
lut = {c: i for i, c in enumerate("ACGT")}
codes = np.array([[lut[c] for c in s] for s in seqs], dtype=np.uint8)
packed = np.packbits(np.unpackbits(codes[..., None], axis=-1)[..., 6:].reshape(len(seqs), -1), axis=1)
np.savez_compressed(os.path.join(HERE, "xtr0_codes.npz"), packed=packed, n=len(seqs), L=101,
                    csv_sha256=hashlib.sha256(open(CSV, "rb").read()).hexdigest())
print(codes.shape, packed.shape)
