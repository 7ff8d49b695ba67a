"""Host-side encoding of DNA sequences into the symbol codes the C ABI takes.

'A','C','G','T' -> 0,1,2,3 (the itertools.product('ACGT') order of the reference's
betas, kernels.py:37,206).  Every other character gets a distinct code >= 4, so the
character-equality kernels (WD, WDS, SS: string slices compared with ==,
kernels.py:79,133,341) keep their semantics, while the spectrum kernel treats any
k-mer holding such a code as matching no beta (kernels.py:23-24).
"""
import numpy as np

ACGT = "ACGT"
_LUT = np.full(128, 255, dtype=np.uint8)
for _c in range(128):
    _LUT[_c] = 4 + _c  # distinct code per non-ACGT ASCII character (4..131)
for _i, _c in enumerate(ACGT):
    _LUT[ord(_c)] = _i


def as_sequence_list(X):
    """The reference reads only ``X.loc[:, 'seq']`` (kernels.py:39,94,149,208,287,377,447)."""
    if hasattr(X, "loc") and hasattr(X, "columns"):
        return [str(s) for s in X.loc[:, "seq"]]
    if isinstance(X, str):
        raise TypeError("expected a DataFrame with a 'seq' column or a sequence of strings")
    return [str(s) for s in X]


def encode(seqs, ldc_align=4):
    """Encode a list of str into (codes uint8[n, ldc], lens int32[n])."""
    seqs = list(seqs)
    n = len(seqs)
    lens = np.fromiter((len(s) for s in seqs), dtype=np.int64, count=n)
    maxlen = int(lens.max()) if n else 0
    ldc = max(ldc_align, -(-maxlen // ldc_align) * ldc_align)
    codes = np.full((n, ldc), 255, dtype=np.uint8)
    if n == 0 or maxlen == 0:
        return codes, lens.astype(np.int32)
    joined = "".join(seqs)
    try:
        raw = np.frombuffer(joined.encode("ascii"), dtype=np.uint8)
        vals = _LUT[raw]
    except UnicodeEncodeError:
        cps = np.frombuffer(joined.encode("utf-32-le"), dtype=np.uint32)
        vals = np.empty(cps.shape, dtype=np.uint8)
        ascii_mask = cps < 128
        vals[ascii_mask] = _LUT[cps[ascii_mask]]
        other = np.unique(cps[~ascii_mask])
        if len(other) > 123:  # codes 132..254: 255 stays the padding code
            raise ValueError("more than 123 distinct non-ASCII characters in the input")
        remap = {int(c): 132 + t for t, c in enumerate(other)}
        vals[~ascii_mask] = np.array([remap[int(c)] for c in cps[~ascii_mask]], dtype=np.uint8)
    rows = np.repeat(np.arange(n), lens)
    starts = np.concatenate(([0], np.cumsum(lens)[:-1]))
    cols = np.arange(len(vals)) - np.repeat(starts, lens)
    codes[rows, cols] = vals
    return codes, lens.astype(np.int32)


def is_acgt_only(codes, lens):
    """True if every symbol inside each sequence is one of A,C,G,T."""
    if codes.size == 0:
        return True
    mask = np.arange(codes.shape[1])[None, :] < lens[:, None]
    return bool(np.all(codes[mask] < 4))


def synthetic(n, length=101, seed=0, p=None):
    """i.i.d. synthetic DNA as codes (SURVEY 8d generator:
    default_rng(seed).integers(0, 4, size=(N, L), dtype=uint8))."""
    rng = np.random.default_rng(seed)
    if p is None:
        codes = rng.integers(0, 4, size=(n, length), dtype=np.uint8)
    else:
        codes = rng.choice(4, size=(n, length), p=p).astype(np.uint8)
    return codes, np.full(n, length, dtype=np.int32)


def decode(codes, lens):
    return ["".join(ACGT[c] if c < 4 else "N" for c in codes[i, :lens[i]]) for i in range(len(lens))]
