"""Inputs of the feature-map goldens (tests/golden/make_golden.py, round 4): rebuilds the
betas and arguments each PHIU / PHIKM / GAPK / BK fixture was made with, in the form the
reference's own callers pass them (kernels.py:37-40, 206-210, 446-449, 322-342)."""
from itertools import product

import numpy as np

PREFIXES = ("PHIU_", "PHIKM_", "GAPK_", "BK_")


def fmt(s):
    """kernels.format (kernels.py:187-193): 'A','C','G','T' -> 1..4, digits stay their value
    (the round-5 fixtures pass values outside 1..4 this way), anything else raises."""
    return np.array([int(c) for c in s.replace("A", "1").replace("C", "2").replace("G", "3")
                     .replace("T", "4")], dtype=np.int64)


def betas(entry):
    kw = entry["kwargs"]
    k = kw["k"]
    if "betas" not in kw:
        return None  # B_k
    if entry["fn"] == "get_phi_u":
        return ["".join(c) for c in product("ACGT", repeat=k)] if kw["betas"] == "canonical" \
            else list(kw["betas"])
    if kw["betas"] == "canonical":
        return np.array([fmt("".join(c)) for c in product("ACGT", repeat=k)])
    return np.array(kw["betas"])


def names(golden):
    return [n for n in golden.names() if n.startswith(PREFIXES)]


def call(mod, golden, name):
    """Call the module-level function of fixture `name` on `mod` (the drop-in kernels.py,
    or anything with the same functions) with the fixture's arguments."""
    e = golden.entry(name)
    kw = e["kwargs"]
    seqs = golden.seqs(name)
    if e["fn"] == "get_phi_u":
        return mod.get_phi_u(seqs[0], kw["k"], betas(e))
    if e["fn"] == "get_phi_km":
        return mod.get_phi_km(fmt(seqs[0]), kw["k"], kw["m"], betas(e))
    if e["fn"] == "gappy_k":
        return mod.gappy_k(fmt(seqs[0]), kw["k"], kw["g"], betas(e))
    return np.array([mod.B_k(kw["lbda"], kw["k"], seqs[0], seqs[1])], dtype=np.float64)
