"""Row sharding of the Gram matrix across ranks (one process per GPU).

Every (i, j) entry depends only on the replicated input and the replicated posting
index, so rank r computes rows [splits[r], splits[r+1]) against all N columns with no
exchange; `gather` (RCCL, kmg_allgather_rows) assembles the full K on every rank when
the caller needs it.
"""
import math


def even_splits(n, parts):
    """Row boundaries giving every rank floor/ceil(n/parts) rows."""
    if parts < 1:
        raise ValueError("parts must be >= 1")
    return [n * r // parts for r in range(parts + 1)]


def weak_scaled_n(n1, world, align=8):
    """N such that each of `world` ranks computes about n1^2 Gram pairs (rows N/world x
    N columns): N = n1 * sqrt(world), rounded to a multiple of `align`."""
    if world <= 1:
        return n1
    return int(round(n1 * math.sqrt(world) / align)) * align


def rank_rows(n, world, rank):
    s = even_splits(n, world)
    return s[rank], s[rank + 1]
