"""Row distribution of the Gram matrix across ranks (one process per GPU).

Every (i, j) entry depends only on the replicated input and the replicated posting
index, so the N x N tile space splits by rows with no exchange until the
final assembly.  Two layouts:

* contiguous slabs (`even_splits`): rank r computes rows [splits[r], splits[r+1]); used
  by `store.gram_to_npy` and `kmg_allgather_rows`.
* block-cyclic (`block_cyclic_ranges`, the kmg_gram_blocks layout): round t holds rows
  [t*R, (t+1)*R), R = world * block, and rank r owns the block [t*R + r*block, +block).
  Each round is one contiguous R-row slab whose blocks sit in rank order, so assembling
  it on every rank is ONE in-place all-gather (send = recv + rank * count) and the
  rounds pipeline: round t is gathered while round t+1 is computed.
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


def rows_padded(n, world, block):
    """Rows of the gather buffer: whole rounds of world * block rows (kmg_rows_padded)."""
    if n <= 0:
        return 0
    r = world * block
    return -(-n // r) * r


def block_cyclic_ranges(n, world, rank, block):
    """[(row0, row1)] of this rank, one per round (clipped to n; may be empty)."""
    if world < 1 or not 0 <= rank < world or block < 1:
        raise ValueError("bad world / rank / block")
    r = world * block
    out = []
    for t in range(-(-n // r) if n > 0 else 0):
        a = min(n, t * r + rank * block)
        out.append((a, min(n, a + block)))
    return out


def round_slab(t, world, block):
    """Rows [t*R, (t+1)*R) of round t: the in-place all-gather target of that round."""
    r = world * block
    return t * r, (t + 1) * r


def default_block(n, world, row_bytes, target_bytes=256 << 20, min_rows=256):
    """Rows per block so one round (world blocks) moves about target_bytes, and there are
    at least 4 rounds to pipeline when the matrix allows it; but at least min_rows rows (or
    the rank's whole share), so a round's Gram launch still fills the GPU (N=100000, G=8:
    80-row blocks made 157 launches of 400 workgroups; collective-free 1.6 ms)."""
    if n <= 0:
        return 1
    b = max(1, target_bytes // max(1, world * row_bytes))
    b = min(b, max(1, -(-n // (4 * world))))
    b = max(b, min(min_rows, -(-n // world)))
    if b >= 8:
        b -= b % 8  # round starts stay multiples of 8 (the upper-triangle slabs' first column)
    return int(b)


def triangle_rounds(n, world, block):
    """Upper-triangle layout (kmg_gram_blocks gather = 2): [(c0, w)] per round, the round's
    first row c0 = t * R and the slab width w = n - c0 (columns >= c0 of its rows)."""
    r = world * block
    return [(t * r, n - t * r) for t in range(-(-n // r) if n > 0 else 0)]


def assemble_upper_triangle(slabs, n, world, block, dtype):
    """Host restatement of the gather = 2 assembly: slabs[t] is round t's gathered slab
    (world * block rows x w_t columns, rank q's block at rows q * block); returns K with
    K[c0 + i][c0 + j] = slab[i][j] and the mirror K[x][c0 + y] = slab[y][x - c0] for
    x >= c0 + R.  Used by the world-size-2 gloo test against the one-rank K."""
    import numpy as np
    K = np.zeros((n, n), dtype=dtype)
    r = world * block
    for (c0, w), S in zip(triangle_rounds(n, world, block), slabs):
        rows = min(r, n - c0)
        K[c0:c0 + rows, c0:] = S[:rows, :w]
        if c0 + r < n:
            K[c0 + r:, c0:c0 + r] = S[:r, r:w].T
    return K


XGMI_LINK_GBPS = 76.5  # one xGMI link, one direction (MI355X: 7 links per GPU, point to point)


def scaling_projection(n, t1_ms, t_index_ms, t_gram_ms, fill_gbps, out_bytes, wire_bytes,
                       chunk=None, worlds=(2, 4, 8), link_gbps=XGMI_LINK_GBPS, link_eff=1.0):
    """Predicted G-GPU times of one full-K build from one-GPU measurements.

    Two builds are modelled:
    * ``every_gpu`` (K complete on every GPU; kmg_gram_blocks gather = 2):
      compute = index + the rank's share of the upper-triangle Gram work (whole column
      chunks at or right of each round's first row, ``chunk`` columns per chunk);
      receive = the round slabs' (G-1)/G share over the G-1 point-to-point links into
      each GPU (fully connected xGMI: S / (G * link)); unpack = every GPU writes the
      whole K (n^2 * out_bytes) and reads the slabs at the measured fill rate.  The three
      run on separate streams, so t = max(stages) + one round of the largest stage
      (pipeline fill).
    * ``collective_free``: every GPU builds the index and its own rows only (the sharded
      reference loop, kernels.py:41-45 / 211-215, without the assembly): index + gram / G.

    Returns {G: {...}} with times in ms and speedups against t1_ms (the measured one-GPU
    build).  Assumptions are in the arguments: link_gbps per link and direction, link_eff
    the fraction of it an all-gather reaches (1.0: upper bound, not measured)."""
    chunk = chunk or n
    out = {}
    nn = float(n) * n
    for g in worlds:
        block = default_block(n, g, n * out_bytes)
        rounds = triangle_rounds(n, g, block)
        r = g * block
        work = slab = 0.0
        for c0, w in rounds:
            rows = min(r, n - c0)
            work += rows * (n - (c0 // chunk) * chunk)
            slab += r * w
        compute = t_index_ms + t_gram_ms * (work / nn) / g
        recv = slab * wire_bytes / (g * link_gbps * link_eff * 1e9) * 1e3
        unpack = (nn * out_bytes + slab * wire_bytes) / (fill_gbps * 1e9) * 1e3
        stages = {"compute_ms": compute, "receive_ms": recv, "unpack_ms": unpack}
        t_every = max(stages.values()) + max(stages.values()) / max(1, len(rounds))
        t_cf = t_index_ms + t_gram_ms / g
        out[g] = {"block_rows": block, "rounds": len(rounds), **stages,
                  "bytes_received_per_gpu": slab * wire_bytes * (g - 1) / g,
                  "bound": max(stages, key=stages.get).replace("_ms", ""),
                  "every_gpu_ms": t_every, "every_gpu_speedup": t1_ms / t_every,
                  "collective_free_ms": t_cf, "collective_free_speedup": t1_ms / t_cf}
    return out


def u8_slab_escapes(counts, row0, col0):
    """Restatement of the uint8 round-slab form the Gram kernels write (kmg_rowacc.h
    emit_row, KMG_U8, with an escape list): `counts` holds rows row0.. at columns col0..;
    the diagonal column is stored as 0 (the unpack takes K_ii from the locally computed
    diagonal) and an off-diagonal count >= 255 is stored as the escape byte 255 plus a
    (row, column, count) entry.  Returns (slab uint8, escapes int64 [m, 3])."""
    import numpy as np
    c = np.asarray(counts, dtype=np.int64)
    rows = np.arange(c.shape[0])[:, None] + row0
    cols = np.arange(c.shape[1])[None, :] + col0
    diag = rows == cols
    esc = (c >= 255) & ~diag
    slab = np.where(diag, 0, np.minimum(c, 255)).astype(np.uint8)
    r, q = np.nonzero(esc)
    return slab, np.stack([r + row0, q + col0, c[r, q]], axis=1).astype(np.int64)


def patch_escapes(K, escapes):
    """Escape entries (row, column, count) into K and its mirror (kmg_gram.hip
    tri_patch8_kernel)."""
    for r, c, v in escapes:
        K[r, c] = v
        K[c, r] = v
    return K
