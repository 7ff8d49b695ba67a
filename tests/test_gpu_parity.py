"""GPU parity: every Gram kernel through the C ABI (and the drop-in kernels.py) against
the reference goldens and the oracle.  Integer kernels and the float64 kernels are
bit-exact (tolerance 0: north_star's 1e-6 relative bound is met with equality)."""
import numpy as np
import pandas as pd
import pytest

import cpu_ref
import cref
from golden_io import load_xtr0, sha256_f64
from kmgram import _lib as L
from kmgram import encode as E
from kmgram import params as P

pytestmark = pytest.mark.gpu


def _X(seqs):
    return pd.DataFrame({"Id": range(len(seqs)), "seq": list(seqs)})


# ------------------------------------------------------------------ goldens via kernels.py
def test_all_goldens_through_dropin(golden):
    import kernels
    fn_map = {
        "get_spectrum_K": kernels.get_spectrum_K, "get_mismatch_K": kernels.get_mismatch_K,
        "get_WD_K": kernels.get_WD_K, "get_WDShifts_K": kernels.get_WDShifts_K,
        "get_string_K": kernels.get_string_K, "get_LA_K": kernels.get_LA_K,
        "get_gappy_K": kernels.get_gappy_K, "select_method": kernels.select_method,
    }
    checked = 0
    for name in golden.names():
        if name == "SP_k6_xtr0_full":
            continue
        e = golden.entry(name)
        if e["fn"] in ("get_phi_u", "get_phi_km", "gappy_k", "B_k"):
            continue  # module-level feature maps: tests/test_gpu_features.py
        if e["fn"] in ("get_WD_d", "get_WDShifts_d"):  # one pair, any L
            x, y = golden.seqs(name)
            v = getattr(kernels, e["fn"])(x, y, **e["kwargs"])
            assert v == golden.K(name)[0], name
            checked += 1
            continue
        X = _X(golden.seqs(name))
        fn = fn_map[e["fn"]]
        if e["error"]:
            with pytest.raises(Exception) as ei:
                fn(X, **e["kwargs"])
            assert type(ei.value).__name__ == e["error"], name
        else:
            K = fn(X, **e["kwargs"])
            ref = golden.K(name)
            assert K.dtype == np.float64 and K.flags.c_contiguous, name
            assert np.array_equal(K, ref), name
            assert sha256_f64(K) == e["sha256_f64"], name
        checked += 1
    assert checked >= 150


def test_config1_spectrum_k6_xtr0_sha(golden):
    """BASELINE configs[0]: get_spectrum_K on Data/Xtr0.csv, k=6 — SHA-256 of the reference K."""
    import kernels
    codes, lens = load_xtr0()
    X = _X(E.decode(codes, lens))
    K = kernels.get_spectrum_K(X, 6)
    assert sha256_f64(K) == golden.entry("SP_k6_xtr0_full")["sha256_f64"]


# ------------------------------------------------------------------ synthetic, config sizes
def _row_sums_spectrum(codes, lens, k):
    """sum_j K_ij = sum_u phi_i(u) * T(u), T = total count of u over all sequences."""
    P_ = codes.shape[1] - k + 1
    km = np.zeros((codes.shape[0], P_), dtype=np.int64)
    for q in range(k):
        km = km * 4 + codes[:, q:q + P_]
    T = np.bincount(km.ravel(), minlength=4 ** k)
    return T[km].sum(axis=1)


def test_spectrum_k8_n20000(ctx):
    """BASELINE configs[1] workload: N=20000, L=101, k=8, int32 exact."""
    codes, lens = E.synthetic(20000, 101, seed=2)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=8), codes, lens, L.KMG_I32)
    for r in np.r_[0:8, 9990:10000, 19992:20000]:
        ref = cref.spectrum(codes, lens, 8, rows=(int(r), int(r) + 1))[0]
        assert np.array_equal(K[r].astype(np.int64), ref)
    # size-independent properties over the whole matrix
    assert np.array_equal(K, K.T)
    assert np.array_equal(K.sum(axis=1, dtype=np.int64), _row_sums_spectrum(codes, lens, 8))
    P_ = 101 - 8 + 1
    km = np.zeros((20000, P_), dtype=np.int64)
    for q in range(8):
        km = km * 4 + codes[:, q:q + P_]
    km.sort(axis=1)
    diag = [int((np.unique(row, return_counts=True)[1] ** 2).sum()) for row in km]
    assert np.array_equal(np.diag(K), np.array(diag))


def test_spectrum_homopolymer_max(ctx):
    """Maximum count: a poly-A row against itself = 94^2 = 8836 at k=8."""
    codes, lens = E.synthetic(64, 101, seed=3)
    codes[5] = 0
    codes[9] = 0
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=8), codes, lens, L.KMG_I32)
    assert K[5, 5] == 94 * 94 and K[5, 9] == 94 * 94
    assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, 8))


@pytest.mark.parametrize("k", [1, 3, 5, 6, 10, 12, 13, 16])
def test_spectrum_k_range(ctx, k):
    codes, lens = E.synthetic(300, 101, seed=k)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=k), codes, lens, L.KMG_I32)
    assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, k))


def test_spectrum_ragged_and_chunks(ctx, tune):
    rng = np.random.default_rng(5)
    seqs = ["".join(rng.choice(list("ACGTN"), p=[.24, .24, .24, .24, .04], size=rng.integers(0, 140)))
            for _ in range(700)]
    codes, lens = E.encode(seqs)
    ref = cref.spectrum(codes, lens, 4)
    for chunk in ("24576", "104", "256"):
        tune(KMG_SP_CHUNK=chunk, KMG_ALGO=2)
        K = ctx.gram(P.make(L.KMG_SPECTRUM, k=4), codes, lens, L.KMG_I32)
        assert np.array_equal(K.astype(np.int64), ref), chunk


def test_index_builds(ctx, tune):
    """The posting-index build (per-block local sort + per-bucket gather) gives bit-identical
    Grams over chunkings and partition block sizes."""
    tune(KMG_ALGO=2)
    codes, lens = E.synthetic(2500, 101, seed=91)
    codes[3] = 0
    ref = cref.spectrum(codes, lens, 8)
    for chunk, seqs_pb in (("24576", "80"), ("700", "7"), ("24576", "1")):
        tune(KMG_SP_CHUNK=chunk, KMG_IDX_SEQS=seqs_pb)
        K = ctx.gram(P.make(L.KMG_SPECTRUM, k=8), codes, lens, L.KMG_I32)
        assert np.array_equal(K.astype(np.int64), ref), (chunk, seqs_pb)
    c2, l2 = codes[:1200], lens[:1200]
    refm = cref.mismatch_raw(c2, l2, 9, 1)
    for seqs_pb in ("80", "7"):
        tune(KMG_IDX_SEQS=seqs_pb)
        raw = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), c2, l2, L.KMG_I32)
        assert np.array_equal(raw.astype(np.int64), refm), seqs_pb


def test_spectrum_long_sequences_unpacked(ctx):
    """P > 255: the 32-bit LDS accumulator variant."""
    codes, lens = E.synthetic(64, 400, seed=9)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=5), codes, lens, L.KMG_I32)
    assert np.array_equal(K.astype(np.int64), cref.spectrum(codes, lens, 5))


def _form(tune, form):
    """"F" -> KMG_MM_FORM=F; "4:T" also KMG_NB_THREADS=T (neighbourhood lists); "4:T:L" also
    KMG_NB_FILL=L (the list fill: 1 sorted + packed, 2 grouped lane-per-run, 3 piece-assembled,
    4 staged)"""
    f, _, rest = form.partition(":")
    t, _, fill = rest.partition(":")
    tune(KMG_MM_FORM=f, KMG_NB_THREADS=(t or None) if f == "4" else None,
         KMG_NB_FILL=(fill or None) if f == "4" else None)


@pytest.mark.parametrize("form", ["0", "4:1024:1", "4:1024:2", "4:512"])
def test_mismatch_k9_n20000(ctx, tune, form):
    """BASELINE configs[2] workload: N=20000 mismatch (9,1), float64 normalised, bit-exact rows
    (default formulation: the neighbourhood lists, 16-bit from the staged fill -- a list is
    read ~7 times here, too few to repay the packed segment 2's sort; the sorted fill with
    packed segments 2; the grouped fill; 512-thread workgroups)."""
    _form(tune, form)
    codes, lens = E.synthetic(20000, 101, seed=3)
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), codes, lens,
                 L.KMG_F64)
    plan = ctx.last_plan()
    assert plan["formulation"] == "neighbourhood"
    if form.startswith("4"):
        assert plan["threads"] == int(form.split(":")[1])
        assert plan["triangle"] == (plan["nchunks"] > 1)
        assert plan["packed"] == form.endswith(":1")
    else:                       # default at k = 9: one chunk, 16-bit lists
        assert (plan["threads"], plan["nchunks"], plan["triangle"], plan["packed"]) == (1024, 1, False, False)
    rows = [0, 1, 7777, 10000, 19999]
    for r in rows:
        ref = cref.mismatch_rows(codes, lens, 9, 1, rows=(r, r + 1))[0]
        assert np.array_equal(K[r], ref), r
    assert np.array_equal(K, K.T)
    assert np.all(np.diag(K) == 1.0)
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), codes[:3000],
                   lens[:3000], L.KMG_I32)
    assert np.array_equal(raw[:16].astype(np.int64), cref.mismatch_raw(codes[:3000], lens[:3000], 9, 1, rows=(0, 16)))


@pytest.mark.parametrize("k", [4, 8, 9, 12])
@pytest.mark.parametrize("fill", ["0", "1", "2", "3", "4"])
def test_mismatch_nb_fill_forms(ctx, tune, k, fill):
    """The neighbourhood-list fills (0 auto -- 16-bit from k = 8: 600 rows read a list < 16
    times --, 1 sorted with a packed segment 2, 2 grouped lane-per-run, 3 piece-
    assembled, 4 staged 16-bit lists) build lists of the same K: raw K bit-exact
    over several column chunkings; 40 poly-A rows make lists past every LDS buffer.  The
    sorted fill refuses (KMG_EUNSUPPORTED) where segment 2 is too sparse to pack (k = 12);
    elsewhere forcing it caps the chunk at the buffer's size (k = 4: ~130 columns)."""
    codes, lens = E.synthetic(600, 101, seed=90 + k)
    codes[:40] = 0  # poly-A rows: long runs, groups past the LDS image
    ref = cref.mismatch_raw(codes, lens, k, 1)
    tune(KMG_MM_FORM=4, KMG_NB_FILL=fill)
    for chunk in (("96", "20480") if k < 12 else ("20480",)):  # (k = 12: 4^12 bins a chunk)
        tune(KMG_MM_CHUNK=chunk)
        params = P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0)
        if fill == "1" and k == 12:  # ~300 columns between Hamming-2 entries: no packing
            with pytest.raises(L.KmgError, match="sorted fill"):
                ctx.gram(params, codes, lens, L.KMG_I32)
            continue
        raw = ctx.gram(params, codes, lens, L.KMG_I32)
        assert np.array_equal(raw.astype(np.int64), ref), chunk
        if fill == "0" and k >= 8:  # a list read 600 x 94 / 4^k < 16 times: 16-bit
            assert not ctx.last_plan()["packed"], chunk


def _near_poly_a(n_poly, n_near, seed):
    """n_poly poly-A rows, then n_near rows of A with a C every 4th position (their 9-mers
    hold 2-3 C: Hamming 2 from A^9 and from each other), then random rows."""
    codes, lens = E.synthetic(600, 101, seed=seed)
    codes[:n_poly] = 0
    near = np.zeros(101, dtype=codes.dtype)
    near[::4] = 1
    codes[n_poly:n_poly + n_near] = near
    for r in range(n_near):  # shifted copies, so the windows differ between rows
        codes[n_poly + r] = np.roll(near, r % 4)
    return codes, lens


@pytest.mark.parametrize("chunk", ["96", "600", "20480"])
def test_mismatch_nb_sorted_spills_and_overflow(ctx, tune, chunk):
    """The sorted fill's exits: lists whose segment 2 exceeds the per-wave LDS buffer (the
    A^9 occurrences of 40 poly-A rows are 3720 Hamming-2 entries of every near-A k-mer's list)
    stay 16-bit; runs of 15 spanning more than 254 columns (sparse, clustered columns) spill
    into the 16-bit part.  Raw and normalised K bit-exact against the oracle."""
    codes, lens = _near_poly_a(40, 40, 96)
    tune(KMG_MM_FORM=4, KMG_NB_FILL="1", KMG_MM_CHUNK=chunk)
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), codes, lens, L.KMG_I32)
    assert np.array_equal(raw.astype(np.int64), cref.mismatch_raw(codes, lens, 9, 1))
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.mismatch_rows(codes, lens, 9, 1))


def test_mismatch_triangle_mirror_ragged_chunks(ctx, tune):
    """A full square K built by its upper block triangle + mirror_chunks_kernel with chunk
    edges that are no multiple of its 64 x 64 tiles (328 columns, 4 chunks): raw int32 and
    normalised float64 bit-exact.  (A 128 x 128 tile and loads issued before the LDS
    stores measured equal at config 5, 27.2 vs 27.3 ms: the mirror runs at the HBM copy
    rate, ~5.3 TB/s for 144 GB read + written.)"""
    codes, lens = E.synthetic(1000, 101, seed=99)
    tune(KMG_MM_FORM=4, KMG_MM_CHUNK="328")
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), codes, lens, L.KMG_I32)
    assert ctx.last_plan()["triangle"]
    assert np.array_equal(raw.astype(np.int64), cref.mismatch_raw(codes, lens, 9, 1))
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.mismatch_rows(codes, lens, 9, 1))


@pytest.mark.parametrize("fill", ["3", "4"])
def test_mismatch_nb_piece_fill_fallbacks(ctx, tune, fill):
    """The piece-assembled and staged fills' fallback: lists longer than the piece table or
    the per-wave LDS buffer (80 poly-A rows: the A^9 list holds 7440 entries, 930 pieces)
    take the lane-per-run copies; raw K bit-exact."""
    codes, lens = E.synthetic(600, 101, seed=97)
    codes[:80] = 0
    ref = cref.mismatch_raw(codes, lens, 9, 1)
    tune(KMG_MM_FORM=4, KMG_NB_FILL=fill)
    for chunk in ("96", "20480"):
        tune(KMG_MM_CHUNK=chunk)
        raw = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), codes, lens,
                       L.KMG_I32)
        assert np.array_equal(raw.astype(np.int64), ref), chunk


@pytest.mark.parametrize("k,m", [(2, 1), (5, 1), (7, 1), (12, 1), (5, 0), (5, 2), (4, 3), (13, 1)])
def test_mismatch_params(ctx, k, m):
    codes, lens = E.synthetic(200, 101, seed=k * 10 + m)
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=0), codes, lens, L.KMG_I32)
    assert np.array_equal(raw.astype(np.int64), cref.mismatch_raw(codes, lens, k, m))
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=m, window=101, normalize=1), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.mismatch_rows(codes, lens, k, m))


@pytest.mark.parametrize("k", [8, 9, 10, 11, 12])
def test_mismatch_slots_k_range(ctx, tune, k):
    """Drop-one slot layout (default for k = 8, forced for 9..12) at every compiled k, raw
    and normalised, over several column chunkings (slot tables grow with 4^(k-1) per
    chunk: k >= 10 stays single-chunk here)."""
    codes, lens = E.synthetic(400, 101, seed=50 + k)
    ref = cref.mismatch_raw(codes, lens, k, 1)
    tune(KMG_MM_FORM=1)
    for chunk in (("64", "300", "20480") if k <= 9 else ("20480",)):
        tune(KMG_MM_CHUNK=chunk)
        raw = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0), codes, lens,
                       L.KMG_I32)
        assert np.array_equal(raw.astype(np.int64), ref), chunk
    Kn = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=1), codes, lens,
                  L.KMG_F64)
    assert np.array_equal(Kn, cref.mismatch_rows(codes, lens, k, 1))


@pytest.mark.parametrize("form", ["2", "4", "4:512", "4::2"])
@pytest.mark.parametrize("k", [3, 4, 5, 6, 7, 8, 9, 10, 11, 12])
def test_mismatch_pairs_k_range(ctx, tune, k, form):
    """The drop-two pair table (2) and the neighbourhood lists (4; 16-bit lists 4::2) at every
    compiled k, raw and normalised, over several column chunkings (chunk = columns per group
    table / list set)."""
    codes, lens = E.synthetic(500, 101, seed=80 + k)
    ref = cref.mismatch_raw(codes, lens, k, 1)
    _form(tune, form)
    for chunk in (("40", "168", "20480") if k <= 9 else ("168", "20480") if k == 10 else ("20480",)):
        tune(KMG_MM_CHUNK=chunk)
        raw = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=0), codes, lens,
                       L.KMG_I32)
        assert np.array_equal(raw.astype(np.int64), ref), chunk
    Kn = ctx.gram(P.make(L.KMG_MISMATCH, k=k, m=1, window=101, normalize=1), codes, lens,
                  L.KMG_F64)
    assert np.array_equal(Kn, cref.mismatch_rows(codes, lens, k, 1))


@pytest.mark.parametrize("form", ["1", "2", "4", "4::1", "4::2", "4::3"])
def test_mismatch_slots_overflow_and_big_groups(ctx, tune, form):
    """Drop-one slots: groups longer than the 60 inline entries (CSR tail) and groups of
    >= 65535 entries (16-bit header overflow, CSR only).  Pair table: groups past 255
    entries (wide marker, read from the exact index).  720 poly-A rows put 720 * 93 = 66960
    occurrences in the AAAAAAAAA groups of every copy / pair."""
    tune(KMG_MM_CHUNK=20480)
    _form(tune, form)
    codes, lens = E.synthetic(760, 101, seed=61)
    codes[:720] = 0
    codes[700] = np.tile([0, 1], 51)[:101]
    codes[701, 50] = 2  # poly-A with one substitution: Hamming-1/2 neighbours of the big group
    raw = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), codes, lens,
                   L.KMG_I32)
    ref = cref.mismatch_raw(codes, lens, 9, 1, rows=(690, 760))
    assert np.array_equal(raw[690:760].astype(np.int64), ref)
    assert np.array_equal(raw[:5].astype(np.int64), cref.mismatch_raw(codes, lens, 9, 1, rows=(0, 5)))
    assert np.array_equal(raw, raw.T)


@pytest.mark.parametrize("form", ["1", "2", "4", "4::1", "4::2", "4::3"])
def test_mismatch_stress_repeats(ctx, tune, form):
    _form(tune, form)
    codes, lens = E.synthetic(40, 101, seed=12)
    codes[3] = 0
    codes[4] = np.tile([0, 1], 51)[:101]
    codes[5] = 3
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=0), codes, lens, L.KMG_I32)
    ref = cref.mismatch_raw(codes, lens, 9, 1)
    assert np.array_equal(K.astype(np.int64), ref)
    assert K[3, 3] == 28 * 93 * 93  # 242,172


def test_mismatch_longer_sequences_use_first_window(ctx):
    codes, lens = E.synthetic(50, 130, seed=13)
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=6, m=1, window=101, normalize=1), codes, lens, L.KMG_F64)
    ref = cref.mismatch_rows(codes[:, :101].copy(), np.full(50, 101, np.int32), 6, 1)
    assert np.array_equal(K, ref)


# ------------------------------------------------------------------ float kernels
@pytest.mark.parametrize("d", [1, 3, 4, 10, 20])
def test_wd_xtr0(ctx, d):
    codes, lens = load_xtr0()
    codes, lens = codes[:400], lens[:400]
    K = ctx.gram(P.make(L.KMG_WD, d=d), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.wd(codes, lens, d))


def test_wd_ragged(ctx):
    rng = np.random.default_rng(3)
    seqs = ["".join(rng.choice(list("ACGTN"), size=rng.integers(1, 200))) for _ in range(150)]
    codes, lens = E.encode(seqs)
    K = ctx.gram(P.make(L.KMG_WD, d=6), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.wd(codes, lens, 6))


def _ragged_family(rng, n, base_len=120, S=7):
    """Rows cut from a few parents with length differences 0..S+1 and shifted copies (a row
    equal to another minus its first s symbols): the clipped-slice suffix matches of
    kernels.py:133 occur in many pairs."""
    parents = ["".join(rng.choice(list("ACGT"), size=base_len + S + 2)) for _ in range(4)]
    out = []
    for _ in range(n):
        p = parents[rng.integers(0, 4)]
        a = int(rng.integers(0, S + 2))
        b = base_len - int(rng.integers(0, S + 2))
        out.append(p[a:b] if rng.random() < 0.8 else p[a:b][:-3] + "NNA")
    return out


@pytest.mark.parametrize("d,S", [(1, 1), (3, 2), (5, 3), (8, 7), (4, 12)])
def test_wds_ragged(ctx, d, S):
    rng = np.random.default_rng(100 + S)
    seqs = _ragged_family(rng, 96, S=S)
    codes, lens = E.encode(seqs)
    K = ctx.gram(P.make(L.KMG_WDS, d=d, S=S), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.wds(codes, lens, d, S))


def test_wd_wds_pair_any_L(engine):
    """get_WD_d / get_WDShifts_d for L below, at and above the lengths (padded pair on the
    device) against the oracle's literal loops."""
    rng = np.random.default_rng(9)
    seqs = _ragged_family(rng, 12, base_len=50, S=3)
    for t in range(0, 12, 2):
        x, y = seqs[t], seqs[t + 1]
        for span in (0, 1, 2, 5, len(x) - 3, len(x), len(y), len(x) + 4, max(len(x), len(y)) + 9):
            assert engine.wd_pair(x, y, 5, span) == cpu_ref.wd_pair(x, y, 5, span)
            assert engine.wds_pair(x, y, 4, 3, span) == cpu_ref.wds_pair(x, y, 4, 3, span)


def test_wd_span_past_shortest_row_rejected(ctx):
    """A full-K call with span > 0 counts positions below min(len_x, len_y, span): a span past
    a row's end would miss the reference's clipped-slice matches, so the C ABI refuses it
    (KMG_EUNSUPPORTED) unless the rows are padded to span (+ S), as engine.wd_pair does."""
    codes, lens = E.synthetic(6, 60, seed=14)
    lens[3] = 40
    for kind, extra in ((L.KMG_WD, {}), (L.KMG_WDS, {"S": 3})):
        with pytest.raises(L.KmgUnsupported):
            ctx.gram(P.make(kind, d=4, span=45, **extra), codes, lens, L.KMG_F64)
    ctx.gram(P.make(L.KMG_WD, d=4, span=40), codes, lens, L.KMG_F64)  # = min len: accepted
    with pytest.raises(L.KmgUnsupported):
        ctx.gram(P.make(L.KMG_WDS, d=4, S=3, span=38), codes, lens, L.KMG_F64)  # 38 + 3 > 40


@pytest.mark.parametrize("d,S", [(1, 0), (3, 1), (5, 3), (10, 5), (8, 7), (4, 12)])
def test_wds_xtr0(ctx, d, S):
    codes, lens = load_xtr0()
    codes, lens = codes[:160], lens[:160]
    K = ctx.gram(P.make(L.KMG_WDS, d=d, S=S), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.wds(codes, lens, d, S))


@pytest.mark.parametrize("lb,k", [(0.5, 3), (1.0, 3), (0.7, 5), (0.3, 2), (0.5, 1), (0.9, 8), (0.6, 11),
                                  (0.8, 4), (0.7, 6), (0.8, 7), (0.9, 9), (0.9, 16), (0.95, 17),
                                  (0.97, 24), (0.99, 33)])
def test_ss_xtr0(ctx, lb, k):
    """Every level count of the grouped sweep (k - 1 = 1..8 exactly, 12 / 16 / 24 / 32
    rounded up) bit-exact against the golden-pinned oracle at L = 101 (k > 16: past the
    round-2 limit)."""
    codes, lens = load_xtr0()
    codes, lens = codes[:48], lens[:48]
    K = ctx.gram(P.make(L.KMG_SUBSTRING, k=k, lbda=lb), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.ss(codes, lens, lb, k))


@pytest.mark.parametrize("k,maxlen", [(3, 150), (12, 150), (3, 100), (6, 100), (20, 110)])
def test_ss_ragged(ctx, k, maxlen):
    """Ragged rows (lengths 0..maxlen): past length 127 the 64-row strip kernel, below it
    the grouped sweep with idle rows / groups of short pairs."""
    rng = np.random.default_rng(4 + k)
    seqs = ["".join(rng.choice(list("ACGT"), size=rng.integers(0, maxlen))) for _ in range(40)]
    codes, lens = E.encode(seqs)
    K = ctx.gram(P.make(L.KMG_SUBSTRING, k=k, lbda=0.8), codes, lens, L.KMG_F64)
    assert np.array_equal(K, cref.ss(codes, lens, 0.8, k))
    if maxlen <= 110:  # rows of another call: the lower triangle without the mirror
        Kr = ctx.gram(P.make(L.KMG_SUBSTRING, k=k, lbda=0.8), codes[5:], lens[5:], L.KMG_F64)
        assert np.array_equal(Kr, K[5:, 5:])


def test_ss_limits(ctx):
    """k = 34 at L = 101 (more than 32 DP levels in registers) and k = 17 past length 127
    are the SS kernels' remaining limits: KMG_EUNSUPPORTED, never a wrong value."""
    codes, lens = load_xtr0()
    with pytest.raises(L.KmgUnsupported):
        ctx.gram(P.make(L.KMG_SUBSTRING, k=34, lbda=0.9), codes[:4], lens[:4], L.KMG_F64)
    c2, l2 = E.encode(["ACGT" * 40, "ACGA" * 40])
    with pytest.raises(L.KmgUnsupported):
        ctx.gram(P.make(L.KMG_SUBSTRING, k=17, lbda=0.9), c2, l2, L.KMG_F64)


def test_gappy_k1g0(ctx):
    import kernels
    seqs = ["ACGT" * 26, "AAAA" * 26, "ACAC" * 26, "GGTT" * 26, ""]
    K = kernels.get_gappy_K(_X(seqs), 1, 0)
    codes, lens = E.encode(seqs)
    ref = cpu_ref.gappy_k1g0(codes, lens)
    assert np.array_equal(K, ref, equal_nan=True)


# ------------------------------------------------------------------ helpers
def test_normalize_and_center(engine):
    import kernels
    rng = np.random.default_rng(1)
    A = rng.integers(0, 50, size=(300, 40)).astype(np.float64)
    K = A @ A.T
    ref = cpu_ref.normalize(K)
    K2 = K.copy()
    out = kernels.normalize_K(K2)
    assert out is K2 and np.array_equal(K2, ref)
    # already normalised -> unchanged
    K3 = ref.copy()
    kernels.normalize_K(K3)
    assert np.array_equal(K3, ref)
    C = kernels.center_K(K)
    assert np.allclose(C, cpu_ref.center(K), rtol=0, atol=1e-9 * np.abs(K).max())


def test_row_slabs_equal_full(ctx):
    """kmg_gram_device on row slabs (the multi-GPU shard unit) == full matrix."""
    codes, lens = E.synthetic(1000, 101, seed=21)
    n, ldc = codes.shape
    full = ctx.gram(P.make(L.KMG_SPECTRUM, k=8), codes, lens, L.KMG_I32)
    fullm = ctx.gram(P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), codes, lens, L.KMG_F64)
    fullw = ctx.gram(P.make(L.KMG_WD, d=5), codes, lens, L.KMG_F64)
    d_codes = ctx.dmalloc(codes.nbytes)
    d_lens = ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    try:
        for params, dt, ref in ((P.make(L.KMG_SPECTRUM, k=8), L.KMG_I32, full),
                                (P.make(L.KMG_MISMATCH, k=9, m=1, window=101, normalize=1), L.KMG_F64, fullm),
                                (P.make(L.KMG_WD, d=5), L.KMG_F64, fullw)):
            esz = np.dtype(L.DTYPES[dt]).itemsize
            out = np.zeros((n, n), dtype=L.DTYPES[dt])
            d_out = ctx.dmalloc(n * n * esz)
            splits = [0, 137, 500, 501, 1000]
            for a, b in zip(splits[:-1], splits[1:]):
                import ctypes
                ctx.gram_device(params, d_codes, d_lens, n, ldc, a, b, dt,
                                ctypes.c_void_p(d_out.value + a * n * esz), n)
            ctx.synchronize()
            ctx.d2h(out, d_out)
            ctx.dfree(d_out)
            assert np.array_equal(out, ref)
    finally:
        ctx.dfree(d_codes)
        ctx.dfree(d_lens)


def test_device_sqrt_div_bits(ctx):
    """The fp64 normalise epilogue reproduces numpy's sqrt and division bits."""
    codes, lens = E.synthetic(500, 101, seed=31)
    K = ctx.gram(P.make(L.KMG_MISMATCH, k=4, m=1, window=101, normalize=1), codes, lens, L.KMG_F64)
    raw = cref.mismatch_raw(codes, lens, 4, 1).astype(np.float64)
    d = np.sqrt(np.diag(raw))
    ref = raw / (d[:, None] * d[None, :])
    np.fill_diagonal(ref, 1.0)
    assert np.array_equal(K, ref)


def test_rccl_allgather_single_rank(ctx):
    """kmg_comm_init / kmg_allgather_rows on a 1-rank communicator (the multi-GPU
    assembly code path; >1 rank needs >1 GPU and is exercised by bench.py --allgather)."""
    codes, lens = E.synthetic(300, 101, seed=41)
    n, ldc = codes.shape
    full = ctx.gram(P.make(L.KMG_SPECTRUM, k=6), codes, lens, L.KMG_I32)
    uid = L.Context.unique_id()
    ctx.comm_init(uid, 1, 0)
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    ctx.h2d(d_codes, codes)
    ctx.h2d(d_lens, lens)
    d_out = ctx.dmalloc(n * n * 4)
    try:
        ctx.gram_device(P.make(L.KMG_SPECTRUM, k=6), d_codes, d_lens, n, ldc, 0, n, L.KMG_I32,
                        d_out, n)
        ctx.allgather_rows(d_out, n, n, L.KMG_I32, [0, n])
        ctx.synchronize()
        out = np.empty((n, n), dtype=np.int32)
        ctx.d2h(out, d_out)
        assert np.array_equal(out, full)
    finally:
        ctx.comm_destroy()
        for p_ in (d_out, d_codes, d_lens):
            ctx.dfree(p_)


@pytest.mark.parametrize("rows", ["1", "2", "4"])
@pytest.mark.parametrize("chunk", ["304", "24576"])
def test_spectrum_rows_per_workgroup(ctx, tune, rows, chunk):
    """gram_sp_kernel with 1, 2 or 4 rows a workgroup (KMG_SP_ROWS), over several column
    chunks and over one: the full K (int32, float64 normalised) and a row range of odd
    length (the last workgroup one row short) equal the oracle (get_spectrum_K,
    kernels.py:28-47; normalize_K, kernels.py:398-415); ragged rows."""
    codes, lens = E.synthetic(1001, 101, seed=78)
    lens[::6] = 30 + (np.arange(len(lens[::6])) % 72)
    tune(KMG_SP_CHUNK=chunk, KMG_SP_ROWS=rows)
    ref = cref.spectrum(codes, lens, 8)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=8), codes, lens, L.KMG_I32)
    assert (ctx.last_plan()["nchunks"] > 1) == (chunk == "304")
    assert np.array_equal(K.astype(np.int64), ref)
    Kn = ctx.gram(P.make(L.KMG_SPECTRUM, k=8, normalize=1), codes, lens, L.KMG_F64)
    d = np.sqrt(np.diag(ref).astype(np.float64))
    refn = ref.astype(np.float64) / (d[:, None] * d[None, :])
    np.fill_diagonal(refn, 1.0)
    assert np.array_equal(Kn, refn)
    n, ldc = codes.shape
    r0, r1 = 17, 520
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc((r1 - r0) * n * 4)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device(P.make(L.KMG_SPECTRUM, k=8), d_codes, d_lens, n, ldc, r0, r1, L.KMG_I32,
                        d_out, n)
        Kr = np.empty((r1 - r0, n), dtype=np.int32)
        ctx.d2h(Kr, d_out)
        assert np.array_equal(Kr.astype(np.int64), ref[r0:r1])
    finally:
        for p_ in (d_codes, d_lens, d_out):
            ctx.dfree(p_)


@pytest.mark.parametrize("rows", ["1", "2", "4"])
def test_spectrum_rows_per_workgroup_long_sequences(ctx, tune, rows):
    """Sequences of 300..700 symbols (more than 255 windows: 32-bit accumulators, so two or
    four rows a workgroup take 2-4x the LDS and fall back to fewer rows past 160 KB): full K
    and a column block equal the oracle (get_spectrum_K, kernels.py:28-47)."""
    codes, lens = E.synthetic(300, 700, seed=79)
    lens[:] = 300 + (np.arange(300) * 7) % 401
    tune(KMG_SP_ROWS=rows, KMG_SP_CHUNK="128")
    ref = cref.spectrum(codes, lens, 7)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=7), codes, lens, L.KMG_I32)
    assert ctx.last_plan()["nchunks"] > 1
    assert np.array_equal(K.astype(np.int64), ref)
    n, ldc = codes.shape
    c0, c1 = 37, 290
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(n * (c1 - c0) * 4)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.gram_device_cols(P.make(L.KMG_SPECTRUM, k=7), d_codes, d_lens, n, ldc, c0, c1,
                             L.KMG_I32, d_out, c1 - c0)
        Kc = np.empty((n, c1 - c0), dtype=np.int32)
        ctx.d2h(Kc, d_out)
        assert np.array_equal(Kc.astype(np.int64), ref[:, c0:c1])
    finally:
        for p_ in (d_codes, d_lens, d_out):
            ctx.dfree(p_)


def test_spectrum_column_chunks(ctx, tune):
    """Spectrum over several column chunks (the config-4 layout at a small N): full K (int32
    and float64 normalised), a row slab and block-cyclic rows of three ranks (several ranges
    per call) equal the oracle (get_spectrum_K, kernels.py:28-47; normalize_K,
    kernels.py:398-415), ragged rows included."""
    import ctypes
    codes, lens = E.synthetic(1300, 101, seed=77)
    lens[::5] = 40 + (np.arange(len(lens[::5])) % 62)
    tune(KMG_SP_CHUNK="304")
    ref = cref.spectrum(codes, lens, 8)
    K = ctx.gram(P.make(L.KMG_SPECTRUM, k=8), codes, lens, L.KMG_I32)
    assert ctx.last_plan()["nchunks"] > 1
    assert np.array_equal(K.astype(np.int64), ref)
    Kn = ctx.gram(P.make(L.KMG_SPECTRUM, k=8, normalize=1), codes, lens, L.KMG_F64)
    d = np.sqrt(np.diag(ref).astype(np.float64))
    refn = ref.astype(np.float64) / (d[:, None] * d[None, :])
    np.fill_diagonal(refn, 1.0)
    assert np.array_equal(Kn, refn)
    n, ldc = codes.shape
    d_codes, d_lens = ctx.dmalloc(codes.nbytes), ctx.dmalloc(lens.nbytes)
    d_out = ctx.dmalloc(n * n * 4)
    try:
        ctx.h2d(d_codes, codes)
        ctx.h2d(d_lens, lens)
        ctx.memset(d_out, 0xA5, n * n * 4)
        ctx.gram_device(P.make(L.KMG_SPECTRUM, k=8), d_codes, d_lens, n, ldc, 100, 900, L.KMG_I32,
                        d_out, n)
        ctx.synchronize()
        rows = np.empty((800, n), dtype=np.int32)
        ctx.d2h(rows, d_out)
        assert np.array_equal(rows.astype(np.int64), ref[100:900])
        ctx.memset(d_out, 0xA5, n * n * 4)
        for r in range(3):
            ctx.gram_blocks(P.make(L.KMG_SPECTRUM, k=8), d_codes, d_lens, n, ldc, L.KMG_I32, d_out,
                            n, 3, r, 100, 0)
        ctx.synchronize()
        full = np.empty((n, n), dtype=np.int32)
        ctx.d2h(full, d_out)
        assert np.array_equal(full.astype(np.int64), ref)
    finally:
        for p_ in (d_out, d_codes, d_lens):
            ctx.dfree(p_)
