"""Generate golden vectors for the string-kernel Gram path by running the UNMODIFIED
reference ``kernels.py`` (afiliot/Kernel-Methods-For-Genomics, mounted read-only at
/root/reference) in THIS container.

This script is test infrastructure. It is run by hand in the build container only
(never on the GPU box, never by the tests): ``python tests/golden/make_golden.py``.
Its outputs are small ``.npz`` / ``.json`` fixtures committed next to it; the tests
read only those fixtures.

Every fixture records the reference function it came from (file:line in
/root/reference/kernels.py).
"""
import hashlib
import io
import json
import os
import sys
import time
import traceback
import contextlib
from concurrent.futures import ProcessPoolExecutor

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _ref():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import kernels as km  # noqa: E402  (the reference module)
    return km


def _load_xtr0():
    import pandas as pd
    return pd.read_csv(os.path.join(REF, "Data", "Xtr0.csv"))


def _frame(seqs):
    import pandas as pd
    return pd.DataFrame({"Id": np.arange(len(seqs)), "seq": list(seqs)})


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# --------------------------------------------------------------------------- jobs
FEATURE_FNS = ("get_phi_u", "get_phi_km", "gappy_k", "B_k")


def feature_call(km, fn, kwargs, seqs):
    """The reference's module-level feature maps called the way its own Gram functions
    call them: get_phi_u on the string with string betas (kernels.py:37-40), get_phi_km and
    gappy_k on format(x) with format()ed betas (kernels.py:206-210, 446-449), B_k on two
    strings (kernels.py:322-342).  kwargs["betas"] == "canonical": all 4^k k-mers in
    itertools.product order; otherwise the explicit list."""
    from itertools import product
    k = kwargs.get("k")
    betas = kwargs.get("betas")
    if fn == "get_phi_u":
        b = [''.join(c) for c in product('ACGT', repeat=k)] if betas == "canonical" else list(betas)
        return km.get_phi_u(seqs[0], k, b)
    if fn == "B_k":
        return np.array([km.B_k(kwargs["lbda"], k, seqs[0], seqs[1])], dtype=np.float64)
    b = (np.array([km.format(''.join(c)) for c in product('ACGT', repeat=k)])
         if betas == "canonical" else np.array(betas))
    if fn == "get_phi_km":
        return km.get_phi_km(km.format(seqs[0]), k, kwargs["m"], b)
    return km.gappy_k(km.format(seqs[0]), k, kwargs["g"], b)


def job(spec):
    """Run one reference call; returns (name, dict of arrays/meta)."""
    name, fn, kwargs, seqs = spec
    km = _ref()
    X = _frame(seqs)
    t0 = time.time()
    out = {"name": name, "fn": fn, "kwargs": kwargs, "n": len(seqs)}
    with contextlib.redirect_stderr(io.StringIO()), contextlib.redirect_stdout(io.StringIO()):
        try:
            if fn == "select_method":
                K = km.select_method(X, kwargs["method"])
            elif fn in FEATURE_FNS:  # module-level feature maps / the SS auxiliary
                K = feature_call(km, fn, kwargs, seqs)
            elif fn in ("get_WD_d", "get_WDShifts_d"):  # one pair: (x, y, ..., L)
                K = np.array([getattr(km, fn)(seqs[0], seqs[1], **kwargs)], dtype=np.float64)
            else:
                K = getattr(km, fn)(X, **kwargs)
            out["K"] = np.asarray(K)
            out["error"] = None
        except Exception as e:  # reference raises for some inputs: record type + message
            out["K"] = None
            out["error"] = type(e).__name__
            out["error_module"] = type(e).__module__
            out["error_msg"] = str(e)[:200]
    out["seconds"] = time.time() - t0
    return out


def main():
    X0 = _load_xtr0()
    seqs = list(X0["seq"])
    rng = np.random.default_rng(20261015)

    # Ragged / edge sequences for the spectrum kernel (uses len(x), kernels.py:21)
    ragged = [seqs[0], seqs[1][:50], seqs[2][:7], "ACG", "", seqs[3][:30] + "N" + seqs[3][31:60],
              "A" * 40, "ACGT" * 10, seqs[4][:101], seqs[5] + "ACGTT", "NNNNNNNN", "acgtACGT" * 3]

    # homopolymer / tandem-repeat stress rows reach the count maxima
    stress = [seqs[i] for i in range(8)] + ["A" * 101, "AC" * 50 + "A", "ACGT" * 25 + "A", "T" * 101]

    jobs = []
    for k in range(1, 9):
        jobs.append((f"SP_k{k}_xtr0_n48", "get_spectrum_K", {"k": k}, seqs[:48]))
    jobs.append(("SP_k3_ragged", "get_spectrum_K", {"k": 3}, ragged))
    jobs.append(("SP_k5_ragged", "get_spectrum_K", {"k": 5}, ragged))
    jobs.append(("SP_k8_stress", "get_spectrum_K", {"k": 8}, stress))
    for k in (3, 4, 5, 6):
        jobs.append((f"MM_k{k}_m1_xtr0_n32", "get_mismatch_K", {"k": k, "m": 1}, seqs[:32]))
    jobs.append(("MM_k5_m1_stress", "get_mismatch_K", {"k": 5, "m": 1}, stress))
    jobs.append(("MM_k5_m0_xtr0_n16", "get_mismatch_K", {"k": 5, "m": 0}, seqs[:16]))
    jobs.append(("MM_k5_m2_xtr0_n16", "get_mismatch_K", {"k": 5, "m": 2}, seqs[:16]))
    jobs.append(("MM_k4_m3_xtr0_n12", "get_mismatch_K", {"k": 4, "m": 3}, seqs[:12]))
    jobs.append(("MM_k9_m1_xtr0_n8", "get_mismatch_K", {"k": 9, "m": 1}, seqs[:8]))
    for d in (1, 2, 4, 5, 10):
        jobs.append((f"WD_d{d}_xtr0_n64", "get_WD_K", {"d": d}, seqs[:64]))
    jobs.append(("WD_d5_stress", "get_WD_K", {"d": 5}, stress))
    for d, S in ((1, 0), (3, 1), (5, 3), (10, 5)):
        jobs.append((f"WDS_d{d}_s{S}_xtr0_n24", "get_WDShifts_K", {"d": d, "S": S}, seqs[:24]))
    jobs.append(("WDS_d5_s3_stress", "get_WDShifts_K", {"d": 5, "S": 3}, stress))
    # ragged WD / WDS: rows whose lengths differ by 1..S (the clipped-slice suffix matches of
    # kernels.py:133), a row that is another minus its first s symbols, and the empty row
    base = seqs[7][:60]
    wragged = [base, base[2:], seqs[8][:59], base[1:], seqs[9][:57], base[3:] + "A", base[:58],
               seqs[10][:61], base[4:], "ACGTA", "", base[:57], "NACGT" * 11, base[3:]]
    jobs.append(("WD_d5_ragged", "get_WD_K", {"d": 5}, wragged))
    jobs.append(("WD_d1_ragged", "get_WD_K", {"d": 1}, wragged))
    for d, S in ((1, 1), (3, 2), (5, 3), (4, 7)):
        jobs.append((f"WDS_d{d}_s{S}_ragged", "get_WDShifts_K", {"d": d, "S": S}, wragged))
    # pair helpers with L != len(x) (kernels.py:64-81, 115-135)
    pairs = [(base, base[2:]), (base[2:], base), (seqs[11][:50], seqs[12][:50]),
             (base, base), ("ACGTACGT", "ACGTAC"), (seqs[13][:40], seqs[13][:40] + "AC")]
    for pi, (x, y) in enumerate(pairs):
        for L in sorted({1, 3, len(x) - 7, len(x) - 1, len(x), len(x) + 1, len(x) + 5,
                         len(y) + 2, len(x) + 12}):
            if L < 0:
                continue
            jobs.append((f"WDd_p{pi}_L{L}", "get_WD_d", {"d": 4, "L": L}, [x, y]))
            jobs.append((f"WDSd_p{pi}_L{L}", "get_WDShifts_d", {"d": 4, "S": 3, "L": L}, [x, y]))
    for lb, k in ((0.5, 3), (1.0, 3), (0.7, 5), (0.3, 2), (0.5, 1)):
        jobs.append((f"SS_l{lb}_k{k}_xtr0_n10", "get_string_K", {"lbda": lb, "k": k}, seqs[:10]))
    jobs.append(("SS_l0.5_k3_short", "get_string_K", {"lbda": 0.5, "k": 3},
                 ["ACGTAC", "AC", "GATTACA", "CCCC", "ACG", seqs[0][:40]]))
    jobs.append(("LA_smith0_eig0_n6", "get_LA_K", {"e": 11, "d": 1, "beta": 0.5, "smith": 0, "eig": 0}, seqs[:6]))
    jobs.append(("LA_smith1_eig0_n6", "get_LA_K", {"e": 11, "d": 1, "beta": 0.5, "smith": 1, "eig": 0}, seqs[:6]))
    jobs.append(("LA_smith0_eig1_n6", "get_LA_K", {"e": 11, "d": 1, "beta": 0.5, "smith": 0, "eig": 1}, seqs[:6]))
    jobs.append(("LA_smith0_eig1_n8", "get_LA_K", {"e": 11, "d": 1, "beta": 0.5, "smith": 0, "eig": 1}, seqs[:8]))
    jobs.append(("GP_k3_g1_n4", "get_gappy_K", {"k": 3, "g": 1}, seqs[:4]))
    jobs.append(("GP_k3_g0_n4", "get_gappy_K", {"k": 3, "g": 0}, seqs[:4]))
    # select_method grammar (kernels.py:461-505)
    for meth in ("SP_k4", "WD_k5", "WD_d4", "MM_k4_m1", "WDS_d3_s1", "SS_l0.5_k2",
                 "LA_e11_d1_b0.5_smith0_eig0", "GP_k3_g1", "XX_k3"):
        jobs.append((f"select_{meth}_n6", "select_method", {"method": meth}, seqs[:6]))
    # module-level feature maps and the SS auxiliary (kernels.py:12-25, 161-175, 308-342,
    # 420-433), round 4
    phx = [seqs[0], seqs[1][:50], "ACGTNACGT", "", "acgtACGT", seqs[2] + "ACGTTG", "A" * 30]
    for xi, x in enumerate(phx):
        for k in (1, 3, 5):
            jobs.append((f"PHIU_x{xi}_k{k}", "get_phi_u", {"k": k, "betas": "canonical"}, [x]))
    jobs.append(("PHIU_x0_k8", "get_phi_u", {"k": 8, "betas": "canonical"}, [seqs[0]]))
    custom = ["ACG", "TTT", "AAA", "GA", "ACGT", "CCC", "GGG", "TGC", "ACG", ""]
    for xi in (0, 2, 6):
        jobs.append((f"PHIU_x{xi}_k3_custom", "get_phi_u", {"k": 3, "betas": custom}, [phx[xi]]))
    kmx = [seqs[0], seqs[3] + "ACG", seqs[4][:50]]
    for xi, x in enumerate(kmx):
        for k, m in ((3, 0), (3, 1), (5, 1), (5, 2), (6, 1)):
            jobs.append((f"PHIKM_x{xi}_k{k}_m{m}", "get_phi_km", {"k": k, "m": m, "betas": "canonical"}, [x]))
    kcustom = [[1, 2, 3], [4, 4, 4], [2, 2, 1], [3, 1, 4]]
    jobs.append(("PHIKM_x0_k3_m1_custom", "get_phi_km", {"k": 3, "m": 1, "betas": kcustom}, [kmx[0]]))
    # round 5: betas and sequences outside A/C/G/T (string / integer identity), and the rows
    # shorter than get_phi_km's 101 window whose short k-mers numpy broadcasts
    nb3 = ["GTN", "TNA", "NAC", "ACG", "NNN", "CGT", "GTA", "AC", "N"]
    for xi in (0, 2):
        jobs.append((f"PHIU_sym_x{xi}_k3", "get_phi_u", {"k": 3, "betas": nb3}, [phx[xi]]))
    jobs.append(("PHIU_sym_x7_k2", "get_phi_u", {"k": 2, "betas": ["XX", "AX", "GX", "XA", "AC", "xA", "X"]},
                 ["AXXCGXAXXA"]))
    jobs.append(("PHIU_sym_x8_k1", "get_phi_u", {"k": 1, "betas": ["A", "N", "-", "C", "n", ""]},
                 ["AN-CnNNA--"]))
    xd = seqs[0][:50] + "5" + seqs[0][51:70] + "0" + seqs[0][71:]
    vb = [[1, 5, 3], [5, 5, 5], [0, 1, 2], [2, 2, 1], [1, 0, 4], [4, 4, 4]]
    for m in (0, 1, 2):
        jobs.append((f"PHIKM_sym_xd_k3_m{m}", "get_phi_km", {"k": 3, "m": m, "betas": vb}, [xd]))
    jobs.append(("PHIKM_sym_xd_k3_m1_canon", "get_phi_km", {"k": 3, "m": 1, "betas": "canonical"}, [xd]))
    jobs.append(("PHIKM_sym_x0_k2_m0_vals", "get_phi_km", {"k": 2, "m": 0, "betas": [[1, 7], [7, 7], [2, 2]]},
                 [seqs[0]]))
    for xi, (x, k, m) in enumerate(((seqs[1][:100], 2, 0), (seqs[1][:100], 2, 1), (seqs[2][:60], 1, 0),
                                    (seqs[2][:60], 1, 1), (seqs[3][:100], 2, 2), ("", 1, 0),
                                    (seqs[4][:99], 2, 1))):
        jobs.append((f"PHIKM_sym_short{xi}_k{k}_m{m}", "get_phi_km", {"k": k, "m": m, "betas": "canonical"}, [x]))
    for xi, x in enumerate([seqs[0], "ACGA", "", seqs[5][:60]]):
        jobs.append((f"GAPK_x{xi}_k1_g0", "gappy_k", {"k": 1, "g": 0, "betas": "canonical"}, [x]))
    for k, g in ((3, 1), (3, 0), (2, 3), (3, 2), (3, 3), (1, 1)):
        jobs.append((f"GAPK_x0_k{k}_g{g}", "gappy_k", {"k": k, "g": g, "betas": "canonical"}, [seqs[0]]))
    jobs.append(("GAPK_xe_k3_g1", "gappy_k", {"k": 3, "g": 1, "betas": "canonical"}, [""]))
    bpairs = [("ACGTAC", "GATTACA"), (seqs[0][:20], seqs[1][:25]), (seqs[2][:30], seqs[3][:30]),
              ("AC", "ACGTAC"), ("ACGNAC", "NACGT"), (seqs[4][:40], seqs[4][:40])]
    for pi, (x, y) in enumerate(bpairs):
        for lb, k in ((0.5, 3), (0.7, 2), (1.0, 4), (0.5, 0), (0.3, 1)):
            jobs.append((f"BK_p{pi}_l{lb}_k{k}", "B_k", {"lbda": lb, "k": k}, [x, y]))

    # config 1 (BASELINE configs[0]): SP k=6 on all of Xtr0
    jobs.append(("SP_k6_xtr0_full", "get_spectrum_K", {"k": 6}, seqs))

    only = set(sys.argv[1:])
    if only:
        # exact names, or prefixes ending in '*' (e.g. 'PHIU*')
        jobs = [j for j in jobs if j[0] in only or
                any(o.endswith("*") and j[0].startswith(o[:-1]) for o in only)]
    # longest first
    order = {"SP_k6_xtr0_full": 0, "MM_k9_m1_xtr0_n8": 1}
    jobs.sort(key=lambda j: order.get(j[0], 9))

    arrays = {}
    meta_path = os.path.join(HERE, "golden_meta.json")
    meta = json.load(open(meta_path)) if (only and os.path.exists(meta_path)) else {}
    npz_path = os.path.join(HERE, "golden.npz")
    if only and os.path.exists(npz_path):
        with np.load(npz_path, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
    seq_sets = {}
    with ProcessPoolExecutor(max_workers=7) as ex:
        for (spec, res) in zip(jobs, ex.map(job, jobs)):
            name = res["name"]
            entry = {"fn": res["fn"], "kwargs": res["kwargs"], "n": res["n"],
                     "seconds": round(res["seconds"], 2), "error": res["error"]}
            if res["error"]:
                entry["error_module"] = res["error_module"]
                entry["error_msg"] = res["error_msg"]
            K = res["K"]
            seq_key = "seqs_" + hashlib.sha1("\n".join(spec[3]).encode()).hexdigest()[:12]
            entry["seqs"] = seq_key
            seq_sets[seq_key] = spec[3]
            if K is not None:
                entry["sha256_f64"] = _sha(np.asarray(K, dtype=np.float64))
                entry["dtype"] = str(K.dtype)
                entry["shape"] = list(K.shape)
                if name == "SP_k6_xtr0_full":
                    # too big to commit whole: keep hash + row sums + a sampled block
                    entry["row_sums"] = [int(v) for v in K.sum(axis=1)]
                    arrays[name + "__block"] = K[:64, :64].astype(np.int32)
                    entry["sum"] = int(K.sum())
                else:
                    arrays[name] = K
            meta[name] = entry
            print(f"{name}: {res['seconds']:.1f}s err={res['error']}", flush=True)
    for key, s in seq_sets.items():
        arrays[key] = np.array(s, dtype="U")
    np.savez_compressed(npz_path, **arrays)
    with open(meta_path, "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
