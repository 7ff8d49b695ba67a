#!/usr/bin/env python3
"""Summarise rocprofv3 output for the committed profiles/ evidence.

usage: python profiles/pmc_summary.py <prof_dir> <tag> [N (default 100000)] [workload]
  <prof_dir>/trace/run_kernel_stats.csv          (--kernel-trace --stats)
  <prof_dir>/pmc_fetch/run_counter_collection.csv (--pmc FETCH_SIZE, own pass)
  <prof_dir>/pmc_write/run_counter_collection.csv (--pmc WRITE_SIZE, own pass)
  (or run_profiles_r02.sh's <prof_dir>/p*/: the pass holding each counter)
writes profiles/<tag>_kernel_stats.csv (copy), profiles/<tag>_pmc.json.

HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide coalesced streaming reads, so
the read side is doubled (an upper bound for narrower reads); WRITE_SIZE is exact for
16-B-per-lane streaming stores (the Gram row stores are 16 B per lane).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))


def per_kernel(path, counter):
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def counter_file(src, sub, counter):
    """<src>/<sub>/run_counter_collection.csv, else the first <src>/p*/ pass with counter."""
    path = os.path.join(src, sub, "run_counter_collection.csv")
    if os.path.exists(path):
        return path
    for d in sorted(os.listdir(src)):
        cand = os.path.join(src, d, "run_counter_collection.csv")
        if d.startswith("p") and os.path.exists(cand):
            with open(cand) as f:
                if any(row["Counter_Name"] == counter for row in csv.DictReader(f)):
                    return cand
    raise FileNotFoundError(f"no pass with {counter} under {src}")


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    src, tag = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 100000  # the bench's spectrum N
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(HERE, f"{tag}_kernel_stats.csv"))
    workload = sys.argv[4] if len(sys.argv) > 4 else "spectrum_k8"
    fetch = per_kernel(counter_file(src, "pmc_fetch", "FETCH_SIZE"), "FETCH_SIZE")
    write = per_kernel(counter_file(src, "pmc_write", "WRITE_SIZE"), "WRITE_SIZE")
    stats = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            stats[short(row["Name"])] = float(row["AverageNs"])
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fk, wk = fetch.get(k, 0.0) * 1024, write.get(k, 0.0) * 1024
        kernels[short(k)] = {"fetch_bytes_raw": fk, "fetch_bytes_x2": 2 * fk, "write_bytes": wk,
                             "hbm_bytes_est": 2 * fk + wk, "avg_ns": stats.get(short(k))}
    gram = next((v for k, v in kernels.items()
                 if any(g in k for g in ("gram_sp_kernel", "gram_pl_kernel", "gram_mm", "gram_nb"))), None)
    out = {"tag": tag, "workload": workload, "N": n, "kernels": kernels,
           "hbm_bytes_per_launch": gram["hbm_bytes_est"] if gram else None}
    with open(os.path.join(HERE, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
