#!/usr/bin/env python3
"""Average PMC counters per kernel over every pass directory of tools/pmc_pass.sh.
usage: python tools/pmc_report.py gpurun_out/pmc_<tag> [kernel-substring]"""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "p*", "run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        if flt and flt not in k:
            continue
        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c in sorted(d):
        v = d[c]
        print(f"   {c:28s} {sum(v)/len(v):16.1f}   (n={len(v)})")
