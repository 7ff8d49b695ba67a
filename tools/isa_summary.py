#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S gfx950 assembly file.
usage: python tools/isa_summary.py <file.s> <mangled-name substring> [--dump]"""
import collections
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    s = open(path).read()
    m = re.search(r"^(_Z\S*%s\S*):" % re.escape(sub), s, re.M)
    if not m:
        sys.exit("kernel not found")
    name = m.group(1)
    start = m.end()
    end = s.find(".Lfunc_end", start)
    body = s[start:end]
    ins = [l.strip() for l in body.split("\n")
           if l.strip() and not l.strip().startswith((";", ".")) and not l.strip().endswith(":")]
    print(name[:100], len(ins), "instructions")
    c = collections.Counter(l.split()[0] for l in ins)
    print(c.most_common(45))
    meta = s[end:end + 4000]
    for key in ("vgpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size"):
        mm = re.search(r"\.%s:\s*(\d+)" % key, meta)
        if mm:
            print(key, mm.group(1))
    mm = re.search(r"; NumVgprs: (\d+).*?; ScratchSize: (\d+).*?; Occupancy: (\d+)", s[end:end + 3000], re.S)
    if mm:
        print("NumVgprs", mm.group(1), "Scratch", mm.group(2), "Occupancy", mm.group(3))
    if "--dump" in sys.argv:
        print(body)


if __name__ == "__main__":
    main()
