#!/bin/bash
# WD kernel rows per pass (KMG_WD_VAR: 0 one row, 2 or 4 rows with independent chains):
# parity of each against the oracle, then an interleaved one-process A/B.
set -u
OUT=gpurun_out/r2bp
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in 2 4; do
  KMG_WD_VAR=$V timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q -k "wd or WD" --timeout 120 --timeout-method thread > "$OUT/pytest_v$V.txt" 2>&1 || { tail -30 $OUT/pytest_v$V.txt; exit 1; }
  tail -n 1 $OUT/pytest_v$V.txt
done
: > "$OUT/ab.jsonl"
for cfg in '{"kind": "wd", "d": 4, "n": 9000, "reps": 3, "steps": 10}' \
           '{"kind": "wd", "d": 5, "n": 9000, "reps": 3, "steps": 10}' \
           '{"kind": "wd", "d": 10, "n": 9000, "reps": 3, "steps": 10}' \
           '{"kind": "wd", "d": 5, "n": 20000, "reps": 3, "steps": 5}'; do
  timeout -k 10 200 python3 -u tools/ab_env.py "$cfg" '[{}, {"KMG_WD_VAR": 2}, {"KMG_WD_VAR": 4}]' >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -20 $OUT/ab.err; exit 1; }
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(json.dumps(r["cfg"]), json.dumps(r["env"]))].append(r["gram_ms"])
for k, v in d.items(): print(k[0][:40], k[1], "min %.4f med %.4f" % (min(v), sorted(v)[len(v)//2]))
PY
