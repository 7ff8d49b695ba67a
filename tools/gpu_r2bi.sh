#!/bin/bash
# Dense Gram: where the time goes (EXPERIMENT store modes: 0 non-temporal, 1 plain, 2 none).
set -u
OUT=gpurun_out/r2bi
mkdir -p "$OUT"
export TMPDIR=/tmp
: > "$OUT/ab.jsonl"
for cfg in '{"kind": "sp", "k": 5, "n": 20000, "reps": 3, "steps": 10}' \
           '{"kind": "mm", "k": 6, "n": 20000, "norm": 0, "reps": 3, "steps": 10, "seed": 3}' \
           '{"kind": "mm", "k": 5, "n": 9000, "norm": 1, "reps": 3, "steps": 10, "seed": 3}'; do
  timeout -k 10 200 python3 -u tools/ab_env.py "$cfg" '[{"KMG_ALGO": 1}, {"KMG_ALGO": 1, "KMG_DENSE_HALF": 1}, {"KMG_ALGO": 1, "KMG_DENSE_STORE": 1}, {"KMG_ALGO": 1, "KMG_DENSE_HALF": 1, "KMG_DENSE_STORE": 1}, {"KMG_ALGO": 1, "KMG_DENSE_STORE": 2}, {"KMG_ALGO": 1, "KMG_DENSE_HALF": 1, "KMG_DENSE_STORE": 2}]' >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -20 $OUT/ab.err; exit 1; }
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(json.dumps(r["cfg"]), json.dumps(r["env"]))].append(r["gram_ms"])
for k, v in d.items(): print(k[0][:40], k[1], "min %.4f med %.4f" % (min(v), sorted(v)[len(v)//2]))
PY
