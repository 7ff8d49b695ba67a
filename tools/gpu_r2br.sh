#!/bin/bash
# Substring kernel: "up" values by DPP wave_shr vs __shfl_up (KMG_SS_SHFL=1): parity with the
# DPP form, then an interleaved one-process A/B.
set -u
OUT=gpurun_out/r2br
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "ss or golden" --timeout 120 --timeout-method thread > "$OUT/pytest.txt" 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -n 1 $OUT/pytest.txt
: > "$OUT/ab.jsonl"
for cfg in '{"kind": "ss", "k": 5, "n": 1000, "reps": 3, "steps": 2}' \
           '{"kind": "ss", "k": 12, "n": 1000, "reps": 3, "steps": 2}'; do
  timeout -k 10 200 python3 -u tools/ab_env.py "$cfg" '[{"KMG_SS_SHFL": 1}, {}]' >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "ab failed"; tail -20 $OUT/ab.err; exit 1; }
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(sys.argv[1]):
    r = json.loads(l); d[(json.dumps(r["cfg"]), json.dumps(r["env"]))].append(r["gram_ms"])
for k, v in d.items(): print(k[0][:40], k[1], "min %.4f med %.4f" % (min(v), sorted(v)[len(v)//2]))
PY
