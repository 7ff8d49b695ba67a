#!/bin/bash
# A/B of two builds of the library (KMGRAM_LIB) on one case file: alternating processes,
# one JSON line each, into $3.  Usage: tools/ab_lib.sh <libA> <libB> <out> <cases.json> [reps]
set -e
A=$1; B=$2; OUT=$3; CASES=$4; REPS=${5:-4}
: > "$OUT"
for i in $(seq "$REPS"); do
  for L in "$A" "$B"; do
    KMGRAM_LIB="$L" timeout -k 10 120 python -u tools/time_mm.py "$(cat "$CASES")" | sed "s|^|{\"lib\": \"$(basename "$L")\", \"r\": |; s|$|}|" >> "$OUT"
  done
done
