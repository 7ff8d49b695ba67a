#!/bin/bash
# Same-box PMC A/B of a tools/time_mm.py case between the round-4 package copy (tools/ab/r04)
# and this tree, one rocprofv3 --pmc pass per counter set and side.
# usage: tools/ab_pmc.sh <tag> '<time_mm cases json>' [kernel substring]
set -u
TAG=$1; CASES=$2; KS=${3:-gram_nb}
OUT=gpurun_out/abpmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr"; do
  i=$((i+1))
  for side in r04 new; do
    if [ $side = r04 ]; then S=tools/ab/r04/tools/time_mm.py; else S=tools/time_mm.py; fi
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/$side/p$i" -o run \
       -- python3 $S "$CASES" > "$OUT/$side.p$i.log" 2>&1 || { echo "pass $i $side failed"; tail -5 "$OUT/$side.p$i.log"; exit 1; }
  done
done
for side in r04 new; do
  python3 tools/pmc_report.py "$OUT/$side" "$KS" > "$OUT/$side.report.txt"
  echo "== $side"; cat "$OUT/$side.report.txt"
done
