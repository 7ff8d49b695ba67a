#!/bin/bash
# PMC passes of two tools/time_mm.py case lists in the same session (this tree), one
# rocprofv3 --pmc pass per counter set and case list.
# usage: tools/pmc_two.sh <tag> '<cases A>' '<cases B>' [kernel substring]
set -u
TAG=$1; CA=$2; CB=$3; KS=${4:-nb_}
OUT=gpurun_out/pmc2_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TD_BUSY_avr" "SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum"; do
  i=$((i+1))
  for side in A B; do
    if [ $side = A ]; then C=$CA; else C=$CB; fi
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/$side/p$i" -o run \
       -- python3 tools/time_mm.py "$C" > "$OUT/$side.p$i.log" 2>&1 || { echo "pass $i $side failed"; tail -5 "$OUT/$side.p$i.log"; exit 1; }
  done
done
for side in A B; do
  python3 tools/pmc_report.py "$OUT/$side" "$KS" > "$OUT/$side.report.txt"
  echo "== $side"; cat "$OUT/$side.report.txt"
done
