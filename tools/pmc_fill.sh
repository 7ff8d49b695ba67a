#!/bin/bash
# PMC passes over the neighbourhood-list fill kernel, one run per counter set and fill form
# (GPU box).  Counters missing from `rocprofv3 -L` are dropped from their set first.
# usage: tools/pmc_fill.sh <tag> [form ...]
set -u
TAG=$1; shift
FORMS=${*:-0}
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || { echo "counter list failed"; exit 1; }
have() { local b=${1%_sum}; b=${b%_avr}; grep -qw "$b" "$OUT/counters.txt"; }
pick() { local r=""; for c in $1; do have "$c" && r="$r $c"; done; echo $r; }
SETS=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR"
      "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES TA_BUSY_avr TA_FLAT_WRITE_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum"
      "TD_BUSY_avr TD_TD_BUSY_sum TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum"
      "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAVES")
for F in $FORMS; do
  CASES='[{"kind":"mm","k":9,"n":20000,"steps":3,"check":false,"KMG_NB_FILL":"'$F'"}]'
  i=0
  for S in "${SETS[@]}"; do
    i=$((i+1))
    CTRS=$(pick "$S")
    echo "form $F set $i: $CTRS" >> "$OUT/sets.txt"
    [ -z "$CTRS" ] && continue
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/f$F/p$i" -o run \
      -- python3 tools/time_mm.py "$CASES" > "$OUT/f$F.p$i.log" 2>&1 || { echo "form $F pass $i failed"; tail -5 "$OUT/f$F.p$i.log"; exit 1; }
  done
  python3 tools/pmc_report.py "$OUT/f$F" nb_fill > "$OUT/f$F.report.txt"
  echo "== form $F"; cat "$OUT/f$F.report.txt"
done
echo pmc fill done
