#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) over tools/time_mm.py cases (GPU box).
# usage: tools/pmc_cmd.sh <tag> '<time_mm json>'
set -u
TAG=$1; CASES=$2
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/p$i" -o run \
     -- python3 tools/time_mm.py "$CASES" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_report.py "$OUT" "${KSUB:-gram_mm}" > "$OUT/report.txt"
cat "$OUT/report.txt"
