#!/bin/bash
# PMC passes for the dense int8-MFMA Gram (gram_dense_kernel) over tools/time_mm.py cases
# (GPU box), one counter set per rocprofv3 run.  usage: tools/pmc_dense.sh <tag> '<time_mm json>'
set -u
TAG=$1; CASES=$2
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for CTRS in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/p$i" -o run \
     -- python3 tools/time_mm.py "$CASES" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 tools/pmc_report.py "$OUT" gram_dense > "$OUT/report.txt"
cat "$OUT/report.txt"
