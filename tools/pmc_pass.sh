#!/bin/bash
# PMC passes for one tune.py workload (GPU box).  usage: tools/pmc_pass.sh <tag> <sp|mm> '<sets json>'
set -u
TAG=$1; WL=$2; SETS=$3
OUT=gpurun_out/pmc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for CTRS in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/p$i" -o run \
     -- python3 tools/tune.py $WL --reps 1 --sets "$SETS" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo pmc done
