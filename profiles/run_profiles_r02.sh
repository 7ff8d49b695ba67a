#!/bin/bash
# Round-2 rocprofv3 evidence beside the bench (run from the repo root on the GPU box):
#   per workload: one --kernel-trace --stats pass, then one run per PMC counter set
#   (FETCH_SIZE and WRITE_SIZE in their own passes; SQ sets apart from TCC).
# Workloads are tools/time_mm.py cases (device-resident builds, the same launches bench.py
# times).  Usage: bash profiles/run_profiles_r02.sh <tag> [workload ...]
set -u
TAG=${1:-r02}; shift
WL=${*:-config4 dense_sp5 wd_n9000}
export TMPDIR=/tmp
case_of() {
  case $1 in
    config4)   echo '[{"kind":"sp","k":8,"n":100000,"steps":10}]' ;;
    sp_n20000) echo '[{"kind":"sp","k":8,"n":20000,"steps":10}]' ;;
    dense_sp5) echo '[{"kind":"sp","k":5,"n":20000,"steps":10}]' ;;
    mm_n20000) echo '[{"kind":"mm","k":9,"n":20000,"steps":5,"check":false}]' ;;
    mm1_n20000) echo '[{"kind":"mm","k":9,"n":20000,"steps":5,"check":false,"KMG_MM_FORM":"1"}]' ;;
    mm3_n20000) echo '[{"kind":"mm","k":9,"n":20000,"steps":5,"check":false,"KMG_MM_FORM":"3"}]' ;;
    wd_n9000)  echo '[{"kind":"wd","d":5,"n":9000,"steps":10,"check":false}]' ;;
    nb_n20000) echo '[{"kind":"mm","k":9,"n":20000,"steps":5,"check":false,"KMG_MM_FORM":"4","KMG_MM_CHUNK":"20000","KMG_MM_TRI":"0"}]' ;;
    nbf1) echo '[{"kind":"mm","k":9,"n":20000,"steps":3,"check":false,"KMG_MM_FORM":"4","KMG_MM_CHUNK":"20000","KMG_MM_TRI":"0","KMG_NB_FILL":"1"}]' ;;
    nbf3) echo '[{"kind":"mm","k":9,"n":20000,"steps":3,"check":false,"KMG_MM_FORM":"4","KMG_MM_CHUNK":"20000","KMG_MM_TRI":"0","KMG_NB_FILL":"3"}]' ;;
    config5_full) echo '[{"kind":"mm","k":9,"n":200000,"norm":0,"seed":5,"steps":2,"check":false}]' ;;
    config5_slab) echo '[{"kind":"mm","k":9,"n":200000,"rows":25000,"norm":1,"seed":5,"steps":3,"check":false}]' ;;
  esac
}
sets_of() {
  case $1 in
    dense_sp5) echo "FETCH_SIZE|WRITE_SIZE|SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES|GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    mm*|config5*|nb*) echo "FETCH_SIZE|WRITE_SIZE|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES|SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY|TCC_HIT_sum TCC_MISS_sum" ;;
    *)         echo "FETCH_SIZE|WRITE_SIZE|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES|TCC_HIT_sum TCC_MISS_sum" ;;
  esac
}
for W in $WL; do
  OUT=gpurun_out/prof_${TAG}_$W
  mkdir -p "$OUT"
  CASES=$(case_of "$W")
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 tools/time_mm.py "$CASES" > "$OUT/trace.log" 2>&1 || { echo "$W trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
  i=0
  IFS='|' read -ra SETS <<< "$(sets_of "$W")"
  for CTRS in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 180 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT/p$i" -o run \
      -- python3 tools/time_mm.py "$CASES" > "$OUT/p$i.log" 2>&1 || { echo "$W pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  done
  python3 tools/pmc_report.py "$OUT" > "$OUT/report.txt"
  echo "== $W"; grep -v "^$" "$OUT/trace.log" | tail -2; cat "$OUT/report.txt"
done
echo profiles done
