#!/bin/bash
# One parametrised GPU-box session (replaces the per-session gpu_r*.sh scripts).
# Every step runs under its own time limit; the session stops at the first failing step.
#
# usage: bash tools/gpu_run.sh <tag> <step> [<step> ...]
#   tests[=EXPR]            GPU test suite (tools/gpu_tests.sh; EXPR: pytest -k expression),
#                           log gpurun_out/<tag>/pytest.txt
#   smoke                   __graft_entry__.smoke()
#   bench[:ARGS]            python bench.py ARGS (colon-separated, e.g. bench:--steps:10)
#   benchprof[:ARGS]        the same under rocprofv3 --kernel-trace --stats
#   prof:WL[,WL...]         rocprofv3 kernel trace + PMC passes (profiles/run_profiles_r02.sh)
#   ab:<cfg json>@@<sets json>   interleaved A/B of KMG_* settings (tools/ab_env.py)
#   time:<cases json>       device-resident build timing (tools/time_mm.py)
# Steps with spaces or JSON must be quoted as one shell word.
set -u
TAG=${1:?tag}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for STEP in "$@"; do
  n=$((n + 1))
  case "$STEP" in
    tests*)
      if [ "$STEP" = "tests" ]; then
        bash tools/gpu_tests.sh "$TAG" > /dev/null || { echo "tests failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
      else
        bash tools/gpu_tests.sh "$TAG" -k "${STEP#tests=}" > /dev/null || { echo "tests failed"; tail -40 "$OUT/pytest.txt"; exit 1; }
      fi
      tail -n 1 "$OUT/pytest.txt"
      ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > "$OUT/smoke.txt" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.txt"; exit 1; }
      tail -n 1 "$OUT/smoke.txt"
      ;;
    benchprof*)
      # bench.py itself under rocprofv3 --kernel-trace --stats (the roofline's kernel average
      # must agree with the rocprof average of the same command)
      ARGS=${STEP#benchprof}
      ARGS=${ARGS#:}
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_trace" -o run \
        -- python3 -u bench.py ${ARGS//:/ } > "$OUT/benchprof$n.json" 2> "$OUT/benchprof$n.err" \
        || { echo "benchprof failed"; tail -30 "$OUT/benchprof$n.err"; exit 1; }
      cut -c1-400 "$OUT/benchprof$n.json"
      grep -m1 gram_sp_kernel "$OUT/bench_trace/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-160
      ;;
    bench*)
      ARGS=${STEP#bench}
      ARGS=${ARGS#:}
      timeout -k 10 600 python3 -u bench.py ${ARGS//:/ } > "$OUT/bench$n.json" 2> "$OUT/bench$n.err" \
        || { echo "bench failed"; tail -30 "$OUT/bench$n.err"; exit 1; }
      cut -c1-400 "$OUT/bench$n.json"
      ;;
    prof:*)
      WL=${STEP#prof:}
      bash profiles/run_profiles_r02.sh "$TAG" ${WL//,/ } > "$OUT/prof$n.log" 2>&1 \
        || { echo "prof failed"; tail -20 "$OUT/prof$n.log"; exit 1; }
      tail -40 "$OUT/prof$n.log"
      ;;
    ab:*)
      REST=${STEP#ab:}
      CFG=${REST%%@@*}
      SETS=${REST#*@@}
      timeout -k 10 600 python3 -u tools/ab_env.py "$CFG" "$SETS" > "$OUT/ab$n.jsonl" 2> "$OUT/ab$n.err" \
        || { echo "ab failed"; tail -20 "$OUT/ab$n.err"; exit 1; }
      cat "$OUT/ab$n.jsonl"
      ;;
    time:*)
      CASES=${STEP#time:}
      timeout -k 10 600 python3 -u tools/time_mm.py "$CASES" > "$OUT/time$n.jsonl" 2> "$OUT/time$n.err" \
        || { echo "time failed"; tail -20 "$OUT/time$n.err"; exit 1; }
      cat "$OUT/time$n.jsonl"
      ;;
    *)
      echo "unknown step $STEP"
      exit 2
      ;;
  esac
done
echo "session $TAG done"
