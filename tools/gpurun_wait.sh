#!/bin/bash
# Submit one gpurun call, waiting for a free slot: re-submits ONLY while gpurun reports
# that no box / slot was free (exit 3: nothing ran, nothing charged).  Any other outcome
# (including a failing GPU step) ends the wrapper with that exit code.
# usage: tools/gpurun_wait.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
  sleep 90
done
exit 3
