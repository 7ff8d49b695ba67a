#!/bin/bash
# Submit one gpurun call, waiting for a free slot.  It re-submits ONLY when nothing ran:
# gpurun exited 3 (no box / slot free), or its status line says that nothing was charged
# ("all ... GPU slot(s) on this pod are busy ...; nothing was charged").  Any other outcome,
# a failing or hung GPU step included, ends the wrapper with that exit code and leaves its
# log in place, so the fault is reported and its cause can be found from that evidence.
# usage: tools/gpurun_wait.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { [ $rc -ne 0 ] && grep -q "nothing was charged" "$LOG" &&
                         grep -q "run 0.0s" "$LOG"; }; then
    cat "$LOG" >> "$LOG.waits"
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
