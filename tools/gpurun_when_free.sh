#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while gpurun answers "no slot free" (exit 3: nothing ran, nothing
# charged).  Any other outcome (success, failure, timeout, refusal) is final.  Usage:
#   tools/gpurun_when_free.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for attempt in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "GPU slot(s) on this pod are busy\|backing off" "$LOG"; then
    echo "gpurun rc=$rc (attempt $attempt)" >> "$LOG"
    exit $rc
  fi
  sleep 200
done
echo "gave up after 20 busy answers" >> "$LOG"
exit 3
