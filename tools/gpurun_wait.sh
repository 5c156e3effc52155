#!/bin/bash
# Container-side helper: submit one gpurun call, re-submitting ONLY while the pool reports
# that no box / slot is free or access is backing off (nothing ran, nothing charged).  Any
# call that actually ran -- pass or fail -- ends the helper; its output is in the log.
# Usage: tools/gpurun_wait.sh <log> <timeout-seconds> '<command>'
LOG=${1:?log}; TO=${2:?timeout}; CMD=${3:?command}
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG"; then
    w=$(grep -o "retry in [0-9]*s" "$LOG" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-120} + 15 ))
    continue
  fi
  exit $rc
done
exit 3
