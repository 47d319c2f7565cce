#!/bin/bash
# Run one gpurun call, waiting for a box: retries ONLY while gpurun reports a
# transient acquisition failure with nothing charged (no part of the command
# ran); any call that ran -- success or failure -- is never repeated.
# usage: tools/gpurun_wait.sh <log> <timeout> '<command>'
log=$1; to=$2; shift 2
for attempt in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && grep -q "charged=0.0s\|charged=Nones" "$log"; then
    echo "[wait] attempt $attempt: transient, retrying in 90 s" >> "$log.attempts"
    sleep 90
    continue
  fi
  if [ $rc -eq 3 ]; then
    echo "[wait] attempt $attempt: no box (rc 3), retrying in 90 s" >> "$log.attempts"
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
