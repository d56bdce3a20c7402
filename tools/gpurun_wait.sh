#!/bin/bash
# Run one gpurun call, waiting for a free GPU slot: retries ONLY while gpurun answers 3 or reports a
# transient status (no box or slot free right now, nothing ran); any other exit (a failed GPU step) ends it.
#   tools/gpurun_wait.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  # 3: no box or slot free; a "transient" status (all slots busy) likewise ran nothing
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$LOG"; then exit $rc; fi
  sleep 150
done
exit 3
