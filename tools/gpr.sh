#!/bin/bash
# retry a gpurun call only when the pool reports a transient (nothing ran, nothing charged)
CMD="$1"; OUTF="$2"; TO="${3:-900}"
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUTF" 2>&1
  if grep -q "status=transient" "$OUTF"; then sleep 60; continue; fi
  break
done
tail -4 "$OUTF"
