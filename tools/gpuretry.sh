#!/bin/bash
# retry a gpurun call while the pool has no free slot / box (nothing ran, nothing charged); stop on any real result
LOG=$1; shift
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG"; then sleep 90; continue; fi
  break
done
