#!/bin/bash
# gpurun with retries while no box is free (exit 3: nothing ran, nothing charged); any other
# outcome — success, failure, refusal — ends it. Usage: scripts/gpurun_wait.sh <log> <timeout> <cmd>
log=$1; to=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && ! grep -q "status=transient" "$log" && break
  sleep 150
done
echo "gpurun rc=$rc" >> "$log"
