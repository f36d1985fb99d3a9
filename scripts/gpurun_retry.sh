#!/bin/bash
# Submit one GPU session through gpurun, re-submitting ONLY when gpurun reports a transient
# condition (no slot / box not ready: nothing ran, nothing charged).  Any run that started --
# pass, fail or fault -- is never repeated here.
# usage: scripts/gpurun_retry.sh <timeout_s> <session script> <log>
to=$1; script=$2; log=$3
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- bash "$script" > "$log" 2>&1
  if grep -q "status=transient" "$log"; then
    echo "[retry $i] transient, waiting" >> "$log.retries"
    sleep 150
    continue
  fi
  break
done
