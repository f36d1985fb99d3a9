#!/bin/bash
# Submit one GPU session through gpurun, re-submitting ONLY when gpurun reports a transient
# condition (no slot / box not ready: nothing ran, nothing charged -- "status": "transient" in
# gpurun_out/.last_call.json).  Any run that started -- pass, fail or fault -- is never repeated.
# usage: scripts/gpurun_retry.sh <timeout_s> <session script> <log>
to=$1; script=$2; log=$3
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- bash "$script" > "$log" 2>&1
  if python3 -c 'import json,sys; sys.exit(0 if json.load(open("gpurun_out/.last_call.json")).get("status") == "transient" else 1)'; then
    echo "[retry $i] transient, waiting" >> "$log.retries"
    sleep 120
    continue
  fi
  break
done
