#!/bin/bash
# gpurun with retry on "transient" (box never ran the command) outcomes only.
# usage: tools/gpr.sh <timeout_s> '<command>'
t=$1; shift
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1 | tail -3
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit 0; fi
  echo "[gpr] transient, retry $attempt"; sleep 60
done
