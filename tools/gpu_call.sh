#!/bin/bash
# gpurun wrapper: re-submits only when the harness reports a transient infrastructure status
# (box not prepared / no slot free; nothing ran, nothing charged).  A command that ran and failed
# is never re-submitted.   usage: tools/gpu_call.sh <timeout_s> '<command>'
t=$1; shift
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > /tmp/gpu_call.out 2>&1
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('/root/repo/gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then break; fi
  echo "[gpu_call] transient (attempt $attempt), waiting"
  sleep 100
done
tail -3 /tmp/gpu_call.out
exit $rc
