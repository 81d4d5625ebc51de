#!/bin/bash
# Submit a gpurun call; resubmit only when the box could not be prepared
# (status "transient": nothing ran, nothing charged), at most 3 times.
for i in 1 2 3; do
  /usr/local/graft/bin/gpurun --timeout "$1" -- "$2" > /tmp/gpurun_last.log 2>&1
  tail -2 /tmp/gpurun_last.log
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  [ "$st" = "transient" ] || exit 0
  sleep 60
done
