#!/bin/bash
# Submit one gpurun call; resubmit only when the box could not be prepared (status "transient",
# or exit code 3 = no box free), never when the command itself ran.
for attempt in 1 2 3 4 5; do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun "$@" > /tmp/gpurun_last.log 2>&1
  rc=$?
  tail -3 /tmp/gpurun_last.log
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" = "transient" ] || [ $rc -eq 3 ]; then
    echo "[gpurun.sh] transient ($st, rc=$rc), retrying in 60s"
    sleep 60
    continue
  fi
  exit $rc
done
