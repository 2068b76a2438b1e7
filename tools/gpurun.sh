#!/bin/bash
# Submit one gpurun call; resubmit only when the box could not be prepared (status=transient / rc 3),
# never when the command itself ran.
for attempt in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1)
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient\|no box or slot"; then
    sleep 60
    continue
  fi
  break
done
