#!/bin/bash
# GPU-box runner: each GPU step under its own time limit; stop at the first fault/abort/timeout.
# Usage: bash tools/steps.sh "<step1>" "<step2>" ...
# A step may fail with rc 1 (pytest test failures, python assertion) and the next step still runs,
# unless its output shows a GPU fault; any other nonzero rc (timeout 124/137, abort 134, segv 139)
# ends the call.
mkdir -p gpurun_out/keep
i=0
for step in "$@"; do
  i=$((i+1))
  echo "=== step $i: $step" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  bash -c "$step"
  rc=$?
  echo "=== step $i rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/steps.log
  if grep -l -E "IllegalAddress|Memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|GPU Hang" gpurun_out/*.log >/dev/null 2>&1; then
    echo "stopping: GPU fault reported" | tee -a gpurun_out/steps.log
    exit 99
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
