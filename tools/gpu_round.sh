#!/bin/bash
# GPU-box runner: each GPU step under its own time limit; stop at the first fault/abort/timeout.
# Usage: bash tools/gpu_round.sh "<step1>" "<step2>" ...   (steps run in order; rc 0/1 continue)
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i+1))
  echo "=== step $i: $step" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  bash -c "$step"
  rc=$?
  echo "=== step $i rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
